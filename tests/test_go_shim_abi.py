"""The cgo shims under go/ cannot be compiled here (no Go toolchain), so this
test checks their calls into the C ABI the way cgo would: every `C.gg_*(...)`
call expression in go/**/*.go must name a function declared in
include/gnark_amd.h (or in the file's own cgo preamble), pass exactly as many
arguments as the prototype has parameters, and pass each argument with a kind
that cgo would accept for that parameter (C.int / C.size_t for integers,
unsafe.Pointer / typed pointers / &x / nil for pointers, the handle conversion
for opaque handles).  References: groth16.go:170 / plonk.go:128 dispatch
(INTEGRATION.md), icicle.go:133-422 (the call sites these shims replace)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gnark_amd.h")
GO_DIR = os.path.join(ROOT, "go")


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _split_top(args):
    out, depth, cur = [], 0, ""
    for ch in args:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _prototypes(text):
    """name -> list of parameter kinds ('int', 'ptr', 'handle:<type>', 'fn')."""
    text = _strip_c_comments(text)
    typedef_handles = set(re.findall(r"typedef\s+struct\s+\w+\s*\*\s*(\w+)\s*;", text))
    typedef_fns = set(re.findall(r"typedef\s+[\w\s\*]+\(\s*\*\s*(\w+)\s*\)", text))
    protos = {}
    for m in re.finditer(r"\b(?:int|size_t|void|double|const\s+char|gg_\w+)\s*\**\s*(gg_\w+)\s*\(([^;{)]*)\)\s*[;{]",
                         text, re.S):
        name, params = m.group(1), m.group(2).strip()
        if params in ("", "void"):
            protos[name] = []
            continue
        kinds = []
        for p in _split_top(params):
            p = " ".join(p.split())
            base = re.sub(r"\b(const|volatile)\b", "", p).strip()
            toks = base.replace("*", " * ").split()
            if "*" in toks:
                kinds.append("ptr")
            elif toks and toks[0] in typedef_handles:
                kinds.append("handle:" + toks[0])
            elif toks and toks[0] in typedef_fns:
                kinds.append("fn")
            else:
                kinds.append("int")
        protos[name] = kinds
    return protos


def _go_calls(src):
    """(name, [args], line) for every C.gg_* call expression."""
    calls = []
    for m in re.finditer(r"\bC\.(gg_\w+)\s*\(", src):
        name = m.group(1)
        i, depth = m.end(), 1
        while depth and i < len(src):
            if src[i] == "(":
                depth += 1
            elif src[i] == ")":
                depth -= 1
            i += 1
        body = src[m.end():i - 1]
        calls.append((name, _split_top(body) if body.strip() else [], src.count("\n", 0, m.start()) + 1))
    return calls


def _arg_kind(a):
    a = a.strip()
    if a == "nil" or a.startswith("unsafe.Pointer(") or a.startswith("&") or a.startswith("(*C.") \
            or a.startswith("(*unsafe.Pointer)(") or re.match(r"^p\(", a) or a.startswith("ptrOr("):
        return "ptr"
    m = re.match(r"^\w+\.\(C\.(gg_\w+_t)\)$", a)  # type assertion on an interface holding a handle
    if m:
        return "handle:" + m.group(1)
    if re.match(r"^C\.(int|size_t|uint32_t|uint64_t|int64_t|uint8_t|double)\(", a) or re.match(r"^C\.GG_\w+$", a) \
            or re.match(r"^-?\d+$", a):
        return "int"
    m = re.match(r"^C\.(gg_\w+_t)\(", a)
    if m:
        return "handle:" + m.group(1)
    if re.match(r"^C\.gg_\w+_fn\(\)$", a) or re.match(r"^C\.gg_go_\w+\(\)$", a):
        return "fn"
    return "var:" + a  # a Go variable: kind resolved from its declaration


def _go_files():
    out = []
    for d, _, fs in os.walk(GO_DIR):
        out += [os.path.join(d, f) for f in fs if f.endswith(".go")]
    return sorted(out)


def test_go_shims_exist():
    assert _go_files(), "no Go shims under go/"


@pytest.mark.parametrize("path", _go_files(), ids=lambda p: os.path.relpath(p, GO_DIR))
def test_cgo_calls_match_header(path):
    protos = _prototypes(open(HEADER).read())
    src = open(path).read()
    # the file's cgo preamble (the comment block before import "C") may add helpers
    pre = re.search(r"/\*(.*?)\*/\s*import\s+\"C\"", src, re.S)
    local = _prototypes(pre.group(1)) if pre else {}
    # Go-side variable kinds: `var h C.gg_x_t`, `h := ...C.gg_x_t(...)`, `rc C.int`
    var_kind = {}
    for m in re.finditer(r"\bvar\s+(\w+)\s+C\.(gg_\w+_t)\b", src):
        var_kind[m.group(1)] = "handle:" + m.group(2)
    for m in re.finditer(r"\b(\w+)\s*,\s*err\s*:=\s*pk\.amdKey\(\)", src):
        var_kind[m.group(1)] = "handle:gg_plonk_pk_t"
    for m in re.finditer(r"func\s+\([^)]*\)\s*amdKey\(\)\s*\(C\.(gg_\w+_t)", src):
        var_kind.setdefault("h", "handle:" + m.group(1))
    calls = [c for c in _go_calls(src) if not c[0].endswith("_t")]  # C.gg_x_t(...) is a conversion
    assert calls or "noamd" in path or "provingkey" in path, f"{path}: no C ABI calls found"
    for name, args, line in calls:
        where = f"{os.path.relpath(path, ROOT)}:{line} C.{name}"
        kinds = protos.get(name, local.get(name))
        assert kinds is not None, f"{where}: not declared in include/gnark_amd.h or the cgo preamble"
        assert len(args) == len(kinds), f"{where}: {len(args)} arguments, prototype has {len(kinds)}"
        for j, (a, want) in enumerate(zip(args, kinds)):
            got = _arg_kind(a)
            if got.startswith("var:"):
                got = var_kind.get(got[4:], "unknown")
            if got == "unknown":
                continue  # a plain Go value of a type declared elsewhere: cgo checks it at build time
            if want.startswith("handle:"):
                ok = got == want or got == "ptr"
            elif want == "fn":
                ok = got in ("fn", "ptr")
            else:
                ok = got == want
            assert ok, f"{where}: argument {j + 1} `{a}` is {got}, parameter is {want}"


def test_shim_symbols_exported():
    """Every ABI function the shims call is exported by the built library."""
    lib = os.path.join(ROOT, "gnark-fork_amd", "lib", "libgnark_amd.so")
    if not os.path.exists(lib):
        pytest.skip("library not built")
    import ctypes
    h = ctypes.CDLL(lib)
    protos = _prototypes(open(HEADER).read())
    missing = []
    for path in _go_files():
        for name, _, _ in _go_calls(open(path).read()):
            if name.endswith("_t") or name not in protos:
                continue
            if not hasattr(h, name):
                missing.append(name)
    assert not missing, f"called by go/ but not exported: {sorted(set(missing))}"
