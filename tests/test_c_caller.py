"""A C99 translation unit against include/gnark_amd.h, as cgo compiles the
header (tests/c_caller/cubic_prove.c; round-4 VERDICT Weak 8).

CPU: the header and the caller compile with `gcc -std=c99 -pedantic -Werror`
and link against libgnark_amd.so (every symbol the caller uses resolves).
GPU: the C program uploads the golden cubic key (examples/cubic, BN254) with
gg_groth16_pk_create, proves twice with gg_groth16_prove from host buffers and
prints Ar / Bs / Krs, which must equal the golden proof
(tests/golden/golden.json, the proof of groth16_test.go:70-88's circuit with
injected r, s; the same values test_gpu_groth16.py checks through ctypes)."""
import os
import shutil
import subprocess

import pytest

from helpers import b, golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c_caller", "cubic_prove.c")
LIBDIR = os.path.join(ROOT, "gnark-fork_amd", "lib")


def _build(tmp_path):
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    exe = str(tmp_path / "cubic_prove")
    cmd = ["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
           "-o", exe, SRC, "-L", LIBDIR, "-lgnark_amd", "-Wl,-rpath," + LIBDIR]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_c_caller_compiles_and_links(tmp_path):
    """the cgo-shaped caller builds as C99 against the header and the library"""
    _build(tmp_path)


def _input(g):
    from gnark_amd import fr
    omega = fr.fr_mont(fr.domain_generator(g["log_n"]))
    gen = fr.fr_mont(fr.FR_MULTIPLICATIVE_GEN)
    lines = [f"log_n {g['log_n']}", f"nb_public {g['nb_public']}", f"omega {bytes(omega).hex()}",
             f"coset_gen {bytes(gen).hex()}"]
    for k in ("g1_A", "g1_B", "g1_Z", "g1_K", "alpha1", "beta1", "delta1", "g2_B", "beta2", "delta2", "wires",
              "solA", "solB", "solC", "r", "s"):
        lines.append(f"{k} {g[k]}")
    lines.append(f"infA {g['infA']}")
    lines.append(f"infB {g['infB']}")
    return "\n".join(lines) + "\n"


@pytest.mark.gpu
@pytest.mark.parametrize("idx", [0, 1])
def test_c_caller_golden_proof(tmp_path, idx):
    g = golden()["groth16"][idx]
    exe = _build(tmp_path)
    r = subprocess.run([exe], input=_input(g), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    out = dict(line.split(" ", 1) for line in r.stdout.strip().splitlines())
    assert out["Ar"] == g["Ar"]
    assert out["Bs"] == g["Bs"]
    assert out["Krs"] == g["Krs"]
    assert len(b(out["Ar"])) == 64
