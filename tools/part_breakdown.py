"""Where one rehearsed PlonK part spends its proof: from a rocprofv3
--kernel-trace database of tools/plonk_part_probe.py (PROBE_PARTS=<one part>),
take the last proof (dispatches after the last GPU-idle gap > gap_ms), and report
its wall span, the GPU-busy time (union of kernel intervals over all streams),
the idle gaps, and busy time per kernel family.
usage: part_breakdown.py run_results.db [gap_ms (default 10)] [title]"""
import re
import sqlite3
import sys
from collections import defaultdict

FAMILIES = [
    ("MSM accumulation", r"k_accum_range"),
    ("MSM sort", r"k_digits_hist|k_bin_scatter|k_bin_starts|k_seg_|k_scan_|k_set_total"),
    ("MSM level 2 + reduction", r"k_bucket|k_reduce_block|k_gather_items|k_normalize|k_comb"),
    ("NTT", r"k_ntt|k_stage_twiddles|k_bitrev|bit_reverse"),
    ("copies / fills", r"__amd_rocclr"),
]


def family(name):
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return "PlonK polynomial kernels (numerator, ratio, fold, Horner, ...)"


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(db, gap_ms=10.0, title="PlonK part"):
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    # the last proof: dispatches after the last GPU-idle gap > gap_ms (the probe
    # sleeps 30 ms between proofs)
    i0, run_end = 0, rows[0][2]
    for i in range(1, len(rows)):
        if rows[i][1] - run_end > gap_ms * 1e6:
            i0 = i
        run_end = max(run_end, rows[i][2])
    last = rows[i0:]
    t0, t1 = last[0][1], max(r[2] for r in last)
    busy = union_len([(s, e) for _, s, e in last])
    fam = defaultdict(list)
    for n, s, e in last:
        fam[family(n)].append((s, e))
    print(f"# {title}\n")
    print(f"source: `{db}`, the last proof ({len(last)} dispatches after a GPU-idle gap > {gap_ms} ms)\n")
    print(f"- wall span of its kernels: {(t1 - t0) / 1e6:.2f} ms")
    print(f"- GPU busy (union over streams): {busy / 1e6:.2f} ms; idle inside the span: {(t1 - t0 - busy) / 1e6:.2f} ms\n")
    print("| kernel family | dispatches | busy ms (union) | sum of durations ms |")
    print("|---|---|---|---|")
    for f, iv in sorted(fam.items(), key=lambda kv: -union_len(kv[1])):
        print(f"| {f} | {len(iv)} | {union_len(iv) / 1e6:.2f} | {sum(e - s for s, e in iv) / 1e6:.2f} |")
    # per kernel (template arguments dropped), the largest first
    per = defaultdict(list)
    for n, s, e in last:
        per[re.sub(r"\(.*", "", n)].append(e - s)
    print("\n| kernel | dispatches | sum ms | avg us |")
    print("|---|---|---|---|")
    for k, ds in sorted(per.items(), key=lambda kv: -sum(kv[1]))[:40]:
        print(f"| `{k[:90]}` | {len(ds)} | {sum(ds) / 1e6:.3f} | {sum(ds) / len(ds) / 1e3:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 10.0,
         sys.argv[3] if len(sys.argv) > 3 else "PlonK part")
