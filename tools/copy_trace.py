"""Kernel + copy timeline of tools/mbench_xqueue2 under rocprofv3
--kernel-trace --memory-copy-trace (rocpd sqlite): for every long k_busy
dispatch (the MSM-shaped kernel), the copies (blit kernels
__amd_rocclr_copyBuffer* and SDMA memory copies) that start while it runs or
right after it, with their start / end relative to the kernel's start and
whether they finished before the kernel did -- the round-4 VERDICT's "copy
completes while the kernel is still running, in a kernel + copy trace".
usage: copy_trace.py run_results.db [min_kernel_ms]"""
import sqlite3
import sys


def main(argv):
    db = argv[0]
    min_ms = float(argv[1]) if len(argv) > 1 else 3.0
    con = sqlite3.connect(db)
    ks = con.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
    copies = [(n, s, e, st, q, "blit") for n, s, e, st, q in ks if "rocclr_copy" in n]
    try:
        for s, e, st, q, size, name in con.execute(
                "select start, end, stream_id, queue_id, size, name from memory_copies order by start"):
            copies.append((f"{name} {size / 1e6:.0f} MB", s, e, st, q, "sdma"))
    except sqlite3.Error:
        pass
    copies.sort(key=lambda c: c[1])
    busy = [k for k in ks if "k_busy" in k[0] and (k[2] - k[1]) * 1e-6 >= min_ms]
    print(f"{len(busy)} k_busy dispatches >= {min_ms} ms; times in ms from each kernel's start")
    for name, s, e, st, q in busy:
        dur = (e - s) * 1e-6
        near = [c for c in copies if s - 0.2e6 <= c[1] <= e + 0.5e6]
        print(f"k_busy stream {st} queue {q}: 0.000 .. {dur:.3f}")
        for cn, cs, ce, cst, cq, kind in near:
            done_in = ce < e
            print(f"    {kind:4s} {cn[:48]:48s} stream {cst} queue {cq}: {(cs - s) * 1e-6:8.3f} .. {(ce - s) * 1e-6:8.3f}"
                  f"  {'finished while the kernel ran' if done_in else 'finished after the kernel'}")


if __name__ == "__main__":
    main(sys.argv[1:])
