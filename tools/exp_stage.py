"""Experiment: host-input staging of the 2^24 Groth16 prove under knobs
(GG_STAGE_NT, GG_STAGE_STREAMS; run under several GPU_MAX_HW_QUEUES).  usage: exp_stage.py [log_n]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    import torch
    from gnark_amd import _lib
    _lib.check(_lib.lib.gg_set_device(0))
    torch.cuda.set_device(0)
    settings = [dict(), dict(GG_STAGE_STREAMS="8"), dict(GG_STAGE_NT="16"), dict(GG_STAGE_NT="4")]
    print("GPU_MAX_HW_QUEUES =", os.environ.get("GPU_MAX_HW_QUEUES"), flush=True)
    for st in settings:
        # the stager reads its knobs at creation: a fresh key per setting
        for k in ("GG_STAGE_NT", "GG_STAGE_STREAMS", "GG_G16_SERIAL"):
            os.environ.pop(k, None)
        os.environ.update(st)
        g = bench.Groth16Bench(log_n, 0, 1, None, None, host_inputs=True)
        g.prove()
        ts = []
        for _ in range(4):
            t = time.perf_counter()
            g.prove()
            ts.append(1e3 * (time.perf_counter() - t))
        tm = g.timings()
        print(st, "prove_ms %.1f" % min(ts), {k: round(v, 1) for k, v in tm.items()}, flush=True)
        if not st:
            v = g.variants()
            print("  variants", {k: (round(x, 1) if isinstance(x, float) else x) for k, x in v.items()
                                 if not isinstance(x, dict)}, flush=True)
            print("  device-inputs stages", {k: round(x, 1) for k, x in v["device_inputs_stage_ms"].items()})
        g.close()
        del g


if __name__ == "__main__":
    main()
