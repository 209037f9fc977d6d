#!/usr/bin/env python3
"""Benchmark of the MI355X Groth16/BN254 hot path.

Headline (BASELINE.json metric "... MSM G1 throughput (Mscalar-mul/s) ...",
workload = configs[1]): BN254 G1 MSM over 2^20 resident points per GPU, scalars
resident in HBM, one process per GPU.  A "step" is one full MSM (digits, sort,
bucket accumulation, bucket reduction, result to host); for N > 1 each rank owns
its own 2^20-point shard (weak scaling) and the per-rank Jacobian partials are
all-gathered over RCCL and added on rank 0 (RCCL has no EC-add reduction).

Also reported (not the headline): a Groth16 prove at --groth16-log-n with a
synthetic key generated on the GPU, and the C restatement (oracle/) of the same
MSM timed on the host cores as cpu_baseline.
"""
import argparse
import datetime
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gnark-fork_amd"))

METRIC = ("Groth16 prove time + MSM G1 throughput (Mscalar-mul/s) BN254 2^24 R1CS, 1/2/4/8 GPU")
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FPMUL_PEAK_G = 135.7  # measured BN254 Fp Montgomery multiplies/s (G), profiles/r01_v2_mbench_field.txt


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def rand_scalars(n, seed):
    """n random fr elements (Montgomery bytes) < 2^253 < r as uint64[n, 4]."""
    import numpy as np
    rng = np.random.default_rng(seed)
    raw = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64) * 2
    raw ^= rng.integers(0, 2, size=(n, 4), dtype=np.uint64)
    raw[:, 3] &= np.uint64((1 << 61) - 1)
    return np.ascontiguousarray(raw)


def g1_generator_mont():
    from gnark_amd import fr
    return fr.fp_mont(1) + fr.fp_mont(2)


def g2_generator_mont():
    from gnark_amd import fr
    x0 = 10857046999023057135944570762232829481370756359578518086990519993285655852781
    x1 = 11559732032986387107991004021392285783925812861821192530917403151452391805634
    y0 = 8495653923123431417604973247489272438418190587263600148770280649306958101930
    y1 = 4082367875863433681332203403145435568316851327593401208105741076214120093531
    return b"".join(fr.fp_mont(v) for v in (x0, x1, y0, y1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=20, help="MSM points per GPU = 2^log_n")
    ap.add_argument("--groth16-log-n", type=int, default=24,
                    help="domain size of the extra Groth16 prove measurement (0 = skip)")
    ap.add_argument("--ntt-log-n", type=int, default=24,
                    help="size of the extra Fr NTT measurement, BASELINE configs[2] (0 = skip)")
    ap.add_argument("--plonk-log-n", type=int, default=22,
                    help="BLS12-381 PlonK hot-op measurement size, BASELINE configs[4] (0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--extras-timeout", type=float, default=480.0,
                    help="seconds allowed for the extra measurements after the headline; past it "
                         "the headline line is printed with the extras marked timed out and the "
                         "process exits (a stuck collective never swallows the headline)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 0))
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import gnark_amd
    from gnark_amd import _lib, msm, DeviceBuffer

    # one process per GPU over RCCL ("nccl").  GG_DIST_BACKEND=gloo is a rehearsal
    # mode only (ranks may share a GPU; partials travel through host memory).
    backend = os.environ.get("GG_DIST_BACKEND", "nccl")
    dev = local_rank % max(1, torch.cuda.device_count())
    _lib.check(_lib.lib.gg_set_device(dev))
    torch.cuda.set_device(dev)
    xdev = torch.device("cuda", dev) if backend == "nccl" else torch.device("cpu")
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev),
                                    timeout=datetime.timedelta(minutes=10))
        else:
            dist.init_process_group(backend, timeout=datetime.timedelta(minutes=10))

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        _lib.check(_lib.lib.gg_synchronize())

    n = 1 << args.log_n
    # ---- synthetic resident key shard (GPU fixed-base batch mul, distinct per rank)
    t0 = time.time()
    ks = rand_scalars(n, 1000 + rank)
    pts = DeviceBuffer(64 * n)
    msm.batch_scalar_mul(msm.G1, g1_generator_mont(), ks, n, out=pts)
    base = msm.MsmBase(msm.G1, pts.ptr, n, on_device=True)
    del pts
    npts, c, W = base.info()
    sc = rand_scalars(n, 2000 + rank)
    dsc = DeviceBuffer.from_host(sc.tobytes())
    log(f"[rank {rank}] key shard ready: n={npts} c={c} windows={W} ({time.time() - t0:.1f}s)")

    from gnark_amd import dist as gdist

    def step():
        j = base.msm_jac(dsc, n, on_device=True)
        if dist is None:
            return j
        # RCCL all-gather of the 96-B Jacobian partials + exact EC add (gnark_amd.dist)
        return gdist.allgather_partial(msm.G1, j, device=xdev)

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device=xdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    ms_per_step = 1e3 * el / args.steps
    value = world * n * args.steps / el / 1e6  # Mscalar-mul/s, whole job

    # ---- roofline of the dominant kernel (bucket accumulation), HIP events on its stream
    gnark_amd._lib.profile_enable(True)
    prof_steps = max(3, min(10, args.steps))
    for _ in range(prof_steps):
        base.msm_jac(dsc, n, on_device=True)
    kernels = {}
    for name in ("msm_sort", "msm_accum", "msm_accum2", "msm_reduce"):
        ms, cnt, units = gnark_amd._lib.profile_get(name)
        kernels[name] = {"avg_ms": ms / cnt if cnt else None, "launches": cnt}
    gnark_amd._lib.profile_enable(False)
    acc_ms = kernels["msm_accum"]["avg_ms"]
    alg_bytes = n * (64 + 32)  # N x (G1 affine 64 B + fr 32 B)
    achieved = alg_bytes / (acc_ms * 1e-3) / 1e9 if acc_ms else None
    traffic, traffic_note = pmc_traffic("k_accum_affine<gg::Fe<gg::FpCfg> >", args.log_n, c, W)
    roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                "traffic_note": traffic_note,
                "kernel": "k_accum_affine<Fp> (bucket accumulation)",
                "algorithmic_bytes_per_launch": alg_bytes, "kernel_avg_ms": acc_ms,
                "note": "EC MSM is VALU-integer bound (SURVEY 8d); HBM fraction reported as required"}

    # VALU view of the same kernel: 8M+2S Fp multiplies per mixed add, one add per
    # non-zero (window, scalar) entry, against the measured Fp-mul peak
    # (profiles/r01_v2_mbench_field.txt, product-scanning Montgomery on MI355X)
    if acc_ms:
        mul_rate = n * W * 10 / (acc_ms * 1e-3) / 1e9
        roofline["valu"] = {"achieved_Gfpmul_s": mul_rate, "peak_Gfpmul_s": FPMUL_PEAK_G,
                            "frac": mul_rate / FPMUL_PEAK_G,
                            "basis": "n*W mixed XYZZ adds x 10 Fp-mul (madd-2008-s)"}
    out = {
        "metric": METRIC, "value": value, "unit": "Mscalar-mul/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32 limbs (BN254 Fp/Fr Montgomery, integer)", "data": "synthetic",
        "config": {"workload": "BN254 G1 MSM, 2^%d resident points + scalars per GPU "
                               "(BASELINE configs[1])" % args.log_n,
                   "points_per_gpu": n, "window_bits": c, "windows": W,
                   "parallelism": "msm point-shard x%d, RCCL all_gather of partials" % world},
        "roofline": roofline, "kernels": kernels,
    }

    # watchdog over the extras: the headline is already measured
    import threading
    printed = threading.Lock()
    stage = {"now": "ntt"}

    def emit():
        if printed.acquire(blocking=False):
            if rank == 0:
                print(json.dumps(out), flush=True)
            return True
        return False

    def bail():
        out.setdefault("extras_timeout", {"stage": stage["now"], "seconds": args.extras_timeout})
        emit()
        os._exit(0)

    wd = threading.Timer(args.extras_timeout, bail)
    wd.daemon = True
    wd.start()

    # ---- Fr NTT 2^24 (BASELINE configs[2]; extra, rank 0 / N = 1 only)
    if rank == 0 and world == 1 and args.ntt_log_n:
        try:
            out["ntt"] = ntt_bench(args.ntt_log_n)
        except Exception as e:  # report, never hide
            out["ntt"] = {"error": repr(e)}

    # ---- PlonK BLS12-381 hot ops (BASELINE configs[4] sizes; extra, rank 0 / N = 1 only)
    stage["now"] = "plonk"
    if rank == 0 and world == 1 and args.plonk_log_n:
        try:
            out["plonk_bls12_381"] = plonk_bench(args.plonk_log_n)
        except Exception as e:  # report, never hide
            out["plonk_bls12_381"] = {"error": repr(e)}

    # ---- PlonK BLS12-381 prove, end to end (BASELINE configs[4]; rank 0 / N = 1 only)
    # (at N > 1 every rank keeps a 1/N slice of the KZG bases; commitments are
    # partial MSMs all-gathered over RCCL, the rest of the prover is replicated)
    stage["now"] = "plonk_prove"
    if args.plonk_log_n:
        try:
            pr = plonk_prove_bench(args.plonk_log_n, rank=rank, world=world, dist=dist, xdev=xdev,
                                   barrier=barrier)
        except Exception as e:  # report, never hide
            pr = {"error": repr(e)}
        if rank == 0:
            out.setdefault("plonk_bls12_381", {})["prove"] = pr

    # ---- Groth16 prove (extra): whole key at N = 1; at N > 1 one key shard per
    # GPU (wires and Z positions partitioned, h computed on every GPU, 576-B
    # partials all-gathered) -- strong scaling of one 2^log_n proof
    stage["now"] = "groth16"
    if args.groth16_log_n:
        try:
            if world == 1:
                g16 = groth16_bench(args.groth16_log_n)
            else:
                g16 = groth16_bench_sharded(args.groth16_log_n, rank, world, dist, xdev, barrier)
        except Exception as e:  # report, never hide
            g16 = {"error": repr(e)}
        if rank == 0:
            out["groth16"] = g16

    # ---- CPU baseline (oracle restatement on the host cores), rank 0 at N = 1
    stage["now"] = "cpu_baseline"
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(base, dsc, sc, n, args.cpu_threads)
        except Exception as e:
            out["cpu_baseline"] = {"error": repr(e)}

    wd.cancel()
    emit()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def pmc_traffic(kernel, log_n, c, W):
    """HBM bytes per launch of `kernel` from the committed PMC profile of the same
    workload (two separate rocprofv3 --pmc passes, FETCH_SIZE x2 per the gfx950
    correction + WRITE_SIZE; tools/pmc_traffic.py).  None if no matching profile."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        wl = d.get("workload", {})
        if (wl.get("log_n"), wl.get("window_bits"), wl.get("windows")) != (log_n, c, W):
            continue
        for k, v in d.get("kernels", {}).items():
            if kernel in k:
                return v["traffic_bytes"], (
                    f"{os.path.basename(f)}: FETCH_SIZE x2 + WRITE_SIZE per dispatch; the W={W} "
                    f"precomputed window copies make the kernel read ~W x 64 B of points per scalar "
                    f"(fixed-base trade: no doublings), so traffic >> the 96 B/scalar algorithmic bytes")
    return None, "no committed PMC profile for this workload"


def cpu_baseline(base, dsc, sc, n, threads):
    """C restatement of the same MSM (oracle/c, OpenMP Pippenger) on a bounded
    sample: the first 2^18 points/scalars of the workload, repeated ~10 s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle
    from gnark_amd import msm
    nt = threads or min(16, os.cpu_count() or 1)
    m = min(n, 1 << 18)
    # the sample's points: regenerate the first m on the GPU and copy to host
    ks = rand_scalars(n, 1000)[:m]
    pts = msm.batch_scalar_mul(msm.G1, g1_generator_mont(), ks, m)
    sb = sc[:m].tobytes()
    reps, t0 = 0, time.perf_counter()
    while True:
        coracle.msm_g1(pts, sb, m, nt)
        reps += 1
        if time.perf_counter() - t0 > 10.0 or reps >= 50:
            break
    el = time.perf_counter() - t0
    return {"value": m * reps / el / 1e6, "unit": "Mscalar-mul/s", "cores": nt, "kind": "port",
            "sample": f"G1 MSM 2^{m.bit_length() - 1} points x {reps} reps (C restatement, "
                      f"signed-digit Pippenger, {nt} OpenMP threads, not gnark)"}


def ntt_bench(log_n, reps=10):
    """Forward DIF + inverse DIT round trip on a resident 2^log_n Fr vector
    (BASELINE configs[2]); per-transform time from wall clock and from HIP events
    on the pass kernel (algorithmic bytes 2*n*32 per transform)."""
    import gnark_amd
    from gnark_amd import _lib, ntt, DeviceBuffer
    n = 1 << log_n
    d = ntt.Domain(log_n)
    x = rand_scalars(n, 77)
    buf = DeviceBuffer.from_host(x.tobytes())
    d.fft(buf, ntt.DIF)
    d.fft_inverse(buf, ntt.DIT)
    _lib.check(_lib.lib.gg_synchronize())
    t = time.perf_counter()
    for _ in range(reps):
        d.fft(buf, ntt.DIF)
        d.fft_inverse(buf, ntt.DIT)
    _lib.check(_lib.lib.gg_synchronize())
    ms = 1e3 * (time.perf_counter() - t) / (2 * reps)
    _lib.profile_enable(True)
    for _ in range(3):
        d.fft(buf, ntt.DIF)
        d.fft_inverse(buf, ntt.DIT)
    tot, cnt, _ = _lib.profile_get("ntt_pass")
    _lib.profile_enable(False)
    _lib.check(_lib.lib.gg_synchronize())
    ok = buf.to_host() == x.tobytes()  # size-independent property: exact round trip
    d.close()
    alg = 2 * n * 32
    passes_per_transform = cnt / 6 if cnt else None
    return {"log_n": log_n, "ms_per_transform": ms, "round_trip_exact": ok,
            "butterflies_per_s": (n // 2) * log_n / (ms * 1e-3),
            "algorithmic_GBps": alg / (ms * 1e-3) / 1e9,
            "hbm_frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "pass_kernel_avg_ms": tot / cnt if cnt else None,
            "passes_per_transform": passes_per_transform,
            "pass_GBps": (alg / (tot / cnt * 1e-3) / 1e9) if cnt else None}


BLS_G1_GEN = (0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
              0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1)


def plonk_bench(log_n, reps=5):
    """BLS12-381 PlonK hot ops at n = 2^log_n (small domain), big domain 4n:
    a KZG-commit-sized G1 MSM (2^log_n resident points), small/big domain Fr
    FFTs, one coset of the fused numerator, divideByXMinusOne on the big domain."""
    from gnark_amd import _lib, fr, msm, ntt, plonk, DeviceBuffer
    n = 1 << log_n
    res = {"log_n": log_n, "big_log_n": log_n + 2}

    def timed(fn, k=reps):
        fn()
        _lib.check(_lib.lib.gg_synchronize())
        t = time.perf_counter()
        for _ in range(k):
            fn()
        _lib.check(_lib.lib.gg_synchronize())
        return 1e3 * (time.perf_counter() - t) / k

    def bls_scalars(k, seed):
        a = rand_scalars(k, seed)
        a[:, 3] &= np.uint64((1 << 60) - 1)  # < r_bls
        return np.ascontiguousarray(a)

    import numpy as np
    gen = fr.bls_fp_mont(BLS_G1_GEN[0]) + fr.bls_fp_mont(BLS_G1_GEN[1])
    pts = DeviceBuffer(96 * n)
    msm.batch_scalar_mul(msm.BLS12_381_G1, gen, bls_scalars(n, 31), n, out=pts)
    base = msm.MsmBase(msm.BLS12_381_G1, pts.ptr, n, on_device=True)
    del pts
    npts, c, W = base.info()
    dsc = DeviceBuffer.from_host(bls_scalars(n, 32).tobytes())
    ms = timed(lambda: base.msm_jac(dsc, n, on_device=True))
    res["msm_g1"] = {"ms": ms, "Mscalar_mul_per_s": n / (ms * 1e-3) / 1e6, "window_bits": c, "windows": W}
    base.close()
    for lg, key in ((log_n, "ntt_small"), (log_n + 2, "ntt_big")):
        d = ntt.Domain(lg, fr.bls_fr_mont(fr.bls_domain_generator(lg)),
                       fr.bls_fr_mont(fr.BLS_FR_MULTIPLICATIVE_GEN), curve=ntt.GG_CURVE_BLS12_381)
        buf = DeviceBuffer.from_host(bls_scalars(1 << lg, 40 + lg).tobytes())
        ms = timed(lambda: (d.fft(buf, ntt.DIF, True), d.fft_inverse(buf, ntt.DIT, True)))
        res[key] = {"ms_per_transform": ms / 2}
        if key == "ntt_big":
            res["divide_by_xn_minus_one_ms"] = timed(lambda: plonk.divide_by_xn_minus_one(d, n, buf))
        d.close()
    # one coset of the numerator: 15 polynomials + 1 BSB22 pair
    xs = [DeviceBuffer.from_host(bls_scalars(n, 50 + i).tobytes()) for i in range(17)]
    tw0 = DeviceBuffer.from_host(bls_scalars(n, 70).tobytes())
    cres = DeviceBuffer(4 * n * 32)
    one = fr.bls_fr_mont(3)
    bl = [[one, one], [one, one], [one, one], [one, one, one]]
    res["numerator_coset_ms"] = timed(lambda: plonk.numerator_coset(
        xs, bl, tw0, one, one, one, fr.bls_fr_mont(7), n, 4, 1, cres))
    # row a21: copy-constraint ratio Z, Horner evaluation + KZG opening quotient,
    # foldH, linearized polynomial (all at the small domain size n)
    perm = DeviceBuffer.from_host(np.random.default_rng(3).permutation(3 * n).astype(np.int64).tobytes())
    z = DeviceBuffer(32 * n)
    w = fr.bls_fr_mont(fr.bls_domain_generator(log_n))
    u = fr.bls_fr_mont(fr.BLS_FR_MULTIPLICATIVE_GEN)
    res["ratio_copy_constraint_ms"] = timed(lambda: plonk.ratio_copy_constraint(
        xs[0], xs[1], xs[2], perm, n, one, fr.bls_fr_mont(5), w, u, z))
    q = DeviceBuffer(32 * n)
    res["evaluate_and_open_quotient_ms"] = timed(lambda: plonk.evaluate(xs[3], n, fr.bls_fr_mont(11), q_out=q))
    hbuf = DeviceBuffer(3 * (n + 2) * 32)
    folded = DeviceBuffer((n + 2) * 32)  # foldH writes n + 2 coefficients
    res["fold_h_ms"] = timed(lambda: plonk.fold_h(hbuf, n, fr.bls_fr_mont(13), folded))
    sc = [3, 5, 7, 11, 13, 17, 19, 23]
    res["linearized_ms"] = timed(lambda: plonk.linearized(z, n, xs[4], n, xs[5:10], n, sc))
    return res


def plonk_prove_bench(log_n, reps=2, per_rep=False, rank=0, world=1, dist=None, xdev=None,
                      barrier=None):
    """BLS12-381 PlonK prove (gnark_amd.plonk_prover: every step of prove.go on the
    GPU) at n = 2^log_n with a synthetic key (random SRS points, selectors and
    copy permutation) and a random witness, inputs resident in HBM.  The proof of
    a random witness does not verify; the work is that of a real proof."""
    import numpy as np
    from gnark_amd import fr, msm, plonk_prover as pp, DeviceBuffer
    n = 1 << log_n

    def bls_dev(k, seed):
        a = rand_scalars(k, seed)
        a[:, 3] &= np.uint64((1 << 60) - 1)
        return DeviceBuffer.from_host(np.ascontiguousarray(a).tobytes())

    t0 = time.time()
    gen = fr.bls_fp_mont(BLS_G1_GEN[0]) + fr.bls_fp_mont(BLS_G1_GEN[1])
    kzg = DeviceBuffer(96 * (n + 3))
    msm.batch_scalar_mul(msm.BLS12_381_G1, gen, bls_dev(n + 3, 61), n + 3, scalars_on_device=True, out=kzg)
    lag = DeviceBuffer(96 * n)
    msm.batch_scalar_mul(msm.BLS12_381_G1, gen, bls_dev(n, 62), n, scalars_on_device=True, out=lag)
    sel = [bls_dev(n, 70 + i) for i in range(8)]
    perm = np.random.default_rng(71).permutation(3 * n).astype(np.int64).tobytes()
    shard, reduce = None, None
    if world > 1:
        from gnark_amd import dist as gdist
        shard = (rank, world)

        def reduce(jac):
            return gdist.allgather_partial(msm.BLS12_381_G1, jac, device=xdev)
    pk = pp.ProvingKey(log_n, kzg, lag, *sel, perm, shard=shard, reduce=reduce)
    del kzg, lag, sel
    L, R_, O = (bls_dev(n, 80 + i) for i in range(3))
    t_setup = time.time() - t0

    def rng():  # the blinding randomness must be identical on every rank
        import random
        return random.Random(1234)

    pp.prove(pk, L, R_, O, rng=rng())
    ts, tim, tims = [], {}, []
    for _ in range(reps):
        if barrier is not None and world > 1:
            barrier()
        t = time.perf_counter()
        tim = {}
        pp.prove(pk, L, R_, O, timings=tim, rng=rng())
        if barrier is not None and world > 1:
            barrier()
        el = 1e3 * (time.perf_counter() - t)
        if world > 1:
            import torch
            tt = torch.tensor([el], dtype=torch.float64, device=xdev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        ts.append(el)
        tims.append(tim)
    tim = tims[ts.index(min(ts))]
    extra = {"stage_ms_all": tims} if per_rep else {}
    return {"log_n": log_n, "n_gpus": world, "prove_ms": min(ts), "prove_ms_all": ts, "stage_ms": tim,
            **extra, "kzg_bases": "1/%d slice per GPU, partial commitments all-gathered" % world,
            "key_setup_s": t_setup, "msms_per_proof": 10, "ntts_per_proof": "16 coset FFTs (L,R,O,Z x 4 cosets; key polynomials resident) + 4 iFFTs of n + 1 coset iFFT of 4n",
            "note": "synthetic key + random witness (timing only; proofs of valid witnesses verify in "
                    "tests/test_gpu_plonk_prove.py)"}


def groth16_bench(log_n, reps=3):
    """Synthetic 2^log_n Groth16 prove, key generated on the GPU; inputs resident."""
    import numpy as np
    from gnark_amd import backend, groth16, msm, DeviceBuffer
    n = 1 << log_n
    n_wires = n - 3
    nb_public = 2
    rng = np.random.default_rng(5)
    infA = np.zeros(n_wires, dtype=np.uint8)
    infB = (rng.random(n_wires) < 0.3).astype(np.uint8)
    nA, nB, nK = n_wires, int((infB == 0).sum()), n_wires - nb_public
    t0 = time.time()
    g1 = g1_generator_mont()

    def g1pts(k, seed):
        return msm.batch_scalar_mul(msm.G1, g1, rand_scalars(k, seed), k)

    d = groth16.ProvingKeyData(
        log_n=log_n, g1_A=g1pts(nA, 1), g1_B=g1pts(nB, 2), g1_Z=g1pts(n - 1, 3), g1_K=g1pts(nK, 4),
        alpha1=g1pts(1, 5), beta1=g1pts(1, 6), delta1=g1pts(1, 7),
        g2_B=msm.batch_scalar_mul(msm.G2, g2_generator_mont(), rand_scalars(nB, 8), nB),
        beta2=msm.batch_scalar_mul(msm.G2, g2_generator_mont(), rand_scalars(1, 9), 1),
        delta2=msm.batch_scalar_mul(msm.G2, g2_generator_mont(), rand_scalars(1, 10), 1),
        infinity_A=infA.tobytes(), infinity_B=infB.tobytes(), nb_public=nb_public)
    pk = groth16.ProvingKey(d)
    t_setup = time.time() - t0
    wires = DeviceBuffer.from_host(rand_scalars(n_wires, 11).tobytes())
    ncons = n - 5
    sa, sb, sc = (DeviceBuffer.from_host(rand_scalars(ncons, 12 + i).tobytes()) for i in range(3))
    sol = groth16.Solution(wires, sa, sb, sc, n_wires, ncons, on_device=True)
    groth16.prove(pk, sol, backend.with_amd_acceleration())
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        groth16.prove(pk, sol, backend.with_amd_acceleration())
        ts.append(1e3 * (time.perf_counter() - t))
    tim = groth16.last_timings()
    # the same prove with the five tasks run one after another: isolated stage times
    os.environ["GG_G16_SERIAL"] = "1"
    try:
        t = time.perf_counter()
        groth16.prove(pk, sol, backend.with_amd_acceleration())
        t_serial = 1e3 * (time.perf_counter() - t)
        tim_serial = groth16.last_timings()
    finally:
        del os.environ["GG_G16_SERIAL"]
    return {"serial_prove_ms": t_serial, "serial_stage_ms": tim_serial,
            "log_n": log_n, "n_constraints": ncons, "n_wires": n_wires,
            "prove_ms": min(ts), "prove_ms_all": ts, "constraints_per_s": ncons / (min(ts) * 1e-3),
            "stage_ms": tim, "key_setup_s": t_setup, "inputs": "resident in HBM"}


def groth16_bench_sharded(log_n, rank, world, dist, xdev, barrier, reps=3):
    """Synthetic 2^log_n Groth16 prove over `world` GPUs: this rank generates only
    its own key shard on its GPU (groth16.KeyShard), inputs resident; the prove
    time is the max over ranks between barriers."""
    import numpy as np
    import torch
    from gnark_amd import backend, groth16, msm, DeviceBuffer
    n = 1 << log_n
    n_wires = n - 3
    nb_public = 2
    rng = np.random.default_rng(5)
    infA = np.zeros(n_wires, dtype=np.uint8)
    infB = (rng.random(n_wires) < 0.3).astype(np.uint8)
    lo, hi, zl, zh = groth16.shard_ranges(n_wires, n, rank, world)
    t0 = time.time()
    g1 = g1_generator_mont()
    sd = 100 * (rank + 1)

    def g1pts(k, seed):
        return msm.batch_scalar_mul(msm.G1, g1, rand_scalars(k, seed), k) if k else b""

    nA = int((infA[lo:hi] == 0).sum())
    nB = int((infB[lo:hi] == 0).sum())
    nK = max(hi, nb_public) - max(lo, nb_public)
    sh = groth16.KeyShard(lo, hi, zl, g1_A=g1pts(nA, sd + 1), g1_B=g1pts(nB, sd + 2),
                          g2_B=msm.batch_scalar_mul(msm.G2, g2_generator_mont(),
                                                    rand_scalars(nB, sd + 8), nB) if nB else b"",
                          g1_K=g1pts(nK, sd + 4), g1_Z=g1pts(zh - zl, sd + 3), k_wire_index=None)
    d = groth16.ProvingKeyData(
        log_n=log_n, g1_A=b"", g1_B=b"", g1_Z=b"", g1_K=b"",
        alpha1=g1pts(1, 5), beta1=g1pts(1, 6), delta1=g1pts(1, 7), g2_B=b"",
        beta2=msm.batch_scalar_mul(msm.G2, g2_generator_mont(), rand_scalars(1, 9), 1),
        delta2=msm.batch_scalar_mul(msm.G2, g2_generator_mont(), rand_scalars(1, 10), 1),
        infinity_A=infA.tobytes(), infinity_B=infB.tobytes(), nb_public=nb_public)
    pk = groth16.ProvingKeyShard(d, rank, world, shard=sh)
    del sh
    t_setup = time.time() - t0
    wires = DeviceBuffer.from_host(rand_scalars(n_wires, 11).tobytes())
    ncons = n - 5
    sa, sb, sc = (DeviceBuffer.from_host(rand_scalars(ncons, 12 + i).tobytes()) for i in range(3))
    sol = groth16.Solution(wires, sa, sb, sc, n_wires, ncons, on_device=True)
    r, s = fr_const(12345), fr_const(67890)
    opt = backend.with_amd_acceleration()
    use_dist_h = groth16.dist_h_supported(n, world)
    if use_dist_h:
        # computeH split over the GPUs: three all-to-alls of n/N^2 x 32 B chunks per proof
        hs = groth16.HShard(log_n, rank, world)
        xchg = groth16.TorchExchange(hs.exchange_bytes, torch.device("cuda", torch.cuda.current_device()))

        def prove_once():
            return groth16.prove_distributed_h(pk, hs, xchg, sol, opt, r=r, s=s, device=xdev)
    else:
        def prove_once():
            return groth16.prove_distributed(pk, sol, opt, r=r, s=s, device=xdev)
    prove_once()
    ts = []
    for _ in range(reps):
        barrier()
        t = time.perf_counter()
        pr = prove_once()
        barrier()
        el = time.perf_counter() - t
        tt = torch.tensor([el], dtype=torch.float64, device=xdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ts.append(1e3 * float(tt.item()))
    tim = groth16.last_timings()
    # every rank must hold the same proof
    pt = torch.frombuffer(bytearray(pr.Ar + pr.Bs + pr.Krs), dtype=torch.uint8).to(xdev)
    p0 = pt.clone()
    dist.broadcast(p0, 0)
    same = bool(torch.equal(pt, p0))
    return {"log_n": log_n, "n_gpus": world, "n_constraints": ncons, "n_wires": n_wires,
            "prove_ms": min(ts), "prove_ms_all": ts, "constraints_per_s": ncons / (min(ts) * 1e-3),
            "rank0_stage_ms": tim, "key_setup_s": t_setup, "proof_identical_on_all_ranks": same,
            "sharding": "wires [lo,hi) of A/B1/K/G2 and Z positions per GPU; 576-B partials all-gathered",
            "compute_h": ("distributed: local n/N transforms + 3 all-to-alls (gg_hshard)" if use_dist_h
                          else "replicated on every GPU"),
            "inputs": "resident in HBM"}


def fr_const(v):
    from gnark_amd import fr
    return fr.fr_mont(v)


if __name__ == "__main__":
    main()
