"""Groth16 at the BASELINE sizes (config 4: a 2^24-constraint BN254 R1CS), bit-exact.

The instance is a satisfied synthetic R1CS of independent MiMC x^5 chains
(std/hash/mimc pow5 shape, 3 constraints per round; oracle/c/oracle_r1cs.c),
solved on the host; the proving key is generated on the GPU from seeded toxic
waste (known discrete logs, setup.go:212-275 layout: infinity flags, filtered
A/B, K of the private wires, Z bit-reversed).  The proof the GPU returns (from
host inputs, the path gnark's Prove takes: prove.go:127-320) must equal
(a G1, b G2, c G1) where (a, b, c) are the proof's discrete logs computed by
the O(n) C oracle (oc_groth16_expected: h(t) Z(t) = A(t) B(t) - C(t) holds on a
satisfied instance, so a wrong h shows up in Krs).  The h the GPU computed is
also checked by h(z) (z^n - 1) = A(z) B(z) - C(z) at a random point z.
"""
import time

import numpy as np
import pytest

import bn254_oracle as o
import coracle
from helpers import random_fr_mont

pytestmark = pytest.mark.gpu

TW = dict(tau=0x1DEA5EED1234567, alpha=0xA1FA0001, beta=0xBE7A0002, delta=0xDE17A0003)
R_, S_ = 0x5EED0001, 0x5EED0002


def _fr(v):
    return o.fr_to_bytes(v % o.R)


def _log(msg, t0):
    print(f"  [{time.time() - t0:6.1f}s] {msg}", flush=True)


def _instance(log_n, t0):
    from gnark_amd import groth16, msm
    rounds = 85
    chains = 1 << (log_n - 8)  # 255 * 2^(log_n-8) constraints: domain exactly 2^log_n
    cr = coracle.MimcR1CS(chains, rounds, 1)
    assert (1 << (log_n - 1)) < cr.ncons <= (1 << log_n)
    inputs = random_fr_mont(chains, 4000 + log_n).tobytes()
    wires = cr.solve(inputs)
    A, B, C, bad = cr.abc(wires)
    assert bad == 0
    _log(f"R1CS: {cr.ncons} constraints, {cr.nw} wires, solved", t0)
    tw = {k: _fr(v) for k, v in TW.items()}
    ks = cr.key_scalars(log_n, tw["tau"], tw["alpha"], tw["beta"], tw["delta"])
    _log("key discrete logs", t0)
    g1, g2 = o.g1_to_bytes(o.G1_GEN), o.g2_to_bytes(o.G2_GEN)

    def p1(sc):
        return msm.batch_scalar_mul(msm.G1, g1, sc, len(sc) // 32)

    def p2(sc):
        return msm.batch_scalar_mul(msm.G2, g2, sc, len(sc) // 32)
    data = groth16.ProvingKeyData(
        log_n=log_n, g1_A=p1(ks["A"]), g1_B=p1(ks["B"]), g1_Z=p1(ks["Z"]), g1_K=p1(ks["K"]),
        alpha1=p1(tw["alpha"]), beta1=p1(tw["beta"]), delta1=p1(tw["delta"]), g2_B=p2(ks["B"]),
        beta2=p2(tw["beta"]), delta2=p2(tw["delta"]), infinity_A=ks["infA"], infinity_B=ks["infB"],
        nb_public=cr.nb_public)
    del ks
    _log("key points (GPU batch scalar mul)", t0)
    exp = cr.expected(log_n, tw["tau"], tw["alpha"], tw["beta"], tw["delta"], wires, _fr(R_), _fr(S_))
    want = (bytes(coracle.g1_batch_mul(g1, exp[0], 1)), bytes(coracle.g2_batch_mul(g2, exp[1], 1)),
            bytes(coracle.g1_batch_mul(g1, exp[2], 1)))
    _log("expected proof (trapdoor)", t0)
    return cr, data, wires, (A, B, C), want


@pytest.mark.parametrize("log_n", [12, 18, 24])
def test_groth16_mimc_bit_exact(log_n):
    from gnark_amd import backend, groth16, DeviceBuffer
    t0 = time.time()
    cr, data, wires, (A, B, C), want = _instance(log_n, t0)
    pk = groth16.ProvingKey(data)
    _log("device key (precomputed windows)", t0)
    opt = backend.with_amd_acceleration()
    n = 1 << log_n
    # host inputs: the gnark path (solution slices in host memory)
    sol = groth16.Solution(bytes(wires), bytes(A), bytes(B), bytes(C), cr.nw, cr.ncons)
    h = DeviceBuffer(32 * n)
    pr = groth16.prove(pk, sol, opt, r=_fr(R_), s=_fr(S_), h_out=h)
    _log(f"prove (host inputs) {groth16.last_timings()['total']:.1f} ms", t0)
    assert (pr.Ar, pr.Bs, pr.Krs) == want
    # h (X^n - 1) = A B - C at a random point (size-independent property)
    z = _fr(0x7A11E5 + log_n)
    hz = o.fr_from_bytes(coracle.eval_bitrev(h.to_host(), log_n, z))
    ev = [o.fr_from_bytes(coracle.eval_lagrange(bytes(v), cr.ncons, log_n, z)) for v in (A, B, C)]
    zz = o.fr_from_bytes(z)
    assert hz * (pow(zz, n, o.R) - 1) % o.R == (ev[0] * ev[1] - ev[2]) % o.R
    _log("h identity", t0)
    # device-resident inputs: same proof
    dev = [DeviceBuffer.from_host(bytes(x)) for x in (wires, A, B, C)]
    sol_d = groth16.Solution(*dev, cr.nw, cr.ncons, on_device=True)
    pr2 = groth16.prove(pk, sol_d, opt, r=_fr(R_), s=_fr(S_))
    assert (pr2.Ar, pr2.Bs, pr2.Krs) == want
    _log("prove (device inputs)", t0)
    # a broken witness must not give the expected proof
    bad = bytearray(wires)
    bad[32 * (cr.nw - 1)] ^= 1
    pr3 = groth16.prove(pk, groth16.Solution(bytes(bad), bytes(A), bytes(B), bytes(C), cr.nw, cr.ncons),
                        opt, r=_fr(R_), s=_fr(S_))
    assert pr3.Krs != want[2]
    pk.close()
    if log_n == 24:  # the 8-GPU split of configs[3], rehearsed with 8 shards on this GPU:
        # wire slices (the product default: gg_groth16_mpk_create_ex, the Go shims'
        # SetDevices, bench's split_projection), then the opt-in bucket stripes
        _mpk_check(data, sol, sol_d, want, 8, t0, split="wires")
        _mpk_check(data, sol, sol_d, want, 8, t0, split="stripes")
    cr.close()


def _mpk_check(data, sol, sol_d, want, world, t0, split="wires"):
    """gg_groth16_mpk_* with `world` key shards (8 = BASELINE configs[3]'s node):
    wire slices (the default) or bucket stripes over whole per-device wire
    tables, and Z slices, the four-step distributed computeH with its three
    all-to-alls as peer copies, partials summed exactly -- same proof bytes,
    from host and from device-resident solutions."""
    import os
    from gnark_amd import backend, groth16
    opt = backend.with_amd_acceleration()
    old = os.environ.get("GG_MPK_SPLIT")
    os.environ["GG_MPK_SPLIT"] = split
    try:
        mpk = groth16.MultiGpuProvingKey(data, [0] * world)
    finally:
        if old is None:
            del os.environ["GG_MPK_SPLIT"]
        else:
            os.environ["GG_MPK_SPLIT"] = old
    assert mpk.info() == (world, True) and mpk.split() == split
    if split == "wires":  # a 2^21-wire slice of the 2^24 key picks its own (smaller) window
        _log(f"{world}-shard key (shard 0 A: c={mpk.base_info(groth16.BASE_A)[1]}, "
             f"W={mpk.base_info(groth16.BASE_A)[2]})", t0)
    else:
        _log(f"{world}-shard key", t0)
    pr = mpk.prove(sol, opt, r=_fr(R_), s=_fr(S_))
    _log(f"{world}-shard prove (host inputs) {mpk.last_timings()['total']:.1f} ms", t0)
    assert (pr.Ar, pr.Bs, pr.Krs) == want
    prd = mpk.prove(sol_d, opt, r=_fr(R_), s=_fr(S_))  # resident solution, shared by the shards of GPU 0
    _log(f"{world}-shard prove (device inputs) {mpk.last_timings()['total']:.1f} ms", t0)
    assert (prd.Ar, prd.Bs, prd.Krs) == want
    mpk.close()


@pytest.mark.parametrize("split", ["stripes", "wires"])
@pytest.mark.parametrize("log_n,world", [(16, 8), (18, 4)])
def test_groth16_mimc_multi_gpu_shards(log_n, world, split):
    """the same check at sizes the suite runs quickly"""
    from gnark_amd import groth16, DeviceBuffer
    t0 = time.time()
    cr, data, wires, (A, B, C), want = _instance(log_n, t0)
    sol = groth16.Solution(bytes(wires), bytes(A), bytes(B), bytes(C), cr.nw, cr.ncons)
    dev = [DeviceBuffer.from_host(bytes(x)) for x in (wires, A, B, C)]
    sol_d = groth16.Solution(*dev, cr.nw, cr.ncons, on_device=True)
    _mpk_check(data, sol, sol_d, want, world, t0, split)
    cr.close()
