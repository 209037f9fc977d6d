"""Distributed computeH (gg_hshard_*) on one GPU: `world` rank
objects run the four phases with the all-to-alls done by the test (host
copies), and each rank's h block must equal the oracle's computeH output
h_bitrev[r m, (r+1) m) bit for bit (prove.go:353-396).  Then the whole sharded
prove with the distributed H runs with one thread per rank and an in-process
exchange, and must give the oracle's proof."""
import threading

import numpy as np
import pytest

import coracle
from helpers import b, golden, random_fr_mont

pytestmark = pytest.mark.gpu


def _exchange_host(sends, world, B):
    """recv_r = concat_k chunk_r(send_k), B bytes per chunk."""
    return [b"".join(sends[k][r * B:(r + 1) * B] for k in range(world)) for r in range(world)]


def dist_h_blocks(a, bb, c, fill, log_n, world, on_device=False, curve="bn254"):
    from gnark_amd import groth16, DeviceBuffer
    hs = [groth16.HShard(log_n, r, world, curve=curve) for r in range(world)]
    xb = hs[0].exchange_bytes
    inputs = (a, bb, c)
    if on_device:
        inputs = tuple(DeviceBuffer.from_host(x) for x in inputs)
    sends = []
    for r in range(world):
        s = DeviceBuffer(xb)
        hs[r].phase(1, *inputs, length=fill, on_device=on_device, out=s)
        sends.append(s.to_host())
    # per rank pair: 3 chunks (a, b, c) after phase 1, 2 (a, b) after phase 2
    assert hs[0].exchange_bytes_after(1) == xb // world
    for ph in (2, 3):
        recvs = _exchange_host(sends, world, hs[0].exchange_bytes_after(ph - 1))
        sends = []
        for r in range(world):
            rb, s = DeviceBuffer.from_host(recvs[r]), DeviceBuffer(xb)
            hs[r].phase(ph, recv=rb, out=s)
            sends.append(s.to_host())
    assert hs[0].exchange_bytes_after(3) == hs[0].m // world * 32  # h: one polynomial
    recvs = _exchange_host(sends, world, hs[0].exchange_bytes_after(3))
    blocks = []
    for r in range(world):
        h = DeviceBuffer(hs[r].m * 32)
        hs[r].phase(4, recv=DeviceBuffer.from_host(recvs[r]), out=h)
        blocks.append(h.to_host())
    return blocks


@pytest.mark.parametrize("log_n,world,fill", [(2, 1, 3), (2, 2, 4), (6, 2, 60), (6, 8, 61),
                                              (10, 4, 1000), (12, 8, 4093), (16, 2, 65531),
                                              (16, 16, 60000), (18, 8, 262139)])
def test_dist_h_vs_oracle(log_n, world, fill):
    n = 1 << log_n
    a, bb, c = (random_fr_mont(fill, 300 + log_n + i).tobytes() for i in range(3))
    exp = coracle.compute_h(a, bb, c, fill, log_n)
    blocks = dist_h_blocks(a, bb, c, fill, log_n, world, on_device=(world == 8))
    assert b"".join(blocks) == exp
    assert all(len(x) == n // world * 32 for x in blocks)


def test_dist_h_golden():
    for g in golden()["groth16"]:
        fill = len(b(g["solA"])) // 32
        blocks = dist_h_blocks(b(g["solA"]), b(g["solB"]), b(g["solC"]), fill, g["log_n"], 2)
        assert b"".join(blocks).hex() == g["h"]


BLS_R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _bls_vec(k, seed):
    from gnark_amd import fr
    rng = np.random.default_rng(seed)
    v = [int.from_bytes(rng.bytes(32), "little") % BLS_R for _ in range(k)]
    return v, b"".join(fr.bls_fr_mont(x) for x in v)


@pytest.mark.parametrize("log_n,world,fill", [(4, 2, 13), (6, 8, 61), (10, 4, 1000), (16, 8, 65000),
                                              (18, 2, 262000)])
def test_dist_h_bls12_381(log_n, world, fill):
    """The four-step computeH over BLS12-381 fr (groth16/bls12-381/prove.go:353-396):
    the blocks equal the one-GPU computeH of the same domain (whose proofs are
    bit-exact vs the oracle, test_gpu_bls_groth16.py); at small sizes h also
    satisfies h(z) (z^n - 1) = A(z) B(z) - C(z) at a random z (pure Python)."""
    from gnark_amd import fr, ntt, DeviceBuffer
    n = 1 << log_n
    # a satisfied "R1CS": c = a b on the domain, so A B - C vanishes there and
    # h (X^n - 1) = A B - C holds as polynomials (checked below at small sizes)
    vs = [_bls_vec(fill, 900 + log_n + i) for i in range(2)]
    cv = [x * y % BLS_R for x, y in zip(vs[0][0], vs[1][0])]
    vs.append((cv, b"".join(fr.bls_fr_mont(x) for x in cv)))
    blocks = dist_h_blocks(*(x[1] for x in vs), fill, log_n, world, on_device=(world == 8), curve="bls12-381")
    assert all(len(x) == n // world * 32 for x in blocks)
    dom = ntt.Domain(log_n, fr.bls_fr_mont(fr.bls_domain_generator(log_n)),
                     fr.bls_fr_mont(fr.BLS_FR_MULTIPLICATIVE_GEN), curve=ntt.GG_CURVE_BLS12_381)
    h = DeviceBuffer(32 * n)
    dom.compute_h(*(x[1] for x in vs), fill, h)
    assert b"".join(blocks) == h.to_host()
    dom.close()
    if log_n <= 10:
        hb = b"".join(blocks)
        brev = [int(format(i, f"0{log_n}b")[::-1], 2) for i in range(n)]
        coef = [fr.bls_fr_unmont(hb[32 * brev[i]:32 * brev[i] + 32]) for i in range(n)]
        z = 0x5EED1234 + log_n
        w = fr.bls_domain_generator(log_n)
        zn1 = (pow(z, n, BLS_R) - 1) % BLS_R
        ninv = pow(n, BLS_R - 2, BLS_R)

        def lag(vals):  # sum_j v_j L_j(z), L_j(z) = w^j (z^n - 1) / (n (z - w^j))
            acc, wj = 0, 1
            for v in vals:
                acc += v * wj * pow(z - wj, BLS_R - 2, BLS_R)
                wj = wj * w % BLS_R
            return acc * zn1 * ninv % BLS_R
        hz = 0
        for cf in reversed(coef):
            hz = (hz * z + cf) % BLS_R
        ea, eb, ec = (lag(x[0]) for x in vs)
        assert hz * zn1 % BLS_R == (ea * eb - ec) % BLS_R


def test_dist_h_phase_order():
    """Phase 4 subtracts the c coefficients phase 2 leaves in the handle: the
    phases of a proof must run 1, 2, 3, 4 on a handle -- a phase out of order
    (a phase 4 with no phase 2, a second proof's phase 2 interleaved) is
    refused, not answered with a wrong h; phase 1 may start over."""
    from gnark_amd import groth16, DeviceBuffer, GnarkAmdError
    hs = groth16.HShard(8, 0, 2)
    xb = hs.exchange_bytes
    recv, h = DeviceBuffer.from_host(bytes(xb)), DeviceBuffer(hs.m * 32)
    with pytest.raises(GnarkAmdError):
        hs.phase(4, recv=recv, out=h)
    a = random_fr_mont(200, 5).tobytes()
    s = DeviceBuffer(xb)
    hs.phase(1, a, a, a, length=200, out=s)
    with pytest.raises(GnarkAmdError):  # phase 1 then 4: c's coefficients were never formed
        hs.phase(4, recv=recv, out=h)
    hs.phase(1, a, a, a, length=200, out=s)  # starting over is allowed
    hs.phase(2, recv=recv, out=s)
    with pytest.raises(GnarkAmdError):  # another proof's phase 2 interleaved
        hs.phase(2, recv=recv, out=s)
    hs.phase(3, recv=recv, out=s)
    hs.phase(4, recv=recv, out=h)  # in order: accepted
    with pytest.raises(GnarkAmdError):  # consumed
        hs.phase(4, recv=recv, out=h)
    hs.close()


def test_dist_h_rejects_bad_world():
    from gnark_amd import groth16, GnarkAmdError
    with pytest.raises(GnarkAmdError):
        groth16.HShard(10, 0, 3)
    with pytest.raises(GnarkAmdError):
        groth16.HShard(4, 0, 8)  # n < world^2


class LocalExchange:
    """In-process all-to-all between `world` rank threads on one GPU (chunks
    staged through host memory with gg_copy_to_host / gg_copy_to_device; no
    torch in this process, so the library keeps its own HIP runtime)."""

    def __init__(self, world, nbytes):
        from gnark_amd import DeviceBuffer
        self.world = world
        self.bar = threading.Barrier(world)
        self.send = [DeviceBuffer(nbytes) for _ in range(world)]
        self.recv = [DeviceBuffer(nbytes) for _ in range(world)]

    def for_rank(self, r):
        import ctypes
        from gnark_amd._lib import check, lib

        def fn(s_ptr, r_ptr, nbytes):
            assert s_ptr == self.send[r].ptr and r_ptr == self.recv[r].ptr
            self.bar.wait()
            tmp = ctypes.create_string_buffer(nbytes)
            for k in range(self.world):
                check(lib.gg_copy_to_host(tmp, ctypes.c_void_p(self.send[k].ptr + r * nbytes), nbytes))
                check(lib.gg_copy_to_device(ctypes.c_void_p(self.recv[r].ptr + k * nbytes), tmp, nbytes))
            self.bar.wait()
        return fn


def _prove_threads(data, sol, world, stripes=False):
    from gnark_amd import groth16
    log_n = data.log_n
    if stripes:  # bucket stripes: the whole wire tables per rank, stripe r of the buckets
        shards = [groth16.ProvingKeyStripe(data, r, world) for r in range(world)]
        assert [sh.stripe() for sh in shards] == [(world.bit_length() - 1, r) for r in range(world)]
    else:
        shards = [groth16.ProvingKeyShard(data, r, world) for r in range(world)]
    hs = [groth16.HShard(log_n, r, world) for r in range(world)]
    ex = LocalExchange(world, hs[0].exchange_bytes)
    parts, errs = [None] * world, []

    def run(r):
        try:
            parts[r] = groth16.prove_partial_dist(shards[r], hs[r], sol, ex.for_rank(r),
                                                  ex.send[r].ptr, ex.recv[r].ptr)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)
            ex.bar.abort()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errs, errs
    return groth16.add_partials(parts)


@pytest.mark.parametrize("idx,world", [(0, 2), (1, 2), (1, 4), (1, 8)])
def test_prove_dist_h_golden(idx, world):
    from gnark_amd import groth16
    from test_gpu_groth16 import _pk_from_golden
    g = golden()["groth16"][idx]
    data = _pk_from_golden(g)
    sol = groth16.Solution(b(g["wires"]), b(g["solA"]), b(g["solB"]), b(g["solC"]),
                           len(b(g["infA"])), len(b(g["solA"])) // 32)
    pr = groth16.finalize(data, _prove_threads(data, sol, world), b(g["r"]), b(g["s"]))
    assert (pr.Ar.hex(), pr.Bs.hex(), pr.Krs.hex()) == (g["Ar"], g["Bs"], g["Krs"])


@pytest.mark.parametrize("stripes", [False, True])
@pytest.mark.parametrize("log_n,n_wires,world,on_device", [(12, 3000, 4, False), (15, 30000, 8, True),
                                                           (13, 6000, 2, True)])
def test_prove_dist_h_vs_oracle(log_n, n_wires, world, on_device, stripes):
    from gnark_amd import groth16, DeviceBuffer
    from test_gpu_groth16 import synthetic_case
    d, wires, sa, sb, sc, ncons, r, s = synthetic_case(log_n, n_wires, 3, 10 + log_n, k_inf_every=5)
    data = groth16.ProvingKeyData(**d)
    exp = coracle.groth16_prove(
        log_n, d["g1_A"], len(d["g1_A"]) // 64, d["g1_B"], len(d["g1_B"]) // 64, d["g1_Z"],
        d["g1_K"], len(d["g1_K"]) // 64, d["alpha1"], d["beta1"], d["delta1"], d["g2_B"],
        d["beta2"], d["delta2"], d["infinity_A"], d["infinity_B"], wires, n_wires, 3, sa, sb, sc,
        ncons, r, s)
    if on_device:
        sol = groth16.Solution(*(DeviceBuffer.from_host(x) for x in (wires, sa, sb, sc)), n_wires,
                               ncons, on_device=True)
    else:
        sol = groth16.Solution(wires, sa, sb, sc, n_wires, ncons)
    pr = groth16.finalize(data, _prove_threads(data, sol, world, stripes), r, s)
    assert (pr.Ar, pr.Bs, pr.Krs) == exp[:3]
