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


def dist_h_blocks(a, bb, c, fill, log_n, world, on_device=False):
    from gnark_amd import groth16, DeviceBuffer
    hs = [groth16.HShard(log_n, r, world) for r in range(world)]
    xb = hs[0].exchange_bytes
    inputs = (a, bb, c)
    if on_device:
        inputs = tuple(DeviceBuffer.from_host(x) for x in inputs)
    sends = []
    for r in range(world):
        s = DeviceBuffer(xb)
        hs[r].phase(1, *inputs, length=fill, on_device=on_device, out=s)
        sends.append(s.to_host())
    for ph in (2, 3):
        recvs = _exchange_host(sends, world, xb // world)
        sends = []
        for r in range(world):
            rb, s = DeviceBuffer.from_host(recvs[r]), DeviceBuffer(xb)
            hs[r].phase(ph, recv=rb, out=s)
            sends.append(s.to_host())
    recvs = _exchange_host(sends, world, hs[0].m // world * 32)  # h: one polynomial
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
