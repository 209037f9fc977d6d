"""Multi-GPU Groth16 on the CPU: the key is cut into shards
(groth16.slice_key), each shard's five MSM partials are computed by the C
oracle (standing in for gg_groth16_prove_partial on its GPU), the partials are
summed with the library's exact group law -- directly, and through a
world-size-2 gloo all-gather -- and gg_groth16_finalize (host code of the
library) must give the golden proof byte for byte (prove.go:177-299)."""
import os
import socket

import numpy as np
import pytest

import bn254_oracle as o
from helpers import b, golden

ONE = o.fp_to_bytes(1)
ZERO = bytes(32)


def _g1_jac(aff: bytes) -> bytes:
    return aff + ONE if aff != bytes(64) else ONE + ONE + ZERO


def _g2_jac(aff: bytes) -> bytes:
    one2 = ONE + ZERO
    return aff + one2 if aff != bytes(128) else one2 + one2 + ZERO + ZERO


def _key(g, explicit_k=False):
    from gnark_amd import groth16
    nw = len(b(g["infA"]))
    nk = len(b(g["g1_K"])) // 64
    kidx = list(range(g["nb_public"], g["nb_public"] + nk)) if explicit_k else None
    return groth16.ProvingKeyData(
        log_n=g["log_n"], g1_A=b(g["g1_A"]), g1_B=b(g["g1_B"]), g1_Z=b(g["g1_Z"]),
        g1_K=b(g["g1_K"]), alpha1=b(g["alpha1"]), beta1=b(g["beta1"]), delta1=b(g["delta1"]),
        g2_B=b(g["g2_B"]), beta2=b(g["beta2"]), delta2=b(g["delta2"]),
        infinity_A=b(g["infA"]), infinity_B=b(g["infB"]), nb_public=g["nb_public"],
        k_wire_index=kidx), nw


def oracle_partials(data, g, rank, world) -> bytes:
    """The five MSM partials of shard `rank`, computed by the C oracle."""
    import coracle
    from gnark_amd import groth16
    sh = groth16.slice_key(data, rank, world)
    W = np.frombuffer(b(g["wires"]), dtype=np.uint8).reshape(-1, 32)
    infA = np.frombuffer(b(g["infA"]), dtype=np.uint8)
    infB = np.frombuffer(b(g["infB"]), dtype=np.uint8)
    wires = np.arange(sh.wire_lo, sh.wire_hi)
    wa = wires[infA[sh.wire_lo:sh.wire_hi] == 0]
    wb = wires[infB[sh.wire_lo:sh.wire_hi] == 0]
    nk = len(sh.g1_K) // 64
    wk = sh.k_wire_index if sh.k_wire_index is not None else \
        np.arange(max(sh.wire_lo, data.nb_public), max(sh.wire_lo, data.nb_public) + nk)
    h = np.frombuffer(b(g["h"]), dtype=np.uint8).reshape(-1, 32)
    nz = len(sh.g1_Z) // 64

    def g1(pts, sc):
        k = len(pts) // 64
        return _g1_jac(coracle.msm_g1(pts, sc.tobytes(), k) if k else bytes(64))

    parts = [g1(sh.g1_A, W[wa]), g1(sh.g1_B, W[wb]), g1(sh.g1_K, W[np.asarray(wk, dtype=np.int64)]),
             g1(sh.g1_Z, h[sh.z_lo:sh.z_lo + nz])]
    k2 = len(sh.g2_B) // 128
    parts.append(_g2_jac(coracle.msm_g2(sh.g2_B, W[wb].tobytes(), k2) if k2 else bytes(128)))
    return b"".join(parts)


@pytest.mark.parametrize("idx", [0, 1])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_sharded_partials_finalize_to_golden(idx, world):
    from gnark_amd import groth16
    g = golden()["groth16"][idx]
    data, nw = _key(g, explicit_k=(world == 3))
    # shards partition the key
    shards = [groth16.slice_key(data, r, world) for r in range(world)]
    assert sum(len(s.g1_A) for s in shards) == len(data.g1_A)
    assert sum(len(s.g1_B) for s in shards) == len(data.g1_B)
    assert sum(len(s.g1_K) for s in shards) == len(data.g1_K)
    assert b"".join(s.g1_Z for s in shards) == data.g1_Z
    parts = [oracle_partials(data, g, r, world) for r in range(world)]
    pr = groth16.finalize(data, groth16.add_partials(parts), b(g["r"]), b(g["s"]))
    assert (pr.Ar.hex(), pr.Bs.hex(), pr.Krs.hex()) == (g["Ar"], g["Bs"], g["Krs"])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, idx, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "gnark-fork_amd"), here):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from gnark_amd import groth16
    from test_groth16_shard_cpu import _key, oracle_partials
    from helpers import b, golden
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = golden()["groth16"][idx]
    data, _ = _key(g)
    part = oracle_partials(data, g, rank, world)
    pr = groth16.gather_and_finalize(data, part, b(g["r"]), b(g["s"]))
    q.put((rank, pr.Ar.hex(), pr.Bs.hex(), pr.Krs.hex()))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_prove_gloo_world2():
    import multiprocessing as mp
    world, idx = 2, 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, idx, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = golden()["groth16"][idx]
    for _, ar, bs, krs in res:
        assert (ar, bs, krs) == (g["Ar"], g["Bs"], g["Krs"])
