"""World-size-2 gloo test of the multi-GPU MSM path on the CPU: shard the key,
compute per-rank partials (the C oracle stands in for the per-GPU gg_msm), then
the product's all-gather + exact combine must equal the unsharded MSM."""
import os
import socket

import pytest

import bn254_oracle as o


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "gnark-fork_amd"), here):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import coracle
    from helpers import random_fr_mont, random_g1_points
    from gnark_amd import dist as gd, msm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pts = random_g1_points(n, 5)
    sc = random_fr_mont(n, 6)
    lo, hi = gd.shard_range(n, rank, world)
    part_aff = coracle.msm_g1(pts[lo * 64:hi * 64].tobytes(), sc[lo:hi].tobytes(), hi - lo)
    # affine -> Jacobian partial (Z = 1, or infinity)
    one = o.fp_to_bytes(1)
    jac = part_aff + one if part_aff != bytes(64) else o.fp_to_bytes(1) * 2 + bytes(32)
    tot = gd.allgather_partial(msm.G1, jac)
    q.put((rank, msm.jac_to_affine(msm.G1, tot)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_msm_allgather_gloo(world):
    import multiprocessing as mp
    import coracle
    from helpers import random_fr_mont, random_g1_points
    n = 3001
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pts = random_g1_points(n, 5)
    sc = random_fr_mont(n, 6)
    exp = coracle.msm_g1(pts.tobytes(), sc.tobytes(), n)
    for _, got in res:
        assert got == exp


def test_shard_ranges_cover():
    from gnark_amd import dist as gd
    for n in (0, 1, 7, 1 << 20):
        for w in (1, 2, 3, 8):
            rs = [gd.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))


def _group_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (root, os.path.join(root, "gnark-fork_amd"), here):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from gnark_amd import dist as gd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    devs = gd.group_devices(10 + rank)
    payload = bytes(range(200)) if rank == 0 else None
    got = gd.broadcast_bytes(payload, 200, 0)
    q.put((rank, devs, got))
    dist.barrier()
    dist.destroy_process_group()


def test_group_devices_and_proof_broadcast_gloo():
    """The process-group plumbing of the leader-driven PlonK key (GroupProvingKey /
    prove_group): every rank learns every rank's device in rank order, and the
    leader's proof bytes reach every rank."""
    import multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_group_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, devs, got in res:
        assert devs == [10, 11]
        assert got == bytes(range(200))


def test_plonk_proof_bytes_round_trip():
    """prove_group ships the proof in the library's layout: Proof.parse and
    proof_bytes are inverse on both curves, with BSB22 commitments."""
    import random as rnd
    from gnark_amd import plonk_prover as pp
    r = rnd.Random(5)
    for curve, pt, R in (("bls12-381", 96, pp.R), ("bn254", 64, None)):
        F = pp._Field(curve)
        for n_cmt in (0, 2):
            pts = [bytes(r.randrange(256) for _ in range(pt)) for _ in range(9 + n_cmt)]
            vals = [r.randrange(F.R) for _ in range(8 + n_cmt)]
            raw = (b"".join(pts[:8 + n_cmt]) + b"".join(F.mont(v) for v in vals[:7 + n_cmt]) + pts[-1]
                   + F.mont(vals[-1]))
            pr = pp.Proof.parse(raw, n_cmt, curve)
            assert pp.proof_bytes(pr, curve) == raw
