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


# ------------------------------------------------- errgroup across ranks
# gnark ends a proof at the first failing task (backend/groth16/bn254/prove.go:
# 198-209 channels, backend/plonk/bls12-381/prove.go:132-173 errgroup); over a
# process group every rank must raise within seconds, not wait out the group's
# timeout.  The GPU work is replaced by stand-ins (no GPU here); the status
# protocol (gnark_amd.dist.RankGuard / broadcast_status) is the product's.

def _init(rank, world, port):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (root, os.path.join(root, "gnark-fork_amd"), here):
        sys.path.insert(0, p)
    import datetime
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # a long group timeout: a test passes only if the failure ends the wait, not the timeout
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=300))


def _outcome(fn):
    import time
    t = time.time()
    try:
        fn()
        return ("ok", "", time.time() - t)
    except BaseException as e:  # noqa: BLE001 - the test inspects it
        return (type(e).__name__, str(e), time.time() - t)


class _Fixed:
    def __init__(self, *a):
        self.closed = False

    def close(self):
        self.closed = True

    def finish(self, part):
        return part


class _Data:
    curve = "bn254"


class _PK:
    data = _Data()


def _g16_worker(rank, world, port, scenario, q):
    _init(rank, world, port)
    import torch
    import torch.distributed as dist
    from gnark_amd import backend, groth16
    from gnark_amd._lib import GnarkAmdError
    groth16.FixedTerms = _Fixed

    def partial(pk, sol):
        if rank == 1:
            raise RuntimeError("injected: bad witness on rank 1")
        return bytes(576)

    class Xchg:
        guard = None
        send = recv = torch.zeros(8)

        def __call__(self, s, r, nbytes):
            if self.guard is not None:
                self.guard.check("computeH all-to-all")
            t = torch.ones(1)
            dist.all_reduce(t)  # the all-to-all's stand-in

    def partial_dist(pk, hs, sol, exchange, send, recv):
        # the library's three exchanges; rank 1 fails between the first and the second
        for k in range(3):
            if rank == 1 and k == 1:
                raise GnarkAmdError(2, "injected: kernel fault on rank 1")
            try:
                exchange(send, recv, 8)
            except Exception:
                raise GnarkAmdError(2, "exchange callback failed")
        return bytes(576)

    groth16.prove_partial = partial
    groth16.prove_partial_dist = partial_dist
    opt = backend.with_amd_acceleration()
    if scenario == "partials":
        res = _outcome(lambda: groth16.prove_distributed(_PK(), None, opt, r=bytes(32), s=bytes(32)))
    else:
        res = _outcome(lambda: groth16.prove_distributed_h(_PK(), None, Xchg(), None, opt, r=bytes(32),
                                                           s=bytes(32)))
    q.put((rank, res))
    dist.destroy_process_group()


def _plonk_worker(rank, world, port, scenario, q):
    _init(rank, world, port)
    import torch.distributed as dist
    from gnark_amd import plonk_prover as pp
    if scenario == "prove":
        def prove(*a, **k):
            raise RuntimeError("injected: out of HBM on the leader")
        pp.prove = prove
        gpk = pp.GroupProvingKey.__new__(pp.GroupProvingKey)
        gpk.rank, gpk.curve, gpk.n_cmt, gpk.comm_device, gpk.pk = rank, "bls12-381", 0, None, object()
        res = _outcome(lambda: pp.prove_group(gpk, None, None, None))
    else:
        # rank r reports GPU "gpu-r" as its device r; rank 0 cannot open id 1 (a
        # launcher that isolates HIP_VISIBLE_DEVICES per rank)
        res = _outcome(lambda: pp.GroupProvingKey(local_device=rank, identity=lambda d: f"gpu-{d}",
                                                  view=lambda d: "gpu-0" if d == 0 else None))
    q.put((rank, res))
    dist.destroy_process_group()


def _run2(target, scenario):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, 2, port, scenario, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_groth16_rank_failure_ends_every_rank_gloo():
    """rank 1's partial fails: rank 0 raises RankFailure naming rank 1 at the
    status step before the partial all-gather, within seconds."""
    res = _run2(_g16_worker, "partials")
    assert res[1][0] == "RuntimeError" and "bad witness" in res[1][1]
    assert res[0][0] == "RankFailure" and "rank 1" in res[0][1] and "bad witness" in res[0][1]
    assert max(r[2] for r in res.values()) < 60


def test_groth16_dist_h_failure_between_exchanges_gloo():
    """rank 1 fails between the distributed computeH's first and second
    all-to-all: rank 0, waiting in the second exchange's status step, raises."""
    res = _run2(_g16_worker, "dist_h")
    assert res[1][0] == "GnarkAmdError" and "kernel fault" in res[1][1]
    assert res[0][0] == "RankFailure" and "kernel fault" in res[0][1]
    assert max(r[2] for r in res.values()) < 60


def test_plonk_leader_failure_ends_every_rank_gloo():
    """the leader's prove fails: the other rank raises RankFailure (no wait in
    the proof broadcast)."""
    res = _run2(_plonk_worker, "prove")
    assert res[0][0] == "RuntimeError" and "out of HBM" in res[0][1]
    assert res[1][0] == "RankFailure" and "rank 0" in res[1][1] and "out of HBM" in res[1][1]
    assert max(r[2] for r in res.values()) < 60


def test_plonk_leader_key_refused_gloo():
    """rank 0 cannot open rank 1's GPU: the leader key is refused on every rank
    with the reason, before any key is built."""
    res = _run2(_plonk_worker, "refuse")
    assert res[0][0] == "ValueError" and "not visible to rank 0" in res[0][1]
    assert res[1][0] == "RankFailure" and "not visible to rank 0" in res[1][1]


def test_check_leader_devices():
    from gnark_amd import dist as gd
    view = {0: "a", 1: "b", 2: "c"}.get
    assert gd.check_leader_devices([0, 1, 2], ["a", "b", "c"], view, "nccl") == []
    # ranks numbering the GPUs differently
    p = gd.check_leader_devices([0, 1], ["a", "c"], view, "nccl")
    assert len(p) == 1 and "numbers the GPUs differently" not in p[0] and "rank 1's GPU 1 is c" in p[0]
    # every rank on its own HIP_VISIBLE_DEVICES: all report id 0
    p = gd.check_leader_devices([0, 0], ["a", "b"], view, "nccl")
    assert any("rank 1's GPU 0 is b" in x for x in p)
    # two ranks on one GPU: refused under RCCL, allowed for a gloo rehearsal
    assert any("share GPU" in x for x in gd.check_leader_devices([0, 0], ["a", "a"], view, "nccl"))
    assert gd.check_leader_devices([0, 0], ["a", "a"], view, "gloo") == []
