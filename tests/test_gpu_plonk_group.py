"""PlonK under a process-per-GPU launch (torch.distributed, one process per
rank; the driver's N > 1 shape): plonk_prover.GroupProvingKey puts a
one-process multi-part key over every rank's GPU on rank 0, and prove_group
broadcasts the proof to every rank (round-4 VERDICT "next" 2).

Rehearsed on one GPU over gloo (every rank on device 0, so the key has N device
parts on that GPU): every rank's proof must be byte-identical to the one-GPU
proof of the same circuit, witness and blinding, and verify (restated
verifier, prove.go / verify.go:45-290 with the SRS trapdoor)."""
import os
import random
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, log_n, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "gnark-fork_amd"), here):
        sys.path.insert(0, p)
    try:
        import torch
        import torch.distributed as dist
        from plonk_circuits import Circuit, srs
        from gnark_amd import plonk_prover as pp, _lib
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        _lib.check(_lib.lib.gg_set_device(0))
        torch.cuda.set_device(0)
        circ = Circuit(log_n, 31 + log_n, nb_public=1, n_cmt=1)
        tau = random.Random(log_n + world).randrange(2, pp.R)
        sel, qcp = circ.selectors()
        perm = circ.permutation()
        cv = circ.F.cv
        s123 = circ.s_polys(perm, cv.omega(circ.n), cv.fr_gen)
        kzg, kzg_lag = srs(log_n, tau)
        gpk = pp.GroupProvingKey(log_n, kzg, kzg_lag, *sel, *s123, perm.tobytes(), qcp=qcp,
                                 nb_public=circ.nb_public, commitment_indexes=circ.cmt_idx, local_device=0)
        if rank == 0:
            assert gpk.pk.devices() == [0] * world
            L, Rv, O, pub, cmts = circ.solve(gpk.pk, 6, commit=gpk.pk.commit_lagrange)
        else:
            L = Rv = O = None
            pub, cmts = [0], [(bytes(32 * circ.n), bytes(96), 0)]
        # public / commitments are only read on rank 0; the shapes must match
        pr = pp.prove_group(gpk, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts)
        q.put((rank, pp.proof_bytes(pr), gpk.devices))
        gpk.close()
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put((rank, "ERR " + repr(e) + traceback.format_exc(), None))


@pytest.mark.parametrize("world", [2, 4])
def test_plonk_group_proof_matches_one_gpu(world):
    import multiprocessing as mp
    import bls12_381_oracle as bo
    from plonk_circuits import Circuit, make_key, srs, to_oracle
    from gnark_amd import plonk_prover as pp
    log_n = 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, log_n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r, b, _ in res:
        assert not (isinstance(b, str) and b.startswith("ERR")), b
    for p in procs:
        assert p.exitcode == 0
    # the one-GPU proof of the same circuit, witness and blinding
    circ = Circuit(log_n, 31 + log_n, nb_public=1, n_cmt=1)
    tau = random.Random(log_n + world).randrange(2, pp.R)
    pk0 = make_key(circ, tau, key_srs=srs(log_n, tau))
    L, Rv, O, pub, cmts = circ.solve(pk0, 6, commit=pk0.commit_lagrange)
    ref = pp.prove(pk0, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts)
    for r, b, devs in res:
        assert devs == [0] * world
        assert b == pp.proof_bytes(ref), f"rank {r}"
    pr, vk = to_oracle(pk0, ref)
    assert bo.plonk_verify_trapdoor(pr, vk, tau, public=pub)
    pk0.close()
