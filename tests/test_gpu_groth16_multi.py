"""One-process multi-GPU Groth16 (gg_groth16_mpk_*: the whole key handed over
once, shard r on devices[r], the distributed computeH's three all-to-alls done
as in-library peer copies) -- the shape a Go caller drives, SURVEY 8(b)/(e).

On the one-GPU test box every shard sits on device 0 (devices may repeat), so
the layout, the exchanges and the partial combination are checked bit-exact
against the golden proofs (prove.go restated in the oracle) and the C oracle;
on an 8-GPU node the same code places one shard per GPU."""
import numpy as np
import pytest

import coracle
from helpers import b, golden

pytestmark = pytest.mark.gpu


def _golden_solution(g):
    from gnark_amd import groth16
    return groth16.Solution(b(g["wires"]), b(g["solA"]), b(g["solB"]), b(g["solC"]),
                            len(b(g["infA"])), len(b(g["solA"])) // 32)


@pytest.mark.parametrize("idx,world", [(0, 1), (0, 2), (1, 2), (1, 3), (1, 4), (1, 8)])
def test_mpk_golden(idx, world):
    from gnark_amd import backend, groth16
    from test_gpu_groth16 import _pk_from_golden
    g = golden()["groth16"][idx]
    data = _pk_from_golden(g)
    mpk = groth16.MultiGpuProvingKey(data, [0] * world)
    w, dist = mpk.info()
    assert w == world and dist == (world & (world - 1) == 0 and (1 << data.log_n) >= world * world)
    pr = mpk.prove(_golden_solution(g), backend.with_amd_acceleration(), r=b(g["r"]), s=b(g["s"]))
    assert (pr.Ar.hex(), pr.Bs.hex(), pr.Krs.hex()) == (g["Ar"], g["Bs"], g["Krs"])
    # a second proof on the same key (barrier / buffers reused)
    pr2 = mpk.prove(_golden_solution(g), backend.with_amd_acceleration(), r=b(g["r"]), s=b(g["s"]))
    assert pr2 == pr
    t = mpk.last_timings()
    assert t["total"] >= t["shards"] > 0
    mpk.close()


@pytest.mark.parametrize("split", ["stripes", "wires"])
@pytest.mark.parametrize("log_n,n_wires,world,kidx", [(12, 3000, 4, False), (13, 7000, 8, True),
                                                      (12, 2500, 3, False), (14, 16000, 16, False)])
def test_mpk_vs_oracle(log_n, n_wires, world, kidx, split, monkeypatch):
    """split: wire slices (the default) or bucket stripes (GG_MPK_SPLIT=stripes,
    power-of-two worlds: whole wire tables per device, shard r takes the
    buckets b = r mod world); a world of 3 always slices wires."""
    from gnark_amd import backend, groth16
    monkeypatch.setenv("GG_MPK_SPLIT", split)
    from test_gpu_groth16 import synthetic_case
    d, wires, sa, sb, sc, ncons, r, s = synthetic_case(log_n, n_wires, 3, 40 + log_n + world, k_inf_every=5)
    if kidx:
        # K over a subset of the private wires (committed wires dropped, prove.go:238-248)
        nK = len(d["g1_K"]) // 64
        keep = np.arange(nK) % 7 != 3
        d["g1_K"] = np.frombuffer(d["g1_K"], np.uint8).reshape(-1, 64)[keep].tobytes()
        d["k_wire_index"] = (np.arange(nK, dtype=np.uint32) + 3)[keep]
    data = groth16.ProvingKeyData(**d)
    ref_pk = groth16.ProvingKey(data)
    sol = groth16.Solution(wires, sa, sb, sc, n_wires, ncons)
    ref = groth16.prove(ref_pk, sol, backend.with_amd_acceleration(), r=r, s=s)
    ref_pk.close()
    if not kidx:
        exp = coracle.groth16_prove(
            log_n, d["g1_A"], len(d["g1_A"]) // 64, d["g1_B"], len(d["g1_B"]) // 64, d["g1_Z"],
            d["g1_K"], len(d["g1_K"]) // 64, d["alpha1"], d["beta1"], d["delta1"], d["g2_B"],
            d["beta2"], d["delta2"], d["infinity_A"], d["infinity_B"], wires, n_wires, 3, sa, sb, sc,
            ncons, r, s)
        assert (ref.Ar, ref.Bs, ref.Krs) == exp[:3]
    mpk = groth16.MultiGpuProvingKey(data, [0] * world)
    assert mpk.split() == (split if world & (world - 1) == 0 else "wires")
    pr = mpk.prove(sol, backend.with_amd_acceleration(), r=r, s=s)
    assert pr == ref
    # the solution resident in HBM (one copy per device, gg_groth16_mpk_prove_ex)
    prd = mpk.prove(groth16.replicate_solution(sol, mpk.devices), backend.with_amd_acceleration(), r=r, s=s)
    assert prd == ref
    assert mpk.shard_devices() == [0] * world
    mpk.close()


def test_mpk_errors():
    from gnark_amd import GnarkAmdError, backend, groth16
    from test_gpu_groth16 import _pk_from_golden
    g = golden()["groth16"][1]
    data = _pk_from_golden(g)
    with pytest.raises(GnarkAmdError):
        groth16.MultiGpuProvingKey(data, [0, 4096])
    mpk = groth16.MultiGpuProvingKey(data, [0, 0])
    sol = _golden_solution(g)
    bad = groth16.Solution(sol.W[:-32], sol.A, sol.B, sol.C, sol.n_wires - 1, sol.n_constraints)
    with pytest.raises(GnarkAmdError):
        mpk.prove(bad, backend.with_amd_acceleration(), r=b(g["r"]), s=b(g["s"]))
    # the key still works after a rejected call
    pr = mpk.prove(sol, backend.with_amd_acceleration(), r=b(g["r"]), s=b(g["s"]))
    assert pr.Ar.hex() == g["Ar"]
    mpk.close()


def test_mpk_rehearsal_mode():
    """gg_groth16_mpk_set_rehearsal(r) (bench.py's split_projection): shard r
    proves alone -- the library returns GG_REHEARSAL (never GG_OK), prove()
    refuses that proof unless asked for a rehearsal, the proof is not the real
    one, and after set_rehearsal(-1) the same key is bit-exact again.  The
    per-shard timings report one prove time per shard and the three exchanges
    of the distributed computeH."""
    from gnark_amd import backend, groth16, GnarkAmdError
    from gnark_amd._lib import GG_REHEARSAL
    from test_gpu_groth16 import synthetic_case
    d, wires, sa, sb, sc, ncons, r, s = synthetic_case(12, 3000, 3, 77, k_inf_every=5)
    data = groth16.ProvingKeyData(**d)
    sol = groth16.Solution(wires, sa, sb, sc, 3000, ncons)
    mpk = groth16.MultiGpuProvingKey(data, [0] * 4)
    opt = backend.with_amd_acceleration()
    ref = mpk.prove(sol, opt, r=r, s=s)
    st = mpk.shard_timings()
    assert len(st) == 4
    for t in st:
        assert t["prove_ms"] > 0 and len(t["exchanges"]) == 3
        # pushes to the 3 peers: phase 1 sends 3 chunks, phase 2 two, phase 3 one
        mb = [e["pushed_MB"] for e in t["exchanges"]]
        assert mb[0] > mb[1] > mb[2] > 0 and abs(mb[0] - 3 * mb[2]) < 1e-9
    mpk.set_rehearsal(1)
    with pytest.raises(GnarkAmdError) as ei:
        mpk.prove(sol, opt, r=r, s=s)
    assert ei.value.code == GG_REHEARSAL
    solo = mpk.prove(sol, opt, r=r, s=s, rehearsal_ok=True)
    assert solo != ref
    st = mpk.shard_timings()
    assert st[1]["prove_ms"] > 0 and st[0]["prove_ms"] == 0
    assert all(e["pushed_MB"] == 0 for e in st[1]["exchanges"])
    mpk.set_rehearsal(-1)
    assert mpk.prove(sol, opt, r=r, s=s) == ref
    with pytest.raises(GnarkAmdError):
        mpk.set_rehearsal(4)  # out of range
    mpk.close()


def test_mpk_distinct_devices_peer_access():
    """Shards on distinct GPUs when the box has them (skipped on a one-GPU box):
    cross-device hipMemcpyPeerAsync, event waits and peer access run for real,
    the proof equals the golden one, and peer access is reported per pair
    (enabled or why not -- a failure stages through host memory silently)."""
    from gnark_amd import backend, groth16, device_count
    from test_gpu_groth16 import _pk_from_golden
    nd = device_count()
    if nd < 2:
        pytest.skip("one GPU visible")
    g = golden()["groth16"][1]
    world = 4 if nd >= 4 else 2
    devs = list(range(world))
    mpk = groth16.MultiGpuProvingKey(_pk_from_golden(g), devs)
    pa = mpk.peer_access()
    assert all(pa[i][i] == "same_device" for i in range(world))
    assert all(pa[i][j] in ("enabled", "unavailable", "enable_failed") for i in range(world) for j in range(world)
               if i != j)
    pr = mpk.prove(_golden_solution(g), backend.with_amd_acceleration(), r=b(g["r"]), s=b(g["s"]))
    assert (pr.Ar.hex(), pr.Bs.hex(), pr.Krs.hex()) == (g["Ar"], g["Bs"], g["Krs"])
    mpk.close()


def test_mpk_peer_access_same_device():
    """All shards on one GPU: every pair reports same_device."""
    from gnark_amd import groth16
    from test_gpu_groth16 import _pk_from_golden
    g = golden()["groth16"][0]
    mpk = groth16.MultiGpuProvingKey(_pk_from_golden(g), [0, 0])
    assert mpk.peer_access() == [["same_device"] * 2] * 2
    mpk.close()
