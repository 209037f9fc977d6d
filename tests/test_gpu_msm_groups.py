"""The precompute-group memory knob (DESIGN.md "MSM", gg_msm_base_layout): a
base stores only every G-th window shift, window G w' + j adds into bucket
group j, and the group sums are recombined by 2^(j c) -- so a key needs
ceil(W / G) point copies instead of W.  Every G stays bit-exact: G1 / G2 /
BLS12-381 MSMs vs the C oracle and the trapdoor identity, the golden Groth16
proofs, and a satisfied MiMC instance, with G forced by GG_MSM_GROUPS or
chosen by the library from gg_set_hbm_budget (the path a key that does not fit
takes: nbConstraints > 2^24 doubles the domain)."""
import pytest

import bn254_oracle as o
import coracle
from helpers import b, golden, random_fr_mont, random_g1_points

pytestmark = pytest.mark.gpu


def _check_layout(base, groups, n, pt_bytes):
    _, c, W = base.info()
    g, ws, nbytes = base.layout()
    assert g == groups and ws == -(-W // groups) and nbytes == ws * n * pt_bytes
    return W


@pytest.mark.parametrize("groups", [2, 4, 16])
@pytest.mark.parametrize("n,dist,c", [(4096, "uniform", 11), (4096, "witness", 6), (1 << 16, "witness", 20),
                                      (1000, "uniform", 0)])
def test_msm_g1_groups_vs_oracle(groups, n, dist, c, monkeypatch):
    from gnark_amd import msm
    monkeypatch.setenv("GG_MSM_GROUPS", str(groups))
    pts = random_g1_points(n, 31000 + n)
    sc = random_fr_mont(n, 32000 + n, dist)
    base = msm.MsmBase(msm.G1, pts, n, window_bits=c)
    W = base.info()[2]
    _check_layout(base, min(groups, 1 << (W.bit_length() - 1)), n, 64)
    assert base.msm(sc, n) == coracle.msm_g1(pts.tobytes(), sc.tobytes(), n)
    base.close()


def test_msm_g2_groups_trapdoor(monkeypatch):
    """G2 at the headline's window (c = 20, 13 windows): 7 stored copies with G = 2."""
    from gnark_amd import msm
    monkeypatch.setenv("GG_MSM_GROUPS", "2")
    n = 1 << 16
    ks = random_fr_mont(n, 33001)
    ss = random_fr_mont(n, 33002, "witness")
    pts = coracle.g2_batch_mul(o.g2_to_bytes(o.G2_GEN), ks.tobytes(), n)
    base = msm.MsmBase(msm.G2, bytes(pts), n, window_bits=20)
    assert _check_layout(base, 2, n, 128) == 13
    e = coracle.fr_dot(ks, ss, n)
    assert base.msm(ss, n) == bytes(coracle.g2_batch_mul(o.g2_to_bytes(o.G2_GEN), e, 1))
    base.close()


@pytest.mark.parametrize("groups", [2, 8])
def test_msm_bls_groups_trapdoor(groups, monkeypatch):
    import bls12_381_oracle as bl
    from gnark_amd import msm
    from test_gpu_bls import _points, _scalars
    monkeypatch.setenv("GG_MSM_GROUPS", str(groups))
    n = 4096
    pts, ks = _points(n, 34000 + groups, 7)
    sv, sb = _scalars(n, 35000 + groups, "uniform")
    base = msm.MsmBase(msm.BLS12_381_G1, pts, n, window_bits=13)
    assert base.layout()[0] == groups
    assert base.msm(sb, n) == bl.g1_to_bytes(bl.msm_g1_trapdoor(ks, sv))
    base.close()


def _golden_prove(idx):
    from gnark_amd import backend, groth16
    from test_gpu_groth16 import _pk_from_golden
    g = golden()["groth16"][idx]
    pk = groth16.ProvingKey(_pk_from_golden(g))
    nw = len(b(g["infA"]))
    ncons = len(b(g["solA"])) // 32
    sol = groth16.Solution(b(g["wires"]), b(g["solA"]), b(g["solB"]), b(g["solC"]), nw, ncons)
    pr = groth16.prove(pk, sol, backend.with_amd_acceleration(), r=b(g["r"]), s=b(g["s"]))
    assert (pr.Ar.hex(), pr.Bs.hex(), pr.Krs.hex()) == (g["Ar"], g["Bs"], g["Krs"])
    return pk


@pytest.mark.parametrize("idx", [0, 1])
def test_groth16_golden_budget_driven_groups(idx, monkeypatch):
    """A budget below the key's G = 1 tables: the library picks G > 1 for every
    base of the key (one value: A/K and B1/G2 keep their shared sorts) and the
    golden proofs stay bit-exact; the budget reset gives G = 1 again."""
    from gnark_amd import msm
    monkeypatch.delenv("GG_MSM_GROUPS", raising=False)
    try:
        msm.set_hbm_budget(1)
        assert msm.get_hbm_budget() == 1
        pk = _golden_prove(idx)
        gs = {pk.base_layout(w)[0] for w in range(5)}
        assert len(gs) == 1 and gs.pop() > 1
        pk.close()
    finally:
        msm.set_hbm_budget(0)
    pk = _golden_prove(idx)
    assert {pk.base_layout(w)[0] for w in range(5)} == {1}
    pk.close()


@pytest.mark.parametrize("log_n,groups", [(12, 4), (18, 2)])
def test_groth16_mimc_groups_bit_exact(log_n, groups, monkeypatch):
    """A satisfied MiMC R1CS (configs[3] shape) proved from a key with G
    precompute groups: bit-exact vs the proof scalars from the toxic waste, and
    the key's tables shrink to ceil(W / G) copies."""
    import time
    from gnark_amd import backend, groth16
    from test_gpu_groth16_size import _instance, _fr, R_, S_
    monkeypatch.setenv("GG_MSM_GROUPS", str(groups))
    cr, data, wires, (A, B, C), want = _instance(log_n, time.time())
    pk = groth16.ProvingKey(data)
    for w in range(5):
        g, ws, nbytes = pk.base_layout(w)
        W = pk.base_info(w)[2]
        assert g == groups and ws == -(-W // groups)
    sol = groth16.Solution(bytes(wires), bytes(A), bytes(B), bytes(C), cr.nw, cr.ncons)
    pr = groth16.prove(pk, sol, backend.with_amd_acceleration(), r=_fr(R_), s=_fr(S_))
    assert (pr.Ar, pr.Bs, pr.Krs) == want
    pk.close()
