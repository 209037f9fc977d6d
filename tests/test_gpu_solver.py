"""GPU R1CS solver (gg_r1cs_*, constraint/bn254/solver.go:418-608) against the
oracle restatement (oracle/r1cs_solver.py): wires and the solution vectors
A, B, C bit-exact on the cubic circuit (examples/cubic), random circuits with
the unknown on every side (divisions, coefficients, zero divisors), the MiMC
chain shape up to the 2^24 headline (vs the C oracle's solver), error
behaviour (unsatisfied constraint, malformed levels), and a Groth16 proof from
the device-resident solution identical to one from host inputs."""
import random

import numpy as np
import pytest

import bn254_oracle as o
import r1cs_solver as rs

# ---------------------------------------------------------------- CPU
def test_oracle_solver_cubic_and_mimc():
    rcs = o.cubic_r1cs()
    lv = rs.levels_of(rcs.nb_public + rcs.nb_secret, rcs.constraints)
    W, A, B, C = rs.solve(rcs.nb_wires, 3, rcs.constraints, [35, 3], lv)
    assert W == o.cubic_witness()
    assert (A, B, C) == tuple(rcs.solution(W))
    with pytest.raises(rs.Unsatisfied) as e:
        rs.solve(rcs.nb_wires, 3, rcs.constraints, [34, 3], lv)
    assert e.value.cid == 2
    m = o.mimc_chain_r1cs(3, 5)
    lvm = rs.levels_of(1 + 3, m.constraints)
    assert len(lvm) == 15 and all(len(x) == 3 for x in lvm)
    Wm, *_ = rs.solve(m.nb_wires, 4, m.constraints, [7, 8, 9], lvm)
    assert Wm == o.mimc_chain_witness(m, [7, 8, 9])


def test_mirror_levels_match_oracle():
    from gnark_amd import solver
    rng = random.Random(5)
    cons = rs.random_circuit(rng, 2, 3, 60)
    off, wires = [0], []
    for side3 in cons:
        for side in side3:
            wires += [w for w, _ in side]
            off.append(len(wires))
    got = solver.compute_levels(5, 65, off, wires)
    assert [sorted(x) for x in got] == [sorted(x) for x in rs.levels_of(5, cons)]


# ---------------------------------------------------------------- GPU
def _fr_list(b):
    return o.fr_vec_from_bytes(bytes(b))


def _host(sol):
    if sol.on_device:
        return [x.to_host() for x in (sol.W, sol.A, sol.B, sol.C)]
    return [bytes(x) for x in (sol.W, sol.A, sol.B, sol.C)]


@pytest.mark.gpu
def test_gpu_solver_cubic():
    from gnark_amd import solver
    rcs = o.cubic_r1cs()
    sys_ = solver.R1CS.from_terms(rcs.nb_public, rcs.nb_secret, rcs.nb_wires, rcs.constraints)
    assert sys_.info() == (5, 3, len(sys_.levels))
    for on_dev in (True, False):
        W, A, B, C = _host(sys_.solve([35, 3], on_device=on_dev))
        w = o.cubic_witness()
        assert _fr_list(W) == w
        ra, rb, rc = rcs.solution(w)
        assert (_fr_list(A), _fr_list(B), _fr_list(C)) == (ra, rb, rc)
    with pytest.raises(solver.UnsatisfiedConstraintError) as e:
        sys_.solve([34, 3])
    assert e.value.cid == 2
    with pytest.raises(ValueError):
        sys_.solve([35])  # invalid witness size (solver.go:72-76)
    # the library enforces it too (a cgo caller has no Python check): a short and
    # a long witness through the C ABI directly
    import ctypes
    from gnark_amd import GnarkAmdError, fr
    from gnark_amd._lib import check, lib, ptr
    bad = ctypes.c_int64()
    for vals in ([35], [35, 3, 9]):
        wb = b"".join(fr.fr_mont(v) for v in vals)
        with pytest.raises(GnarkAmdError, match="invalid witness size"):
            check(lib.gg_r1cs_solve(sys_.handle, ptr(wb), len(vals), 0, None, None, None, None, 0,
                                    ctypes.byref(bad)))
    sys_.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,zero", [(1, False), (2, False), (3, True), (4, True)])
def test_gpu_solver_random_circuits(seed, zero):
    from gnark_amd import solver
    rng = random.Random(seed)
    nbp, nbs, nint = 3, 4, 300
    cons = rs.random_circuit(rng, nbp, nbs, nint, zero_divisor=zero)
    nw = nbp + nbs + nint
    lv = rs.levels_of(nbp + nbs, cons)
    wit = [rng.randrange(o.R) for _ in range(nbp - 1 + nbs)]
    W, A, B, C = rs.solve(nw, nbp + nbs, cons, wit, lv)
    sys_ = solver.R1CS.from_terms(nbp, nbs, nw, cons)
    gW, gA, gB, gC = _host(sys_.solve(wit))
    assert _fr_list(gW) == W
    assert _fr_list(gA) == A and _fr_list(gB) == B and _fr_list(gC) == C
    sys_.close()


@pytest.mark.gpu
def test_gpu_solver_rejects_bad_levels():
    from gnark_amd import solver, GnarkAmdError
    rcs = o.mimc_chain_r1cs(2, 2)
    n = len(rcs.constraints)
    # every constraint in one level: later rounds see two unsolved wires
    sys_ = solver.R1CS.from_terms(rcs.nb_public, rcs.nb_secret, rcs.nb_wires, rcs.constraints,
                                  levels=[list(range(n))])
    with pytest.raises(GnarkAmdError):
        sys_.solve([5, 6])
    sys_.close()
    with pytest.raises(GnarkAmdError):  # a constraint missing from the levels
        solver.R1CS.from_terms(rcs.nb_public, rcs.nb_secret, rcs.nb_wires, rcs.constraints,
                               levels=[list(range(n - 1))])


def mimc_csr(nb_chains, rounds, nb_public_inputs):
    """The C oracle's MiMC R1CS (oracle/c/oracle_r1cs.c) as CSR + levels, vectorized."""
    ncons = 3 * nb_chains * rounds
    ch = np.repeat(np.arange(nb_chains, dtype=np.int64), rounds)
    rd = np.tile(np.arange(rounds, dtype=np.int64), nb_chains)
    base = 1 + nb_chains + 3 * (ch * rounds + rd)          # t of round (ch, rd)
    x = np.where(rd == 0, 1 + ch, base - 1)                # the round's input x
    t, u, xn = base, base + 1, base + 2
    # per round: L, R, O of 3 constraints -> terms (O of the third has 2 terms)
    nper = 3 + 3 + 3 + 1
    wires = np.empty((nb_chains * rounds, nper), dtype=np.uint32)
    coef = np.zeros((nb_chains * rounds, nper), dtype=np.uint32)
    wires[:, 0], wires[:, 1], wires[:, 2] = x, x, t
    wires[:, 3], wires[:, 4], wires[:, 5] = t, t, u
    wires[:, 6], wires[:, 7], wires[:, 8], wires[:, 9] = u, x, xn, 0
    coef[:, 9] = 1 + rd  # coefficient index of -(7 rd + 3)
    counts = np.tile(np.array([1, 1, 1, 1, 1, 1, 1, 1, 2], dtype=np.int64), nb_chains * rounds)
    off = np.zeros(3 * ncons + 1, dtype=np.uint32)
    off[1:] = np.cumsum(counts)
    table = [1] + [(-(r * 7 + 3)) % o.R for r in range(rounds)]
    # levels: constraint 3 (ch rounds + rd) + k sits at level 3 rd + k
    cid = np.arange(ncons, dtype=np.int64)
    lvl = 3 * ((cid // 3) % rounds) + cid % 3
    order = np.argsort(lvl, kind="stable")
    levels = np.split(order.astype(np.uint32), np.cumsum(np.bincount(lvl))[:-1])
    return dict(off=off, wires=wires.reshape(-1), coef=coef.reshape(-1), table=table, levels=levels,
                nw=1 + nb_chains + ncons, ncons=ncons, nb_public=1 + nb_public_inputs,
                nb_secret=nb_chains - nb_public_inputs)


@pytest.mark.gpu
@pytest.mark.parametrize("log_n", [12, 20, 24])
def test_gpu_solver_mimc_vs_c_oracle(log_n):
    import coracle
    from gnark_amd import solver
    from helpers import random_fr_mont
    rounds = 85  # bench.py's MIMC_ROUNDS: 2^(log_n - 8) chains (the headline shape at 2^24)
    chains = 1 << (log_n - 8)
    m = mimc_csr(chains, rounds, 1)
    sys_ = solver.R1CS(m["nb_public"], m["nb_secret"], m["nw"], m["off"], m["wires"], m["coef"], m["table"],
                       levels=m["levels"])
    inputs = random_fr_mont(chains, seed=log_n).tobytes()
    ref = coracle.MimcR1CS(chains, rounds, 1)
    wref = ref.solve(inputs)
    A, B, C, bad = ref.abc(wref)
    assert bad == 0
    sol = sys_.solve(inputs)
    gW, gA, gB, gC = _host(sol)
    assert gW == bytes(wref)
    assert gA == bytes(A) and gB == bytes(B) and gC == bytes(C)
    sys_.close()
    ref.close()


@pytest.mark.gpu
def test_gpu_solver_feeds_groth16_bit_exact():
    """solve on the GPU -> prove from the HBM-resident solution: the same proof as
    from host inputs (the cubic golden key, fixed r, s)."""
    from gnark_amd import backend, groth16, solver
    from helpers import b, golden
    g = golden()["groth16"][0]
    pk = groth16.ProvingKey(groth16.ProvingKeyData(
        log_n=g["log_n"], g1_A=b(g["g1_A"]), g1_B=b(g["g1_B"]), g1_Z=b(g["g1_Z"]),
        g1_K=b(g["g1_K"]), alpha1=b(g["alpha1"]), beta1=b(g["beta1"]), delta1=b(g["delta1"]),
        g2_B=b(g["g2_B"]), beta2=b(g["beta2"]), delta2=b(g["delta2"]),
        infinity_A=b(g["infA"]), infinity_B=b(g["infB"]), nb_public=g["nb_public"]))
    rcs = o.cubic_r1cs()
    sys_ = solver.R1CS.from_terms(rcs.nb_public, rcs.nb_secret, rcs.nb_wires, rcs.constraints)
    sol = sys_.solve([35, 3])
    opt = backend.with_amd_acceleration()
    pr = groth16.prove(pk, sol, opt, r=b(g["r"]), s=b(g["s"]))
    assert (pr.Ar.hex(), pr.Bs.hex(), pr.Krs.hex()) == (g["Ar"], g["Bs"], g["Krs"])
    sys_.close()
    pk.close()


@pytest.mark.gpu
@pytest.mark.parametrize("levels_only", [False, True])
def test_gpu_solver_strand_and_level_schedules_agree(levels_only, monkeypatch):
    """The strand schedule (one launch per super-level, a thread per chain
    segment) and the plain level launches (GG_SOLVER_LEVELS=1) give the same
    bit-exact solution (MiMC 2^12 shape and a random circuit)."""
    import coracle
    from gnark_amd import solver
    from helpers import random_fr_mont
    monkeypatch.setenv("GG_SOLVER_LEVELS", "1" if levels_only else "0")
    m = mimc_csr(16, 85, 1)
    sys_ = solver.R1CS(m["nb_public"], m["nb_secret"], m["nw"], m["off"], m["wires"], m["coef"], m["table"],
                       levels=m["levels"])
    inputs = random_fr_mont(16, seed=3).tobytes()
    ref = coracle.MimcR1CS(16, 85, 1)
    wref = ref.solve(inputs)
    assert _host(sys_.solve(inputs))[0] == bytes(wref)
    sys_.close()
    ref.close()
    rng = random.Random(9)
    cons = rs.random_circuit(rng, 2, 3, 200, zero_divisor=True)
    wit = [rng.randrange(o.R) for _ in range(4)]
    W, A, B, C = rs.solve(205, 5, cons, wit, rs.levels_of(5, cons))
    sys_ = solver.R1CS.from_terms(2, 3, 205, cons)
    gW, gA, gB, gC = _host(sys_.solve(wit))
    assert _fr_list(gW) == W and _fr_list(gC) == C
    sys_.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,zero", [(5, False), (6, True)])
def test_gpu_solver_bls12_381(seed, zero):
    """gg_r1cs_create_ex(GG_CURVE_BLS12_381): backend/groth16/bls12-381's solver
    (constraint/bls12-381/solver.go), bit-exact vs the oracle over r_BLS."""
    from gnark_amd import fr, solver
    Rb = fr.BLS_R
    rng = random.Random(seed)
    cons = rs.random_circuit(rng, 3, 4, 300, zero_divisor=zero, R=Rb)
    wit = [rng.randrange(Rb) for _ in range(6)]
    W, A, B, C = rs.solve(307, 7, cons, wit, rs.levels_of(7, cons), R=Rb)
    sys_ = solver.R1CS.from_terms(3, 4, 307, cons, curve="bls12-381")
    gW, gA, gB, gC = _host(sys_.solve(wit))
    vals = lambda b: [fr.bls_fr_unmont(bytes(b)[i:i + 32]) for i in range(0, len(b), 32)]
    assert vals(gW) == W and vals(gA) == A and vals(gB) == B and vals(gC) == C
    sys_.close()
