"""GPU sparse-R1CS (PlonK) solver (gg_scs_*, constraint/blueprint_scs.go:53-151,
evaluateLROSmallDomain system.go:221-264) against the oracle restatement
(oracle/scs_solver.py): wires and the L, R, O columns bit-exact on random
BLS12-381 and BN254 systems (new wires at xa / xb / xc, add and mul gates,
assertions, commitment rows), and the error cases (unsatisfied assertion,
division by zero, malformed levels)."""
import random

import pytest

import scs_solver as ss

BLS_R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
BN_R = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001


def _circuit(seed, mod, nbp=3, nbs=4, n=300, commit_every=0):
    rng = random.Random(seed)
    cons, flags, nw = ss.random_circuit(rng, mod, nbp, nbs, n, commit_every=commit_every)
    wit = [rng.randrange(mod) for _ in range(nbp + nbs)]
    cons = ss.fill_assertions(mod, cons, wit)
    return cons, flags, nw, wit


def test_oracle_scs_levels_and_solve():
    from gnark_amd import solver
    cons, flags, nw, wit = _circuit(1, BLS_R, commit_every=13)
    lv = ss.levels_of(7, cons)
    got = solver.compute_scs_levels(7, nw, [w for k in cons for w in k[:3]])
    assert [sorted(x) for x in got] == [sorted(x) for x in lv]
    W = ss.solve(BLS_R, nw, cons, wit, lv, flags)
    for k, f in zip(cons, flags):  # every non-commitment constraint holds
        if not f:
            xa, xb, xc, qL, qR, qO, qM, qC = k
            assert (qL * W[xa] + qR * W[xb] + qO * W[xc] + qM * W[xa] * W[xb] + qC) % BLS_R == 0


def _vals(b, mod):
    from gnark_amd import fr
    f = fr.bls_fr_unmont if mod == BLS_R else fr.fr_unmont
    b = bytes(b)
    return [f(b[i:i + 32]) for i in range(0, len(b), 32)]


@pytest.mark.gpu
@pytest.mark.parametrize("levels_only", [False, True])
@pytest.mark.parametrize("seed,curve,commit", [(1, "bls12-381", 0), (2, "bls12-381", 11), (3, "bn254", 0),
                                               (4, "bn254", 7)])
def test_gpu_scs_solver_random(seed, curve, commit, levels_only, monkeypatch):
    """Both schedules (strands: one launch per super-level; GG_SOLVER_LEVELS=1:
    one launch per r1cs.Levels level) bit-exact vs the oracle."""
    from gnark_amd import solver
    monkeypatch.setenv("GG_SOLVER_LEVELS", "1" if levels_only else "0")
    mod = BLS_R if curve == "bls12-381" else BN_R
    cons, flags, nw, wit = _circuit(seed, mod, commit_every=commit)
    lv = ss.levels_of(7, cons)
    W = ss.solve(mod, nw, cons, wit, lv, flags)
    L, R, O = ss.lro(W, cons, 3)
    sys_ = solver.SparseR1CS.from_constraints(3, 4, nw, cons, flags=flags, curve=curve)
    assert sys_.domain == len(L)
    for on_dev in (True, False):
        out = sys_.solve(wit, on_device=on_dev)
        gW, gL, gR, gO = (x.to_host() for x in out) if on_dev else out
        assert _vals(gW, mod) == W
        assert _vals(gL, mod) == L and _vals(gR, mod) == R and _vals(gO, mod) == O
    strands, launches, segs = sys_.schedule()
    assert strands == (not levels_only)
    assert launches <= len(lv) and (levels_only or segs >= 1)
    sys_.close()


@pytest.mark.gpu
def test_gpu_scs_solver_errors():
    from gnark_amd import solver, GnarkAmdError
    mod = BLS_R
    # assertion x0 - x1 = 0 fails for distinct inputs
    sys_ = solver.SparseR1CS.from_constraints(1, 1, 3, [(0, 1, 2, 1, 0, mod - 1, 0, 0), (0, 1, 0, 1, mod - 1, 0, 0, 0)])
    with pytest.raises(solver.UnsatisfiedConstraintError) as e:
        sys_.solve([5, 6])
    assert e.value.cid == 1
    W, *_ = sys_.solve([5, 5])
    assert _vals(W.to_host(), mod) == [5, 5, 5]
    # witness size enforced by the library (solver.go:71-76): short and long, C ABI directly
    import ctypes
    from gnark_amd import fr
    from gnark_amd._lib import check, lib, ptr
    bad = ctypes.c_int64()
    for vals in ([5], [5, 5, 5]):
        wb = b"".join(fr.bls_fr_mont(v) for v in vals)
        with pytest.raises(GnarkAmdError, match="invalid witness size"):
            check(lib.gg_scs_solve(sys_.handle, ptr(wb), len(vals), 0, None, None, None, None, 0,
                                   ctypes.byref(bad)))
    sys_.close()
    # the new wire at xa with qL + qM xb = 0: errDivideByZero
    sys_ = solver.SparseR1CS.from_constraints(1, 1, 3, [(2, 1, 0, 0, 1, 1, 0, 0)])
    with pytest.raises(solver.UnsatisfiedConstraintError) as e:
        sys_.solve([5, 6])
    assert e.value.cid == 0
    sys_.close()
    # two unknowns in one constraint: the levels do not match the system
    sys_ = solver.SparseR1CS.from_constraints(1, 0, 3, [(1, 2, 0, 1, 1, 0, 0, 0)], levels=[[0]])
    with pytest.raises(GnarkAmdError):
        sys_.solve([5])
    sys_.close()


def scs_mimc(nb_chains, rounds, mod):
    """MiMC-style chains as sparse R1CS (std/hash/mimc encryptPow5 through
    frontend/cs/scs: a = x + k_r (add gate), b = a a, c = b b, x' = c a), four
    constraints per round, chain-major constraint ids; the witness is x0 of
    every chain (secret).  Returns (wires, qidx, table, levels, n_wires) with
    r1cs.Levels = the 4 rounds positions (4 * rounds levels of nb_chains)."""
    import numpy as np
    K, R = nb_chains, rounds
    rng = random.Random(77)
    ks = [rng.randrange(mod) for _ in range(R)]
    table = [0, 1, mod - 1] + ks  # 0, 1, -1, round constants
    c = np.arange(K * R * 4, dtype=np.int64).reshape(K, R, 4)
    new = K + c  # the wire each constraint introduces
    x = np.empty((K, R), dtype=np.int64)  # round input wire
    x[:, 0] = np.arange(K)
    x[:, 1:] = new[:, :-1, 3]
    a, b, cc = new[..., 0], new[..., 1], new[..., 2]
    wires = np.stack([np.stack([x, x, a], -1), np.stack([a, a, b], -1), np.stack([b, b, cc], -1),
                      np.stack([cc, a, new[..., 3]], -1)], 2)  # K, R, 4, 3
    q = np.zeros((K, R, 4, 5), dtype=np.int64)  # qL, qR, qO, qM, qC (table ids)
    q[:, :, 0, 0] = 1
    q[:, :, 0, 2] = 2
    q[:, :, 0, 4] = 3 + np.arange(R)[None, :]
    q[:, :, 1:, 2] = 2
    q[:, :, 1:, 3] = 1
    levels = [c[:, r, i].reshape(-1) for r in range(R) for i in range(4)]
    return wires.reshape(-1), q.reshape(-1), table, levels, K + K * R * 4, ks


@pytest.mark.gpu
@pytest.mark.parametrize("log_n", [12, 22])
def test_gpu_scs_solver_strands_mimc(log_n, monkeypatch):
    """configs[4]-sized sparse R1CS (2^22 constraints: 16,384 MiMC chains of 64
    rounds, 256 levels): the strand schedule solves it in ONE launch and agrees
    byte for byte with the 256 level launches; sampled chains match a big-int
    restatement of the rounds."""
    from gnark_amd import fr, solver
    mod = BLS_R
    K = 1 << (log_n - 8)
    wires, qidx, table, levels, nw, ks = scs_mimc(K, 64, mod)
    rng = random.Random(log_n)
    wit = [rng.randrange(mod) for _ in range(K)]
    out = {}
    for lv_only in (True, False):
        monkeypatch.setenv("GG_SOLVER_LEVELS", "1" if lv_only else "0")
        sys_ = solver.SparseR1CS(0, K, nw, wires, qidx, table, levels=levels, curve="bls12-381")
        assert sys_.domain == 1 << log_n
        W, L, Rv, O = sys_.solve(wit, on_device=False)
        out[lv_only] = (bytes(W), bytes(L), bytes(Rv), bytes(O))
        strands, launches, segs = sys_.schedule()
        assert (strands, launches) == ((False, 256) if lv_only else (True, 1))
        if not lv_only:
            assert segs == K
        sys_.close()
    assert out[True] == out[False]
    W = out[False][0]
    for j in rng.sample(range(K), min(K, 16)):
        x = wit[j]
        for r in range(64):
            a = (x + ks[r]) % mod
            x = pow(a, 5, mod)
        last = K + ((j * 64 + 63) * 4 + 3)
        assert fr.bls_fr_unmont(W[32 * last:32 * last + 32]) == x


class _ScsCircuit:
    """A sparse R1CS laid out as gnark's BuildTrace does (setup.go:173-220):
    public placeholder rows (-x + qk = 0, qk completed by the prover), the
    constraints, padding rows; every unused slot is wire 0, matching
    evaluateLROSmallDomain's solution[0] padding.  Provides what
    plonk_circuits.make_key reads (selectors, permutation, S polynomials)."""

    def __init__(self, cons, nb_public, n_wires):
        import numpy as np
        from plonk_circuits import Circuit, FIELDS
        self._C = Circuit
        self.F, self.curve = FIELDS["bls12-381"], "bls12-381"
        n = 1
        while n < len(cons) + nb_public:
            n <<= 1
        self.n, self.log_n = n, n.bit_length() - 1
        self.nb_public, self.n_cmt, self.cmt_idx, self.committed = nb_public, 0, [], []
        self.nvar, self.cons = n_wires, cons
        self.a, self.b, self.c = (np.zeros(n, np.int64) for _ in range(3))
        self.a[:nb_public] = np.arange(nb_public)
        for j, k in enumerate(cons):
            self.a[nb_public + j], self.b[nb_public + j], self.c[nb_public + j] = k[0], k[1], k[2]

    def selectors(self):
        from plonk_circuits import m2b
        MONT, NEG_ONE_M = self.F.MONT, self.F.NEG_ONE_M
        cols = [bytearray(32 * self.n) for _ in range(5)]  # ql, qr, qm, qo, qk
        for i in range(self.nb_public):
            cols[0][32 * i:32 * i + 32] = m2b(NEG_ONE_M)
        for j, (xa, xb, xc, qL, qR, qO, qM, qC) in enumerate(self.cons):
            r = self.nb_public + j
            for col, q in zip(cols, (qL, qR, qM, qO, qC)):
                col[32 * r:32 * r + 32] = m2b(q % BLS_R * MONT % BLS_R)
        return [bytes(c) for c in cols], []

    def permutation(self):
        return self._C.permutation(self)

    def s_polys(self, perm, omega, u):
        return self._C.s_polys(self, perm, omega, u)


@pytest.mark.gpu
def test_gpu_scs_solve_feeds_plonk_prove():
    """spr.Solve on the GPU -> L, R, O in HBM -> gg_plonk_prove -> the restated
    verifier accepts; a wrong public input is rejected."""
    import bls12_381_oracle as blo
    from gnark_amd import plonk_prover as pp, solver
    from plonk_circuits import make_key, to_oracle
    rng = random.Random(21)
    nbp, nbs = 2, 3
    cons, flags, nw = ss.random_circuit(rng, BLS_R, nbp, nbs, 100)
    wit = [rng.randrange(BLS_R) for _ in range(nbp + nbs)]
    cons = ss.fill_assertions(BLS_R, cons, wit)
    circ = _ScsCircuit(cons, nbp, nw)
    tau = 987654321
    pk = make_key(circ, tau)
    sys_ = solver.SparseR1CS.from_constraints(nbp, nbs, nw, cons, curve="bls12-381")
    assert sys_.domain == circ.n
    W, L, Rv, O = sys_.solve(wit)  # DeviceBuffers
    pub = wit[:nbp]
    proof = pp.prove(pk, L, Rv, O, rng=random.Random(5), public=pub)
    pr, vk = to_oracle(pk, proof)
    assert blo.plonk_verify_trapdoor(pr, vk, tau, public=pub)
    assert not blo.plonk_verify_trapdoor(pr, vk, tau, public=[pub[0] + 1, pub[1]])
    sys_.close()
    pk.close()
