"""Synthetic sparse-R1CS circuits for the PlonK tests (BASELINE configs[4] shape):
the trace layout of backend/plonk/bls12-381/setup.go BuildTrace (:173-220) --
public-input placeholder rows (-x + qk = 0, qk completed by the prover), then the
constraints -- with the BSB22 commitment rows of frontend/cs/scs/api.go:623-655
(one "-v + Pi = 0" row per committed value, qcp = 1 there, and the commitment
row "-c + qk = 0" whose qk the prover injects), and a solver that runs the
bsb22Hint (prove.go:316-352) through the device key.

Values are kept in Montgomery form (m = x 2^256 mod r) so the 2^22 solve stays
a cheap Python loop; the permutation is built with numpy (cycles over the slots
of each variable, setup.go:323-376 semantics).
"""
import random

import numpy as np

import bls12_381_oracle as bo
import plonk_prover_oracle as po

R = bo.R
MONT = (1 << 256) % R
MINV = pow(1 << 256, -1, R)
ONE_M = MONT
NEG_ONE_M = (R - 1) * MONT % R

K_PUB, K_ADD, K_MUL, K_CMTD, K_CMT = 0, 1, 2, 3, 4


class Field:
    """Scalar field (Montgomery constants) and G1 encodings of a PlonK curve."""

    def __init__(self, curve="bls12-381"):
        self.curve = curve
        self.cv = po.curve(curve)
        self.R = R_ = self.cv.R
        self.MONT = (1 << 256) % R_
        self.MINV = pow(1 << 256, -1, R_)
        self.ONE_M, self.NEG_ONE_M = self.MONT, (R_ - 1) * self.MONT % R_
        if curve == "bls12-381":
            self.g1_from_bytes, self.g1_to_bytes, self.pt = bo.g1_from_bytes, bo.g1_to_bytes, 96
        else:
            import bn254_oracle as bn
            self.g1_from_bytes, self.g1_to_bytes, self.pt = bn.g1_from_bytes, bn.g1_to_bytes, 64


FIELDS = {c: Field(c) for c in ("bls12-381", "bn254")}


def m2b(v):  # Montgomery int -> 32 B
    return v.to_bytes(32, "little")


class Circuit:
    """Rows of a sparse R1CS over n = 2^log_n slots (no padding rows).  a/b/c:
    variable ids of the L/R/O slots (-1 = unused), kind: row type."""

    def __init__(self, log_n, seed, nb_public=0, n_cmt=0, committed_per=3, curve="bls12-381"):
        self.F = FIELDS[curve]
        self.curve = curve
        self.log_n, self.n = log_n, 1 << log_n
        n = self.n
        self.nb_public, self.n_cmt = nb_public, n_cmt
        rnd = np.random.default_rng(seed)
        self.kind = np.full(n, K_ADD, np.int8)
        self.a = np.full(n, -1, np.int64)
        self.b = np.full(n, -1, np.int64)
        self.c = np.full(n, -1, np.int64)
        self.nvar = 0

        def new():
            self.nvar += 1
            return self.nvar - 1
        row = 0
        self.pub_vars = []
        for _ in range(nb_public):
            v = new()
            self.kind[row], self.a[row] = K_PUB, v
            self.pub_vars.append(v)
            row += 1
        # a first stretch of gates so there is something to commit to
        body = rnd.random(n) < 0.5
        prev = new()  # a secret input
        self.secret_first = prev
        first_gate = row

        def gate(r, a_var, b_var):
            self.kind[r] = K_MUL if body[r] else K_ADD
            self.a[r], self.b[r] = a_var, b_var
            self.c[r] = new()
            return self.c[r]
        pre = max(8, (n - nb_public - n_cmt * (committed_per + 1)) // 4)
        for _ in range(pre):
            b_var = self.pub_vars[row % nb_public] if (nb_public and row % 5 == 2) else new()
            prev = gate(row, prev, b_var)
            row += 1
        self.cmt_idx, self.committed = [], []
        cmt_vars = []
        for j in range(n_cmt):
            rows = []
            for k in range(committed_per):
                v = int(self.c[first_gate + 3 * k + j])  # an earlier gate output
                self.kind[row], self.a[row] = K_CMTD, v
                rows.append(row)
                row += 1
            cv = new()
            self.kind[row], self.a[row] = K_CMT, cv
            self.cmt_idx.append(row - nb_public)
            self.committed.append(rows)
            cmt_vars.append(cv)
            row += 1
        # the rest; the commitment outputs and public inputs are used again
        while row < n:
            if cmt_vars and row % 7 == 3:
                b_var = cmt_vars[row % len(cmt_vars)]
            elif nb_public and row % 5 == 2:
                b_var = self.pub_vars[row % nb_public]
            elif row % 4 == 3:
                b_var = self.secret_first
            else:
                b_var = new()
            prev = gate(row, prev, b_var)
            row += 1
        assert self.kind[n - 1] in (K_ADD, K_MUL)  # last row: qcp = 0 (bsb22Hint blinds it)
        self.cmt_vars = cmt_vars

    # ---------------------------------------------------------------- key inputs
    def selectors(self):
        """ql, qr, qm, qo, qk (incomplete) and qcp_j, Lagrange regular (bytes)."""
        n, k = self.n, self.kind
        tab = np.array([[b for b in m2b(x)] for x in (0, self.F.ONE_M, self.F.NEG_ONE_M)], np.uint8)

        def col(idx):
            return tab[idx].tobytes()
        z = np.zeros(n, np.int64)
        ql = np.where((k == K_PUB) | (k == K_CMTD) | (k == K_CMT), 2, np.where(k == K_ADD, 1, 0))
        qr = np.where(k == K_ADD, 1, 0)
        qm = np.where(k == K_MUL, 1, 0)
        qo = np.where((k == K_ADD) | (k == K_MUL), 2, 0)
        qcp = []
        for rows in self.committed:
            q = z.copy()
            q[rows] = 1
            qcp.append(col(q))
        return [col(ql), col(qr), col(qm), col(qo), col(z)], qcp

    def permutation(self):
        """pk.trace.S: 3n slots, cycles over the slots of each variable."""
        n = self.n
        var = np.concatenate([self.a, self.b, self.c])
        free = var < 0
        var[free] = self.nvar + np.arange(int(free.sum()))  # unused slots: fixed points
        order = np.argsort(var, kind="stable")
        sv = var[order]
        p = np.arange(3 * n)
        start = np.r_[True, sv[1:] != sv[:-1]]
        last = np.r_[sv[1:] != sv[:-1], True]
        gs = np.maximum.accumulate(np.where(start, p, 0))
        nxt = np.where(last, gs, p + 1)
        perm = np.empty(3 * n, np.int64)
        perm[order] = order[nxt]
        return perm

    def s_polys(self, perm, omega, u):
        """S1, S2, S3 in Lagrange form: ID(perm[j n + i]), ID(s) = u^(s div n) w^(s mod n)
        (getSupportPermutation, setup.go:391-407), gathered from a 3n-entry table."""
        n = self.n
        R, MONT = self.F.R, self.F.MONT
        tab = bytearray(32 * 3 * n)
        for blk, shift in enumerate((1, u, u * u % R)):
            x = shift * MONT % R
            o = 32 * blk * n
            for i in range(n):
                tab[o + 32 * i:o + 32 * i + 32] = m2b(x)
                x = x * omega % R
        t = np.frombuffer(bytes(tab), np.uint8).reshape(3 * n, 32)
        return [t[perm[j * n:(j + 1) * n]].tobytes() for j in range(3)]

    # ---------------------------------------------------------------- solver
    def solve(self, pk, seed, public=None, commit=None, hint_rng=None):
        """L, R, O (Montgomery bytes), the public witness (ints) and the BSB22
        commitment data (values, digest, hashed) of each commitment, running the
        bsb22Hint through `commit` (kzg.Commit on pk.KzgLagrange)."""
        n = self.n
        F = self.F
        R, MONT, MINV = F.R, F.MONT, F.MINV
        rnd = random.Random(seed)
        hint_rng = hint_rng or random.Random(seed + 1)
        val = [None] * self.nvar
        public = public if public is not None else [rnd.randrange(R) for _ in range(self.nb_public)]
        for v, x in zip(self.pub_vars, public):
            val[v] = x % R * MONT % R

        def get(v):
            if val[v] is None:
                val[v] = rnd.randrange(R)  # a free secret (Montgomery form of a random value)
            return val[v]
        L, Rv, O = bytearray(32 * n), bytearray(32 * n), bytearray(32 * n)
        cmts = []
        kind, a, b, c = self.kind.tolist(), self.a.tolist(), self.b.tolist(), self.c.tolist()
        ci = 0
        for r in range(n):
            k = kind[r]
            if k == K_CMT:
                # bsb22Hint: committed values at their rows, random at the commitment
                # row and at the last constraint (prove.go:326-334)
                vals = bytearray(32 * n)
                for rr in self.committed[ci]:
                    vals[32 * rr:32 * rr + 32] = m2b(val[a[rr]])
                for rr in (r, n - 1):
                    vals[32 * rr:32 * rr + 32] = m2b(hint_rng.randrange(R))
                dig = commit(bytes(vals))
                # htfFunc.Write(commitment.Marshal()) (prove.go:341): the uncompressed encoding
                hv = F.cv.hash_to_field(F.cv.raw(F.g1_from_bytes(dig)))
                val[a[r]] = hv * MONT % R
                cmts.append((bytes(vals), dig, hv))
                ci += 1
            va = get(a[r])
            L[32 * r:32 * r + 32] = m2b(va)
            if k in (K_ADD, K_MUL):
                vb = get(b[r])
                vc = (va + vb) % R if k == K_ADD else va * vb % R * MINV % R
                val[c[r]] = vc
                Rv[32 * r:32 * r + 32] = m2b(vb)
                O[32 * r:32 * r + 32] = m2b(vc)
        return bytes(L), bytes(Rv), bytes(O), public, cmts


def srs(log_n, tau, curve="bls12-381"):
    """pk.Kzg.G1[:n+3] = [tau^i]G and pk.KzgLagrange.G1 = [L_i(tau)]G on the GPU
    (batch scalar multiplication); L_i(tau) = w^i (tau^n - 1) / (n (tau - w^i))
    with one batch inversion."""
    from gnark_amd import msm
    F = FIELDS[curve]
    R, MONT = F.R, F.MONT
    group = msm.BLS12_381_G1 if curve == "bls12-381" else msm.G1
    n = 1 << log_n
    w = F.cv.omega(n)
    gen = F.g1_to_bytes(F.cv.G1)
    pw, x = bytearray(32 * (n + 3)), 1
    for i in range(n + 3):
        pw[32 * i:32 * i + 32] = m2b(x * MONT % R)
        x = x * tau % R
    kzg = msm.batch_scalar_mul(group, gen, bytes(pw), n + 3)
    wi, dens = [1] * n, [0] * n
    for i in range(n):
        if i:
            wi[i] = wi[i - 1] * w % R
        dens[i] = (tau - wi[i]) % R
    pre, acc = [0] * n, 1
    for i in range(n):
        pre[i] = acc
        acc = acc * dens[i] % R
    inv = pow(acc, -1, R)
    cst = (pow(tau, n, R) - 1) * pow(n, -1, R) % R * MONT % R
    lag = bytearray(32 * n)
    for i in range(n - 1, -1, -1):
        d_inv = inv * pre[i] % R
        inv = inv * dens[i] % R
        lag[32 * i:32 * i + 32] = m2b(wi[i] * d_inv % R * cst % R)
    return kzg, msm.batch_scalar_mul(group, gen, bytes(lag), n)


def make_key(circ, tau, key_srs=None, shard=None, reduce=None, devices=None):
    from gnark_amd import plonk_prover as pp
    sel, qcp = circ.selectors()
    perm = circ.permutation()
    cv = circ.F.cv
    s123 = circ.s_polys(perm, cv.omega(circ.n), cv.fr_gen)
    kzg, kzg_lag = key_srs if key_srs is not None else srs(circ.log_n, tau, circ.curve)
    return pp.ProvingKey(circ.log_n, kzg, kzg_lag, *sel, *s123, perm.tobytes(), qcp=qcp,
                         nb_public=circ.nb_public, commitment_indexes=circ.cmt_idx, shard=shard, reduce=reduce,
                         devices=devices, curve=circ.curve)


def to_oracle(pk, proof):
    g = bo.g1_from_bytes
    vk = {"n": pk.n, "omega": pk.omega, "u": pk.g, "S": [g(s) for s in pk.vk.S], "Ql": g(pk.vk.Ql),
          "Qr": g(pk.vk.Qr), "Qm": g(pk.vk.Qm), "Qo": g(pk.vk.Qo), "Qk": g(pk.vk.Qk),
          "Qcp": [g(q) for q in pk.vk.Qcp], "nb_public": pk.vk.nb_public, "cmt_idx": pk.vk.commitment_indexes}
    pr = {"LRO": [g(x) for x in proof.LRO], "Z": g(proof.Z), "H": [g(x) for x in proof.H],
          "batched_H": g(proof.batched_H), "claimed": list(proof.claimed_values),
          "zs_H": g(proof.z_shifted_H), "zu": proof.z_shifted_value, "bsb22": [g(x) for x in proof.bsb22]}
    return pr, vk


def check_gates(circ, L, Rv, O, public, cmts):
    """Every row's constraint holds (Montgomery bytes in): a sanity check of the solver."""
    n = circ.n
    R, MINV = circ.F.R, circ.F.MINV

    def v(buf, i):
        return int.from_bytes(buf[32 * i:32 * i + 32], "little") * MINV % R
    ci = 0
    for r in range(n):
        k = int(circ.kind[r])
        if k == K_PUB:
            assert v(L, r) == public[r] % R
        elif k == K_CMTD:
            pass  # -v + Pi = 0 by construction of Pi
        elif k == K_CMT:
            assert v(L, r) == cmts[ci][2]
            ci += 1
        elif k == K_ADD:
            assert (v(L, r) + v(Rv, r) - v(O, r)) % R == 0
        else:
            assert (v(L, r) * v(Rv, r) - v(O, r)) % R == 0
