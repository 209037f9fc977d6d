"""Test infrastructure (oracle): a CPU restatement of gnark's PlonK prover,
backend/plonk/<curve>/prove.go:116-1391 (BLS12-381 and BN254 are the same
generated code), end to end -- commitToLRO, completeQk, deriveGammaAndBeta
(bindPublicData), buildRatioCopyConstraint, computeNumerator per coset,
divideByXMinusOne, commitToQuotient, openZ, foldH, computeLinearizedPolynomial,
batchOpening -- with the blinding coefficients injected (getRandomPolynomial,
prove.go:1175-1189) so its proof can be compared with the GPU prover's byte
for byte.  Only tests/ import it.

It is written from prove.go / verify.go, not from the GPU code: plain
big-integer lists, O(n log n) textbook FFTs, and KZG commitments evaluated with
the SRS trapdoor ([p(tau)]G is exactly the MSM over the [tau^i]G of the key).
Transcript bytes follow gnark-crypto's fiat-shamir (challenge i = H(name_i |
digest_(i-1) | bindings)) with G1Affine.Marshal = RawBytes (uncompressed), the
layout the reference's BN254 Solidity verifier hashes
(backend/plonk/bn254/solidity.go:407-536, 961-1024: derive_gamma / beta /
alpha / zeta, compute_gamma_kzg, hash_fr) -- the reference-held statement of
challenge order and encoding.  gnark-crypto's iop/kzg algorithms ([ext]:
BuildRatioCopyConstraint, kzg.Open, BatchOpenSinglePoint) are restated from
their call sites and published algorithms.
"""
import hashlib

import bls12_381_oracle as _bls


# ---------------------------------------------------------------- curve adapters
class Curve:
    """Scalar field and G1 of a pairing curve, as the prover needs them."""

    def __init__(self, name, R, fr_gen, g1_gen, add, mul, inf, raw):
        self.name, self.R, self.fr_gen, self.G1 = name, R, fr_gen, g1_gen
        self.add, self.mul, self.INF, self.raw = add, mul, inf, raw

    def omega(self, n):
        """fft.NewDomain's generator: fr_gen^((r-1)/n) (fri_test.go:35 pins it for BN254)."""
        return pow(self.fr_gen, (self.R - 1) // n, self.R)

    def hash_to_field(self, msg, dst=b"BSB22-Plonk"):
        """fr.Hash(msg, dst, 1): 48 bytes of expand_message_xmd (SHA-256), big-endian,
        mod r -- the hash_fr of plonk/bn254/solidity.go:672-760."""
        return int.from_bytes(_bls.expand_message_xmd(msg, dst, 48), "big") % self.R


BLS12_381 = Curve("bls12-381", _bls.R, _bls.FR_GEN, _bls.G1_GEN, _bls.g1_add, _bls.g1_mul, _bls.INF,
                  _bls.g1_raw_bytes)


def _bn254():
    import bn254_oracle as b

    def add(p, q):
        return b.g1_add(p, q)

    def mul(p, k):
        return b.g1_mul(p, k % b.R)

    def raw(p):
        # RawBytes of bn254 (mUncompressed = 0): X | Y big-endian, infinity all zero
        if p is None:
            return bytes(64)
        return p[0].to_bytes(32, "big") + p[1].to_bytes(32, "big")
    return Curve("bn254", b.R, b.FR_GEN, b.G1_GEN, add, mul, None, raw)


def curve(name):
    return BLS12_381 if name == "bls12-381" else _bn254()


# ---------------------------------------------------------------- field helpers
def _bitrev(i, logn):
    return int(format(i, f"0{logn}b")[::-1], 2) if logn else 0


def _dif(a, w, R):
    n, m = len(a), len(a) >> 1
    while m >= 1:
        wm = pow(w, n // (2 * m), R)
        for st in range(0, n, 2 * m):
            t = 1
            for j in range(m):
                u, v = a[st + j], a[st + j + m]
                a[st + j] = (u + v) % R
                a[st + j + m] = (u - v) * t % R
                t = t * wm % R
        m >>= 1
    return a


def _natural(a):
    lg = len(a).bit_length() - 1
    return [a[_bitrev(i, lg)] for i in range(len(a))]


def evals(coeffs, w, R, shift=1):
    """p(shift w^j), j < n, natural order (coefficients natural order, len n)."""
    a = [c * pow(shift, j, R) % R for j, c in enumerate(coeffs)]
    return _natural(_dif(a, w, R))


def interpolate(values, w, R, shift=1):
    """coefficients (natural order) of the polynomial with p(shift w^j) = values[j]."""
    n = len(values)
    c = _natural(_dif(list(values), pow(w, -1, R), R))
    ninv, sinv = pow(n, -1, R), pow(shift, -1, R)
    return [x * ninv % R * pow(sinv, j, R) % R for j, x in enumerate(c)]


def horner(c, x, R):
    r = 0
    for v in reversed(c):
        r = (r * x + v) % R
    return r


class Transcript:
    """gnark-crypto fiat-shamir: challenge i = H(name_i | digest_(i-1) | bindings_i),
    the field element SetBytes(digest) (solidity.go: mod(digest, R_MOD))."""

    def __init__(self, R, names, h=None):
        self.R, self.h, self.order = R, h or hashlib.sha256, list(names)
        self.data, self.digest = {k: b"" for k in names}, {}

    def bind(self, name, b):
        self.data[name] += bytes(b)

    def challenge(self, name):
        i = self.order.index(name)
        prev = self.digest[self.order[i - 1]] if i else b""
        self.digest[name] = self.h(name.encode() + prev + self.data[name]).digest()
        return int.from_bytes(self.digest[name], "big") % self.R


# ---------------------------------------------------------------- key
def setup(cv, log_n, ql, qr, qm, qo, qk, s1, s2, s3, qcp, perm, nb_public, cmt_idx, tau, big_log=None):
    """The key the prover reads (setup.go:110-161, 229-272): trace polynomials in
    canonical form (inputs are Lagrange regular, as BuildTrace leaves them),
    the KZG SRS as its trapdoor tau, vk digests [p(tau)]G."""
    R = cv.R
    n = 1 << log_n
    big_log = big_log if big_log is not None else log_n + (2 if n >= 6 else 3)
    w = cv.omega(n)
    can = {k: interpolate(v, w, R) for k, v in dict(ql=ql, qr=qr, qm=qm, qo=qo, qk=qk, s1=s1, s2=s2,
                                                        s3=s3).items()}
    qcp_c = [interpolate(v, w, R) for v in qcp]
    key = dict(cv=cv, n=n, log_n=log_n, big=1 << big_log, omega=w, omega_big=cv.omega(1 << big_log),
               u=cv.fr_gen, tau=tau, trace=can, qk_lag=list(qk), qcp=qcp_c, perm=list(perm),
               nb_public=nb_public, cmt_idx=list(cmt_idx))
    com = lambda c: commit(key, c)  # noqa: E731
    key["vk"] = dict(S=[com(can["s1"]), com(can["s2"]), com(can["s3"])], Ql=com(can["ql"]), Qr=com(can["qr"]),
                     Qm=com(can["qm"]), Qo=com(can["qo"]), Qk=com(can["qk"]), Qcp=[com(c) for c in qcp_c])
    return key


def commit(key, coeffs):
    """kzg.Commit(coeffs, pk.Kzg) = sum c_i [tau^i]G = [p(tau)]G."""
    cv = key["cv"]
    return cv.mul(cv.G1, horner(coeffs, key["tau"], cv.R))


def commit_lagrange(key, values):
    """kzg.Commit(values, pk.KzgLagrange) (prove.go:336, 494)."""
    return commit(key, interpolate(values, key["omega"], key["cv"].R))


# ---------------------------------------------------------------- prover
def prove(key, L, Rv, O, public=(), cmts=(), blinding=None, challenge_hash=None, folding_hash=None):
    """Prove after Solve (prove.go:116-176).  L, Rv, O: solution.L/R/O (Lagrange
    regular ints); public: fullWitness[:len(spr.Public)]; cmts: per BSB22
    commitment (committed-value vector (Lagrange, n ints), digest point, hashed
    value) as bsb22Hint left them (prove.go:316-352); blinding: the 9 coefficients
    of Bl, Br, Bo (2 each) and Bz (3), in that order (initBlindingPolynomials,
    prove.go:295-302).  Returns the proof as a dict (prove.go:96-114)."""
    cv = key["cv"]
    R, n, w, u = cv.R, key["n"], key["omega"], key["u"]
    tr, vk = key["trace"], key["vk"]
    bl, br, bo, bz = blinding[0:2], blinding[2:4], blinding[4:6], blinding[6:9]
    tn1 = (pow(key["tau"], n, R) - 1) % R

    # commitToPolyAndBlinding (prove.go:492-502) + commitBlindingFactor (:1159-1172):
    # [p(tau)] + [b(tau) (tau^n - 1)]
    def commit_blinded(lag, b):
        return cv.add(commit_lagrange(key, lag), cv.mul(cv.G1, horner(b, key["tau"], R) * tn1 % R))
    proof = dict(LRO=[commit_blinded(L, bl), commit_blinded(Rv, br), commit_blinded(O, bo)],
                 bsb22=[c[1] for c in cmts])
    # completeQk (prove.go:397-423)
    qk = list(key["qk_lag"])
    for i, x in enumerate(public):
        qk[i] = x % R
    for (vals, dig, hv), ci in zip(cmts, key["cmt_idx"]):
        qk[key["nb_public"] + ci] = hv % R
    # deriveGammaAndBeta (prove.go:454-489), bindPublicData (verify.go:296-340)
    fs = Transcript(R, ("gamma", "beta", "alpha", "zeta"), challenge_hash)
    for p in vk["S"] + [vk["Ql"], vk["Qr"], vk["Qm"], vk["Qo"], vk["Qk"]] + vk["Qcp"]:
        fs.bind("gamma", cv.raw(p))
    for x in public:
        fs.bind("gamma", (x % R).to_bytes(32, "big"))
    for p in proof["LRO"]:
        fs.bind("gamma", cv.raw(p))
    gamma = fs.challenge("gamma")
    beta = fs.challenge("beta")
    # buildRatioCopyConstraint (prove.go:600-632; iop.BuildRatioCopyConstraint [ext]):
    # Z[0] = 1, Z[i+1] = Z[i] prod_j (f_j[i] + beta ID(j n + i) + gamma) / (f_j[i] + beta ID(S[j n + i]) + gamma),
    # ID(s) = u^(s div n) w^(s mod n) (getSupportPermutation, setup.go:391-407)
    ids = [pow(u, s // n, R) * pow(w, s % n, R) % R for s in range(3 * n)]
    f = (L, Rv, O)
    Zl = [1] * n
    for i in range(n - 1):
        num = den = 1
        for j in range(3):
            num = num * (f[j][i] + beta * ids[j * n + i] + gamma) % R
            den = den * (f[j][i] + beta * ids[key["perm"][j * n + i]] + gamma) % R
        Zl[i + 1] = Zl[i] * num % R * pow(den, -1, R) % R
    proof["Z"] = commit_blinded(Zl, bz)
    # deriveAlpha (prove.go:504-512)
    for p in proof["bsb22"]:
        fs.bind("alpha", cv.raw(p))
    fs.bind("alpha", cv.raw(proof["Z"]))
    alpha = fs.challenge("alpha")
    # computeNumerator (prove.go:837-1079) on rho cosets g w_big^i of the small domain
    lc, rc, oc, zc = (interpolate(v, w, R) for v in (L, Rv, O, Zl))
    qkc = interpolate(qk, w, R)
    pi_c = [interpolate(c[0], w, R) for c in cmts]
    ident = [0] * n
    ident[1] = beta  # beta X (prove.go:562-565)
    lone = [pow(n, -1, R)] * n  # Lagrange (1, 0, ..., 0) in canonical form
    rho, big = key["big"] // n, key["big"]
    lb = big.bit_length() - 1
    cres = [0] * big
    cs, css = u, u * u % R  # Domain[1].FrMultiplicativeGen and its square (prove.go:869-871)
    tw0 = [pow(w, j, R) for j in range(n)]
    for i in range(rho):
        sh = u * pow(key["omega_big"], i, R) % R
        tmp = (pow(sh, n, R) - 1) % R
        # bl <- bl (s w^i)^n - 1) s^j (prove.go:985-993)
        bsc = [[c * tmp % R * pow(sh, j, R) % R for j, c in enumerate(b)] for b in (bl, br, bo, bz)]
        ev = lambda c: evals(c, w, R, sh)  # noqa: E731
        xl, xr, xo, xz = ev(lc), ev(rc), ev(oc), ev(zc)
        xql, xqr, xqm, xqo, xqk = ev(tr["ql"]), ev(tr["qr"]), ev(tr["qm"]), ev(tr["qo"]), ev(qkc)
        xs1, xs2, xs3 = ev(tr["s1"]), ev(tr["s2"]), ev(tr["s3"])
        xid, xlone = ev(ident), ev(lone)
        xqc = [ev(c) for c in key["qcp"]]
        xpi = [ev(c) for c in pi_c]
        for j in range(n):
            # allConstraints (prove.go:928-954)
            s1, s2, s3 = xs1[j] * beta % R, xs2[j] * beta % R, xs3[j] * beta % R
            lv = (xl[j] + horner(bsc[0], tw0[j], R)) % R
            rv = (xr[j] + horner(bsc[1], tw0[j], R)) % R
            ov = (xo[j] + horner(bsc[2], tw0[j], R)) % R
            zv = (xz[j] + horner(bsc[3], tw0[j], R)) % R
            zs = (xz[(j + 1) % n] + horner(bsc[3], tw0[(j + 1) % n], R)) % R
            ic = (xql[j] * lv + xqr[j] * rv + xqm[j] * lv % R * rv + xqo[j] * ov + xqk[j]) % R
            for q, p in zip(xqc, xpi):
                ic = (ic + q[j] * p[j]) % R
            a = (gamma + lv + xid[j]) % R
            b = (xid[j] * cs + rv + gamma) % R
            c = (xid[j] * css + ov + gamma) % R
            r = a * b % R * c % R * zv % R
            a, b, c = (s1 + lv + gamma) % R, (s2 + rv + gamma) % R, (s3 + ov + gamma) % R
            l_ = (a * b % R * c % R * zs - r) % R
            rl = (zv - 1) * xlone[j] % R
            cres[_bitrev(rho * j + i, lb)] = ((rl * alpha + l_) * alpha + ic) % R
    # divideByXMinusOne (prove.go:1223-1276): cres is LagrangeCoset / BitReverse on the big domain
    xn = [(pow(u, n, R) * pow(pow(key["omega_big"], n, R), i, R) - 1) % R for i in range(rho)]
    xinv = [pow(x, -1, R) for x in xn]
    vals = [cres[_bitrev(k, lb)] * xinv[k % rho] % R for k in range(big)]  # natural order
    h = interpolate(vals, key["omega_big"], R, u)
    h1, h2, h3 = h[:n + 2], h[n + 2:2 * (n + 2)], h[2 * (n + 2):3 * (n + 2)]
    assert all(v == 0 for v in h[3 * (n + 2):]), "quotient degree > 3(n + 2)"
    proof["H"] = [commit(key, x) for x in (h1, h2, h3)]
    for p in proof["H"]:
        fs.bind("zeta", cv.raw(p))
    zeta = fs.challenge("zeta")

    # getBlindedCoefficients (prove.go:1148-1156): p - b + b X^n
    def blinded(c, b):
        out = list(c) + list(b)
        for k in range(len(b)):
            out[k] = (out[k] - b[k]) % R
        return out
    # openZ (prove.go:635-652): kzg.Open(blindedZ, zeta w)
    bzc = blinded(zc, bz)
    zw = zeta * w % R
    zu = horner(bzc, zw, R)
    proof["zu"] = zu
    proof["zs_H"] = commit(key, _div_x_minus_a(bzc, zu, zw, R))
    # foldH (prove.go:670-705)
    zp = pow(zeta, n + 2, R)
    folded = [((h3[k] * zp + h2[k]) * zp + h1[k]) % R for k in range(n + 2)]
    fdig = cv.add(cv.mul(cv.add(cv.mul(proof["H"][2], zp), proof["H"][1]), zp), proof["H"][0])
    # computeLinearizedPolynomial (prove.go:707-775, 1289-1389)
    zn1 = (pow(zeta, n, R) - 1) % R
    lz, rz, oz = ((horner(c, zeta, R) + horner(b, zeta, R) * zn1) % R for c, b in ((lc, bl), (rc, br), (oc, bo)))
    qcpz = [horner(c, zeta, R) for c in key["qcp"]]
    s1z, s2z = horner(tr["s1"], zeta, R), horner(tr["s2"], zeta, R)
    ls1 = (s1z * beta + lz + gamma) % R * ((s2z * beta + rz + gamma) % R) % R * zu % R * beta % R
    uz, uuz = zeta * u % R, zeta * u * u % R
    ls2 = -((beta * zeta + lz + gamma) * (beta * uz + rz + gamma) % R * (beta * uuz + oz + gamma)) % R
    lag = zn1 * pow(zeta - 1, -1, R) % R * alpha % R * alpha % R * pow(n, -1, R) % R
    lin = []
    for k, zk in enumerate(bzc):
        t = zk * ls2 % R
        if k < n:
            t = (t + tr["s3"][k] * ls1) % R
        t = t * alpha % R
        if k < n:
            t = (t + tr["ql"][k] * lz + tr["qm"][k] * (rz * lz % R) + tr["qr"][k] * rz + tr["qo"][k] * oz
                 + tr["qk"][k]) % R
            for pc, qz in zip(pi_c, qcpz):
                t = (t + pc[k] * qz) % R
        lin.append((t + zk * lag) % R)
    ldig = commit(key, lin)
    # batchOpening: kzg.BatchOpenSinglePoint (prove.go:777-833)
    polys = [folded, lin, blinded(lc, bl), blinded(rc, br), blinded(oc, bo), tr["s1"], tr["s2"]] + key["qcp"]
    digests = [fdig, ldig] + proof["LRO"] + [vk["S"][0], vk["S"][1]] + vk["Qcp"]
    claimed = [horner(p, zeta, R) for p in polys]
    fk = Transcript(R, ("gamma",), folding_hash)
    fk.bind("gamma", zeta.to_bytes(32, "big"))
    for d in digests:
        fk.bind("gamma", cv.raw(d))
    for c in claimed:
        fk.bind("gamma", c.to_bytes(32, "big"))
    fk.bind("gamma", zu.to_bytes(32, "big"))  # dataTranscript: ZShiftedOpening.ClaimedValue.Marshal()
    gk = fk.challenge("gamma")
    m = max(len(p) for p in polys)
    fold, fv, gp = [0] * m, 0, 1
    for p, c in zip(polys, claimed):
        for k, x in enumerate(p):
            fold[k] = (fold[k] + gp * x) % R
        fv = (fv + gp * c) % R
        gp = gp * gk % R
    proof["batched_H"] = commit(key, _div_x_minus_a(fold, fv, zeta, R))
    proof["claimed"] = claimed
    proof["challenges"] = dict(gamma=gamma, beta=beta, alpha=alpha, zeta=zeta, gamma_kzg=gk)
    return proof


def _div_x_minus_a(f, fa, a, R):
    """(f - f(a)) / (X - a) by synthetic division (kzg.Open's quotient [ext])."""
    f = list(f)
    f[0] = (f[0] - fa) % R
    for i in range(len(f) - 2, -1, -1):
        f[i] = (f[i] + f[i + 1] * a) % R
    return f[1:]


# ---------------------------------------------------------------- verifier
def verify_trapdoor(key, proof, public=(), challenge_hash=None, folding_hash=None):
    """Verify (verify.go:45-290) over the key's curve with the SRS trapdoor tau in
    place of the two pairings; the transcript as prove() (and solidity.go) binds it."""
    cv = key["cv"]
    R, n, u, w, tau, vk = cv.R, key["n"], key["u"], key["omega"], key["tau"], key["vk"]
    bsb = proof["bsb22"]
    if len(bsb) != len(vk["Qcp"]) or len(public) != key["nb_public"]:
        return False
    fs = Transcript(R, ("gamma", "beta", "alpha", "zeta"), challenge_hash)
    for p in vk["S"] + [vk["Ql"], vk["Qr"], vk["Qm"], vk["Qo"], vk["Qk"]] + vk["Qcp"]:
        fs.bind("gamma", cv.raw(p))
    for x in public:
        fs.bind("gamma", (x % R).to_bytes(32, "big"))
    for p in proof["LRO"]:
        fs.bind("gamma", cv.raw(p))
    gamma, beta = fs.challenge("gamma"), fs.challenge("beta")
    for p in bsb + [proof["Z"]]:
        fs.bind("alpha", cv.raw(p))
    alpha = fs.challenge("alpha")
    for p in proof["H"]:
        fs.bind("zeta", cv.raw(p))
    zeta = fs.challenge("zeta")
    zn1 = (pow(zeta, n, R) - 1) % R
    lag1 = zn1 * pow(zeta - 1, -1, R) % R * pow(n, -1, R) % R
    # PI(zeta) with the hashed BSB22 commitments at their rows (verify.go:102-155)
    pi = 0
    for i, x in enumerate(public):
        wi = pow(w, i, R)
        pi = (pi + wi * zn1 % R * pow(n * (zeta - wi), -1, R) * x) % R
    for j, c in enumerate(bsb):
        wi = pow(w, key["nb_public"] + key["cmt_idx"][j], R)
        pi = (pi + wi * zn1 % R * pow(n * (zeta - wi), -1, R) * cv.hash_to_field(cv.raw(c))) % R
    zu, cl = proof["zu"], proof["claimed"]
    hq, lin, l, r, o, s1, s2 = cl[:7]
    t = (s1 * beta + l + gamma) * (s2 * beta + r + gamma) % R * (o + gamma) % R * alpha % R * zu % R
    if hq != (lin + pi + t - lag1 * alpha % R * alpha) % R * pow(zn1, -1, R) % R:
        return False
    zp = pow(zeta, n + 2, R)
    fh = cv.add(cv.add(proof["H"][0], cv.mul(proof["H"][1], zp)), cv.mul(proof["H"][2], zp * zp % R))
    a1 = zu * beta % R * ((beta * s1 + l + gamma) % R) % R * ((beta * s2 + r + gamma) % R) % R * alpha % R
    a2 = (beta * zeta + l + gamma) * ((beta * zeta * u + r + gamma) % R) % R * ((beta * zeta * u * u + o + gamma) % R)
    a2 = (-a2 * alpha + lag1 * alpha % R * alpha) % R
    ld = cv.INF
    for p, s in zip(bsb + [vk["Ql"], vk["Qr"], vk["Qm"], vk["Qo"], vk["Qk"], vk["S"][2], proof["Z"]],
                    cl[7:] + [l, r, l * r % R, o, 1, a1, a2]):
        ld = cv.add(ld, cv.mul(p, s))
    digests = [fh, ld] + proof["LRO"] + [vk["S"][0], vk["S"][1]] + vk["Qcp"]
    fk = Transcript(R, ("gamma",), folding_hash)
    fk.bind("gamma", zeta.to_bytes(32, "big"))
    for d in digests:
        fk.bind("gamma", cv.raw(d))
    for c in cl:
        fk.bind("gamma", (c % R).to_bytes(32, "big"))
    fk.bind("gamma", (zu % R).to_bytes(32, "big"))
    gk = fk.challenge("gamma")
    fd, fy, gp = cv.INF, 0, 1
    for d, y in zip(digests, cl):
        fd, fy, gp = cv.add(fd, cv.mul(d, gp)), (fy + gp * y) % R, gp * gk % R

    def kzg_ok(digest, h, point, value):  # [w(tau)](tau - z) == C - [y]G
        rhs = cv.add(digest, cv.mul(cv.G1, (-value) % R))
        return cv.mul(h, (tau - point) % R) == rhs
    return kzg_ok(fd, proof["batched_H"], zeta, fy) and kzg_ok(proof["Z"], proof["zs_H"], zeta * w % R, zu)
