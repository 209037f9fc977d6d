"""PlonK BLS12-381 prover orchestration over the device kernels (SURVEY 8a rows
a18-a21; host mirror of backend/plonk/bls12-381/prove.go:116-1079).

The steps follow prove.go one to one, each on the GPU through the C ABI:

  commitToLRO            (:425-452, 492-502, 1159-1172)  gg_msm on pk.KzgLagrange + blinding
  deriveGammaAndBeta     (:454-489)                       Fiat-Shamir on the host (sha256)
  buildRatioCopyConstraint (:600-633)                     gg_plonk_ratio_copy_constraint + commit
  evaluateConstraints    (:520-597)  computeNumerator (:837-1079): per coset, every polynomial's
                          coset evaluations (gg_ntt DIT on the canonical bit-reversed copy) and
                          gg_plonk_numerator_coset; divideByXMinusOne; commitToQuotient (:1199-1218)
  openZ                  (:635-652)  gg_bls12_381_fr_horner (value + quotient) + commit
  foldH                  (:670-705)  gg_plonk_fold_h; digest folded by a 3-point MSM
  computeLinearizedPolynomial (:707-775, 1289-1389)  gg_plonk_linearized + commit
  batchOpening           (:777-835)  kzg.BatchOpenSinglePoint: evaluations, folding
                          (gg_bls12_381_fr_axpy), opening quotient, commit

Scope of this mirror: no public inputs and no BSB22 commitments (the reference's
extra terms for those are host bookkeeping).  The transcript restates gnark-crypto's
fiat-shamir (sha256; each challenge hashes its name, the previous challenge and its
bindings; points bound uncompressed, big-endian) -- gnark-crypto is absent here, so
the transcript bytes are not pinned; proofs are checked by the PlonK verifier
equations (verify.go:45-290) with the SRS trapdoor in tests/.
Device polynomials are bls12-381 fr Montgomery (gnark-crypto memory layout).
"""
from __future__ import annotations

import ctypes
import dataclasses
import hashlib
import secrets
from typing import List, Optional

from . import fr, msm, ntt, plonk
from ._lib import DeviceBuffer, check, lib, ptr, GG_CURVE_BLS12_381

R = fr.BLS_R
P = fr.BLS_P
ORDER_BLINDING = (1, 1, 1, 2)  # order_blinding_L, _R, _O, _Z (prove.go:88-93)


# ------------------------------------------------------------------ encodings
def fr_int(b: bytes) -> int:
    return fr.bls_fr_unmont(b)


def fr_b(x: int) -> bytes:
    return fr.bls_fr_mont(x % R)


def g1_marshal(aff: bytes) -> bytes:
    """G1Affine.RawBytes / Marshal: X | Y big-endian (48 B each), infinity flag 0x40."""
    if aff == bytes(96):
        return bytes([0x40]) + bytes(95)
    x, y = fr.bls_fp_unmont(aff[:48]), fr.bls_fp_unmont(aff[48:])
    return x.to_bytes(48, "big") + y.to_bytes(48, "big")


def fr_marshal(x: int) -> bytes:
    return (x % R).to_bytes(32, "big")


class Transcript:
    """fiat-shamir Transcript (gnark-crypto, restated): challenge i hashes
    name_i | value_(i-1) | bindings_i."""

    def __init__(self, *names: str, h=hashlib.sha256):
        self.order = list(names)
        self.bind_data = {n: [] for n in names}
        self.values = {}
        self.h = h

    def bind(self, name: str, data: bytes):
        if name in self.values:
            raise ValueError(f"challenge {name} already computed")
        self.bind_data[name].append(bytes(data))

    def compute(self, name: str) -> bytes:
        i = self.order.index(name)
        h = self.h()
        h.update(name.encode())
        if i > 0:
            h.update(self.values[self.order[i - 1]])
        for d in self.bind_data[name]:
            h.update(d)
        self.values[name] = h.digest()
        return self.values[name]


def derive_randomness(fs: Transcript, name: str, *points: bytes) -> int:
    """deriveRandomness (verify.go:342-360): bind the points, fr.SetBytes(challenge)."""
    for p in points:
        fs.bind(name, g1_marshal(p))
    return int.from_bytes(fs.compute(name), "big") % R


# ------------------------------------------------------------------ device helpers
def dcopy(dst, src, nbytes: int):
    check(lib.gg_copy_device(ptr(dst), ptr(src), nbytes))


def dzero(buf, nbytes: int):
    check(lib.gg_memset_device(ptr(buf), 0, nbytes))


def bit_reverse(src, dst, n: int):
    check(lib.gg_bls12_381_fr_bit_reverse(ptr(src), ptr(dst), n, None))


def axpy(y, x, n: int, a: int):
    check(lib.gg_bls12_381_fr_axpy(ptr(y), ptr(x), n, fr_b(a), None))


def poly_eval(buf, n: int, x: int) -> int:
    return fr_int(plonk.evaluate(buf, n, fr_b(x)))


def host_eval(coeffs: List[int], x: int) -> int:
    r = 0
    for c in reversed(coeffs):
        r = (r * x + c) % R
    return r


# ------------------------------------------------------------------ keys
@dataclasses.dataclass
class VerifyingKey:
    """backend/plonk/bls12-381 VerifyingKey (setup.go:41-70) minus the G2 part:
    Size, SizeInv, Generator, CosetShift, S[3], Ql, Qr, Qm, Qo, Qk (affine bytes)."""
    size: int
    generator: int
    coset_shift: int
    S: List[bytes]
    Ql: bytes
    Qr: bytes
    Qm: bytes
    Qo: bytes
    Qk: bytes


class ProvingKey:
    """Device-resident PlonK proving key (setup.go:88-106): the trace polynomials
    in canonical form (regular and bit-reversed copies), the permutation, the two
    KZG bases (pk.Kzg.G1[:n+3] and pk.KzgLagrange.G1[:n]) and the domains."""

    def __init__(self, log_n: int, kzg_g1: bytes, kzg_lagrange_g1: bytes, ql, qr, qm, qo, qk,
                 s1, s2, s3, perm, vk: Optional[VerifyingKey] = None, big_log: int = None,
                 shard=None, reduce=None):
        """kzg_g1: n+3 affine points [tau^i]G; kzg_lagrange_g1: n points [L_i(tau)]G;
        ql..qk: Lagrange regular selectors; s1..s3: permutation polynomials in
        Lagrange regular form (computePermutationPolynomials); perm: 3n int64
        (pk.trace.S).  All fr vectors: Montgomery bytes or device buffers of n fr.

        Multi-GPU: shard = (rank, world) keeps only this rank's
        contiguous slice of each KZG base resident; every commitment is then a
        partial MSM over the slice and `reduce(jac) -> jac` (an all-gather + exact
        add across ranks, gnark_amd.dist.allgather_partial) completes it.  All
        other work is replicated, so every rank holds the same polynomials and
        transcript (the blinding randomness must be the same on all ranks)."""
        self.log_n = log_n
        self.n = n = 1 << log_n
        self.big_log = big_log if big_log is not None else log_n + 2
        self.rho = 1 << (self.big_log - log_n)
        w = fr.bls_domain_generator(log_n)
        wb = fr.bls_domain_generator(self.big_log)
        g = fr.BLS_FR_MULTIPLICATIVE_GEN
        self.omega, self.omega_big, self.g = w, wb, g
        self.d0 = ntt.Domain(log_n, fr_b(w), fr_b(g), curve=GG_CURVE_BLS12_381)
        self.d1 = ntt.Domain(self.big_log, fr_b(wb), fr_b(g), curve=GG_CURVE_BLS12_381)
        # coset domains of computeNumerator: coset i of the big domain is shift s_i = g wb^i
        self.coset_shift = [g * pow(wb, i, R) % R for i in range(self.rho)]
        self.dcos = [ntt.Domain(log_n, fr_b(w), fr_b(s), curve=GG_CURVE_BLS12_381) for s in self.coset_shift]
        on_dev = isinstance(kzg_g1, DeviceBuffer)
        from .dist import shard_range
        rank, world = shard if shard is not None else (0, 1)
        self.reduce = reduce if reduce is not None else (lambda j: j)
        self.k_lo, self.k_hi = shard_range(n + 3, rank, world)
        self.l_lo, self.l_hi = shard_range(n, rank, world)

        def base(points, lo, hi, dev):
            if dev:
                return msm.MsmBase(msm.BLS12_381_G1, points.ptr + 96 * lo, hi - lo, on_device=True)
            return msm.MsmBase(msm.BLS12_381_G1, points[96 * lo:96 * hi], hi - lo)

        self.kzg = base(kzg_g1, self.k_lo, self.k_hi, on_dev)
        self.kzg_lag = base(kzg_lagrange_g1, self.l_lo, self.l_hi,
                            isinstance(kzg_lagrange_g1, DeviceBuffer))
        if on_dev:  # the two 3-point slices of commitBlindingFactor, to the host
            lo, hi = bytearray(96 * 3), bytearray(96 * 3)
            check(lib.gg_copy_to_host(ptr(lo), ptr(kzg_g1), len(lo)))
            check(lib.gg_copy_to_host(ptr(hi), ctypes.c_void_p(kzg_g1.ptr + 96 * n), len(hi)))
            blind_lo, blind_hi = bytes(lo), bytes(hi)
        else:
            blind_lo, blind_hi = kzg_g1[:96 * 3], kzg_g1[96 * n:96 * (n + 3)]
        nb = 32 * n
        # trace: canonical regular (commitments, openings, linearization) and
        # canonical bit-reversed (input of the coset DIT FFTs)
        self.reg, self.brev = {}, {}
        for name, v in (("Ql", ql), ("Qr", qr), ("Qm", qm), ("Qo", qo), ("Qk", qk),
                        ("S1", s1), ("S2", s2), ("S3", s3)):
            b = DeviceBuffer(nb)
            if isinstance(v, DeviceBuffer):
                dcopy(b, v, nb)
            else:
                check(lib.gg_copy_to_device(ctypes.c_void_p(b.ptr), ptr(v), nb))
            self.d0.fft_inverse(b, ntt.DIF)        # Lagrange regular -> canonical bit-reversed
            reg = DeviceBuffer(nb)
            bit_reverse(b, reg, n)                 # ToRegular
            self.brev[name], self.reg[name] = b, reg
        self.perm = DeviceBuffer.from_host(perm) if not isinstance(perm, DeviceBuffer) else perm
        # blinding-commitment bases: G1[:3] and G1[n:n+3] (commitBlindingFactor)
        self.blind_lo, self.blind_hi = blind_lo, blind_hi  # G1[:3], G1[n:n+3] (host)
        # constant polynomials of computeNumerator: LOne (canonical: 1/n everywhere)
        # and s.twiddles0 (w^j)
        self.lone = DeviceBuffer(nb)
        inv_n = fr_b(pow(n, -1, R))
        chunk = inv_n * min(n, 1 << 16)
        for off in range(0, nb, len(chunk)):
            m = min(len(chunk), nb - off)
            check(lib.gg_copy_to_device(ctypes.c_void_p(self.lone.ptr + off), ptr(chunk[:m]), m))
        self.tw0 = _twiddles_dev(self)
        # coset evaluations of the key's polynomials, computed once (the reference
        # recomputes these rho * 2 FFTs per proof, prove.go:990-994, to save memory;
        # on 288 GB of HBM they stay resident): Ql..S3, X (for ID = beta X) and LOne
        xb = DeviceBuffer(nb)
        dzero(xb, nb)
        if n > 1:
            check(lib.gg_copy_to_device(ctypes.c_void_p(xb.ptr + 32 * (n // 2)), ptr(fr_b(1)), 32))
        else:
            check(lib.gg_copy_to_device(ctypes.c_void_p(xb.ptr), ptr(fr_b(0)), 32))
        src = dict(self.brev)
        src["X"], src["LOne"] = xb, self.lone
        self.coset_evals = {}
        for name, b in src.items():
            evs = []
            for i in range(self.rho):
                e = DeviceBuffer(nb)
                dcopy(e, b, nb)
                self.dcos[i].fft(e, ntt.DIT, coset=True)
                evs.append(e)
            self.coset_evals[name] = evs
        del xb
        self.ws = {}  # per-proof workspace, allocated on first use and reused
        self.vk = vk if vk is not None else commit_trace(self)

    def buf(self, name: str, nbytes: int) -> DeviceBuffer:
        """Workspace buffer reused across proofs (no per-proof hipMalloc)."""
        b = self.ws.get(name)
        if b is None or b.nbytes < nbytes:
            b = self.ws[name] = DeviceBuffer(nbytes)
        return b

    def commit_jac(self, buf, length: int) -> bytes:
        """kzg.Commit(p, pk.Kzg) (Jacobian) of a canonical polynomial of `length`
        <= n+3 coefficients: this rank's partial MSM, completed by reduce()."""
        src = buf
        if length < self.k_hi:
            src = self.buf("commit_pad", 32 * (self.n + 3))
            dzero(src, src.nbytes)
            dcopy(src, buf, 32 * length)
        addr = (src.ptr if isinstance(src, DeviceBuffer) else src.value) + 32 * self.k_lo
        return self.reduce(self.kzg.msm_jac(addr, self.k_hi - self.k_lo, on_device=True))

    def commit(self, buf, length: int) -> bytes:
        return msm.jac_to_affine(msm.BLS12_381_G1, self.commit_jac(buf, length))

    def commit_lagrange_jac(self, buf) -> bytes:
        """kzg.Commit(p, pk.KzgLagrange) of n Lagrange values (Jacobian)."""
        addr = (buf.ptr if isinstance(buf, DeviceBuffer) else buf.value) + 32 * self.l_lo
        return self.reduce(self.kzg_lag.msm_jac(addr, self.l_hi - self.l_lo, on_device=True))


def commit_trace(pk: ProvingKey) -> VerifyingKey:
    """commitTrace (setup.go:229-272): vk.S[0..2], Ql, Qr, Qm, Qo, Qk."""
    c = {k: pk.commit(pk.reg[k], pk.n) for k in ("Ql", "Qr", "Qm", "Qo", "Qk", "S1", "S2", "S3")}
    return VerifyingKey(pk.n, pk.omega, pk.g, [c["S1"], c["S2"], c["S3"]], c["Ql"], c["Qr"],
                        c["Qm"], c["Qo"], c["Qk"])


@dataclasses.dataclass
class Proof:
    """backend/plonk/bls12-381 Proof (prove.go:95-112), affine points (Montgomery bytes)."""
    LRO: List[bytes]
    Z: bytes
    H: List[bytes]
    batched_H: bytes
    claimed_values: List[int]
    z_shifted_H: bytes
    z_shifted_value: int


# ------------------------------------------------------------------ prover
def _blind_commit(pk: ProvingKey, coeffs: List[int]) -> bytes:
    """commitBlindingFactor (prove.go:1159-1172): [b(X) (X^n - 1)]."""
    G = msm.BLS12_381_G1
    acc = None
    for j, c in enumerate(coeffs):
        for base, k in ((pk.blind_hi, c), (pk.blind_lo, (-c) % R)):
            t = msm.scalar_mul(G, base[96 * j:96 * (j + 1)], fr_b(k))
            acc = t if acc is None else msm.jac_add(G, acc, t)
    return acc


def _commit_poly_and_blinding(pk: ProvingKey, lag, coeffs: List[int]) -> bytes:
    """commitToPolyAndBlinding (prove.go:492-502): Commit(p, pk.KzgLagrange) + [b (X^n - 1)]."""
    j = pk.commit_lagrange_jac(lag)
    return msm.jac_to_affine(msm.BLS12_381_G1, msm.jac_add(msm.BLS12_381_G1, j, _blind_commit(pk, coeffs)))


def _blinded_coeffs(pk: ProvingKey, canon_reg, b: List[int], name: str):
    """getBlindedCoefficients (prove.go:1148-1157): p | b, with p[i] -= b[i]."""
    n = pk.n
    out = pk.buf("blinded_" + name, 32 * (n + len(b)))
    dcopy(out, canon_reg, 32 * n)
    tail = b"".join(fr_b(c) for c in b)
    check(lib.gg_copy_to_device(ctypes.c_void_p(out.ptr + 32 * n), ptr(tail), len(tail)))
    head = DeviceBuffer.from_host(b"".join(fr_b((-c) % R) for c in b))
    axpy(out, head, len(b), 1)  # out[i] = p[i] - b[i], i < len(b)
    return out


def _open(pk: ProvingKey, poly, length: int, point: int):
    """kzg.Open (gnark-crypto [ext]): claimed value f(point) and H = Commit((f - f(a))/(X - a))."""
    q = pk.buf("open_q", 32 * max(length - 1, 1))
    val = fr_int(plonk.evaluate(poly, length, fr_b(point), q_out=q))
    return val, pk.commit(q, length - 1)


def prove(pk: ProvingKey, L, R_, O, rng=None, timings: Optional[dict] = None) -> Proof:
    """Prove after Solve (prove.go:116-176) for a circuit without public inputs
    or BSB22 commitments.  L, R_, O: the solver's Lagrange-regular vectors
    (Montgomery bytes or device buffers of n fr)."""
    import time
    rnd = rng or secrets.SystemRandom()
    n, nb = pk.n, 32 * pk.n
    t0 = time.perf_counter()
    tick = {}

    def mark(k):
        tick[k] = time.perf_counter()

    def dev(v):
        if isinstance(v, DeviceBuffer):
            return v
        return DeviceBuffer.from_host(v)

    x = {"L": dev(L), "R": dev(R_), "O": dev(O)}
    # initBlindingPolynomials (prove.go:295-302): random polynomials of order 1, 1, 1, 2
    bp = [[rnd.randrange(R) for _ in range(o + 1)] for o in ORDER_BLINDING]

    # commitToLRO
    lro = [_commit_poly_and_blinding(pk, x[k], bp[i]) for i, k in enumerate(("L", "R", "O"))]
    mark("commit_lro")
    # deriveGammaAndBeta + bindPublicData (verify.go:296-340; no public inputs)
    fs = Transcript("gamma", "beta", "alpha", "zeta")
    for p_ in pk.vk.S + [pk.vk.Ql, pk.vk.Qr, pk.vk.Qm, pk.vk.Qo, pk.vk.Qk]:
        fs.bind("gamma", g1_marshal(p_))
    gamma = derive_randomness(fs, "gamma", *lro)
    beta = int.from_bytes(fs.compute("beta"), "big") % R

    # buildRatioCopyConstraint
    z = pk.buf("z", nb)
    plonk.ratio_copy_constraint(x["L"], x["R"], x["O"], pk.perm, n, fr_b(beta), fr_b(gamma),
                                fr_b(pk.omega), fr_b(pk.g), z)
    z_commit = _commit_poly_and_blinding(pk, z, bp[3])
    mark("ratio_z")
    alpha = derive_randomness(fs, "alpha", z_commit)

    # canonical forms: bit-reversed (coset FFT input) and regular (openings)
    brev, reg = {}, {}
    for k, v in (("L", x["L"]), ("R", x["R"]), ("O", x["O"]), ("Z", z)):
        b = pk.buf("brev_" + k, nb)
        dcopy(b, v, nb)
        pk.d0.fft_inverse(b, ntt.DIF)
        r = pk.buf("reg_" + k, nb)
        bit_reverse(b, r, n)
        brev[k], reg[k] = b, r
    mark("canonical")

    # computeNumerator: per coset i, evaluations of every polynomial on g wb^i <w>;
    # the key's polynomials (and X, LOne) come precomputed from the key
    order = ["L", "R", "O", "Z", None, "Ql", "Qr", "Qm", "Qo", "Qk", "S1", "S2", "S3", "ID", "LOne"]
    ev = [pk.buf("ev%d" % k, nb) for k in range(5)] + [None] * 10
    idb = pk.buf("ev_id", nb)
    cres = pk.buf("cres", 32 * n * pk.rho)
    tw0 = pk.tw0
    for i in range(pk.rho):
        s = pk.coset_shift[i]
        for slot, k in enumerate(order[:4]):
            dcopy(ev[slot], brev[k], nb)
            pk.dcos[i].fft(ev[slot], ntt.DIT, coset=True)  # bit-reversed -> natural coset evaluations
        for slot in range(5, 13):
            ev[slot] = pk.coset_evals[order[slot]][i]
        dzero(idb, nb)
        axpy(idb, pk.coset_evals["X"][i], n, beta)  # ID = beta X (prove.go:578-580)
        ev[13], ev[14] = idb, pk.coset_evals["LOne"][i]
        # ZS(x) = Z(w x): the evaluations shifted by one (Shift(1), prove.go:582)
        dcopy(ev[4], ctypes.c_void_p(ev[3].ptr + 32), nb - 32)
        dcopy(ctypes.c_void_p(ev[4].ptr + nb - 32), ev[3], 32)
        sn1 = (pow(s, n, R) - 1) % R
        bl = [[fr_b(c * pow(s, j, R) % R * sn1) for j, c in enumerate(q)] for q in bp]
        plonk.numerator_coset(ev, bl, tw0, fr_b(beta), fr_b(gamma), fr_b(alpha), fr_b(pk.g), n,
                              pk.rho, i, cres)
    check(lib.gg_synchronize())
    mark("numerator")
    plonk.divide_by_xn_minus_one(pk.d1, n, cres)  # h, canonical regular, rho n
    mark("divide")
    # commitToQuotient: h1, h2, h3 of n + 2 coefficients
    hs = [ctypes.c_void_p(cres.ptr + 32 * (n + 2) * k) for k in range(3)]
    H = [pk.commit(hs[k], n + 2) for k in range(3)]
    mark("quotient")
    zeta = derive_randomness(fs, "zeta", *H)

    # openZ at w zeta (blinded Z)
    bz = _blinded_coeffs(pk, reg["Z"], bp[3], "Z")
    zu, zs_H = _open(pk, bz, n + 3, zeta * pk.omega % R)
    mark("open_z")

    # foldH
    zp = pow(zeta, n + 2, R)
    folded = pk.buf("folded_h", 32 * (n + 2))
    plonk.fold_h(cres, n, fr_b(zp), folded)
    folded_digest = fold_digests(H, [1, zp, zp * zp % R])
    mark("fold_h")

    # computeLinearizedPolynomial
    zn1 = (pow(zeta, n, R) - 1) % R

    def blinded_eval(k, b):  # evaluateBlinded (prove.go:1118-1145)
        return (poly_eval(reg[k], n, zeta) + host_eval(b, zeta) * zn1) % R

    l_z, r_z, o_z = blinded_eval("L", bp[0]), blinded_eval("R", bp[1]), blinded_eval("O", bp[2])
    s1_z, s2_z = poly_eval(pk.reg["S1"], n, zeta), poly_eval(pk.reg["S2"], n, zeta)
    mark("evaluations")
    sc = plonk.linearized_scalars(l_z, r_z, o_z, alpha, beta, gamma, zeta, zu, s1_z, s2_z, pk.g, n)
    lin = pk.buf("lin", 32 * (n + 3))
    dcopy(lin, bz, 32 * (n + 3))
    plonk.linearized(lin, n + 3, pk.reg["S3"], n,
                     [pk.reg[k] for k in ("Ql", "Qr", "Qm", "Qo", "Qk")], n, sc)
    mark("linearize")
    lin_digest = pk.commit(lin, n + 3)
    mark("linearized")

    # batchOpening: kzg.BatchOpenSinglePoint at zeta
    polys = [(folded, n + 2), (lin, n + 3), (_blinded_coeffs(pk, reg["L"], bp[0], "L"), n + 2),
             (_blinded_coeffs(pk, reg["R"], bp[1], "R"), n + 2),
             (_blinded_coeffs(pk, reg["O"], bp[2], "O"), n + 2),
             (pk.reg["S1"], n), (pk.reg["S2"], n)]
    digests = [folded_digest, lin_digest, lro[0], lro[1], lro[2], pk.vk.S[0], pk.vk.S[1]]
    claimed = [poly_eval(p_, m, zeta) for p_, m in polys]
    gfold = fold_gamma(zeta, digests, claimed, fr_marshal(zu))
    acc = pk.buf("fold_acc", 32 * (n + 3))
    dzero(acc, acc.nbytes)
    gp = 1
    for p_, m in polys:
        axpy(acc, p_, m, gp)
        gp = gp * gfold % R
    _, batched_H = _open(pk, acc, n + 3, zeta)
    mark("batch_open")
    if timings is not None:
        prev = t0
        for k, v in tick.items():
            timings[k] = 1e3 * (v - prev)
            prev = v
        timings["total"] = 1e3 * (prev - t0)
    return Proof(lro, z_commit, H, batched_H, claimed, zs_H, zu)


def fold_digests(points: List[bytes], scalars: List[int]) -> bytes:
    """sum k_i P_i for a handful of digests (host scalar multiplications)."""
    G = msm.BLS12_381_G1
    acc = None
    for p_, k in zip(points, scalars):
        j = msm.scalar_mul(G, p_, fr_b(k))
        acc = j if acc is None else msm.jac_add(G, acc, j)
    return msm.jac_to_affine(G, acc)


def fold_gamma(point: int, digests: List[bytes], claimed: List[int], data: bytes) -> int:
    """deriveGamma of kzg.BatchOpenSinglePoint (gnark-crypto [ext], restated): a
    one-challenge transcript binding the point, the digests, the claimed values
    and the caller's data (here Z(w zeta), prove.go:829)."""
    fs = Transcript("gamma")
    fs.bind("gamma", fr_marshal(point))
    for d in digests:
        fs.bind("gamma", g1_marshal(d))
    for c in claimed:
        fs.bind("gamma", fr_marshal(c))
    fs.bind("gamma", data)
    return int.from_bytes(fs.compute("gamma"), "big") % R


def _twiddles_dev(pk: ProvingKey):
    """s.twiddles0 = w^j (j < n) on the device: FFT of the coefficient vector e_1."""
    n = pk.n
    if n == 1:
        return DeviceBuffer.from_host(fr_b(1))
    b = DeviceBuffer(32 * n)
    dzero(b, b.nbytes)
    check(lib.gg_copy_to_device(ctypes.c_void_p(b.ptr + 32 * (n // 2)), ptr(fr_b(1)), 32))
    # coefficients of X in bit-reversed layout -> DIT gives evaluations w^j in natural order
    pk.d0.fft(b, ntt.DIT)
    return b
