"""PlonK BLS12-381 quotient-path kernels (backend/plonk/bls12-381/prove.go):
the per-coset allConstraints evaluation of computeNumerator (:850-935, with the
bit-reversed scatter of :1030-1041), divideByXMinusOne (:1223-1276) and
fr.BatchInvert (:1273).  Buffers are device memory, bls12-381 fr Montgomery."""
from __future__ import annotations

import ctypes

from ._lib import check, lib, ptr

# s.x order (prove.go:60-77)
ID_L, ID_R, ID_O, ID_Z, ID_ZS, ID_QL, ID_QR, ID_QM, ID_QO, ID_QK, ID_S1, ID_S2, ID_S3, \
    ID_ID, ID_LONE, ID_QCI = range(16)
MAX_BCOEF = 4


def numerator_coset(x_bufs, blinding, twiddles0, beta: bytes, gamma: bytes, alpha: bytes,
                    coset_gen: bytes, n: int, rho: int, coset: int, cres, stream=None):
    """x_bufs: device buffers in id_ order; blinding: 4 lists of fr bytes (Bl, Br,
    Bo, Bz coefficients, already coset-scaled)."""
    arr = (ctypes.c_void_p * len(x_bufs))(*[ptr(x).value for x in x_bufs])
    bc = bytearray(4 * MAX_BCOEF * 32)
    deg = (ctypes.c_int * 4)()
    for q, coeffs in enumerate(blinding):
        assert len(coeffs) <= MAX_BCOEF
        deg[q] = len(coeffs)
        for k, c in enumerate(coeffs):
            bc[(q * MAX_BCOEF + k) * 32:(q * MAX_BCOEF + k + 1) * 32] = c
    check(lib.gg_plonk_numerator_coset(arr, len(x_bufs), ptr(bc), deg, ptr(twiddles0), ptr(beta),
                                       ptr(gamma), ptr(alpha), ptr(coset_gen), n, rho, coset,
                                       ptr(cres), ptr(stream)))


def divide_by_xn_minus_one(big_domain, n_small: int, data, stream=None):
    check(lib.gg_plonk_divide_by_xn_minus_one(big_domain.handle, n_small, ptr(data), ptr(stream)))


def batch_invert(data, n: int, stream=None):
    check(lib.gg_bls12_381_fr_batch_invert(ptr(data), n, ptr(stream)))


# ------------------------------------------------ row a21: ratio, evaluate, fold, linearize
def _need(buf, nbytes: int, what: str):
    """Host-side bound check for sized buffers (DeviceBuffer / torch): the kernels
    cannot see the allocation, so an undersized buffer is refused before launch."""
    have = getattr(buf, "nbytes", None)
    if have is None and hasattr(buf, "numel"):
        have = buf.numel() * buf.element_size()
    if have is not None and have < nbytes:
        raise ValueError(f"{what}: buffer of {have} B, needs {nbytes} B")


def ratio_copy_constraint(l, r, o, perm_dev, n: int, beta: bytes, gamma: bytes, omega: bytes,
                          coset_shift: bytes, z_out, stream=None):
    """iop.BuildRatioCopyConstraint([L, R, O], pk.trace.S, beta, gamma,
    {Lagrange, Regular}, pk.Domain[0]) -> z_out (n fr, device)."""
    for b_, nm in ((l, "L"), (r, "R"), (o, "O"), (z_out, "Z")):
        _need(b_, 32 * n, nm)
    _need(perm_dev, 24 * n, "permutation")
    check(lib.gg_plonk_ratio_copy_constraint(ptr(l), ptr(r), ptr(o), ptr(perm_dev), n, ptr(beta),
                                             ptr(gamma), ptr(omega), ptr(coset_shift), ptr(z_out),
                                             ptr(stream)))


def prefix_product(data, n: int, stream=None):
    _need(data, 32 * n, "data")
    check(lib.gg_bls12_381_fr_prefix_product(ptr(data), n, ptr(stream)))


def evaluate(f, n: int, a: bytes, q_out=None, stream=None) -> bytes:
    """f(a) for canonical regular f (n fr, device); with q_out, also the KZG
    opening quotient (f - f(a)) / (X - a) (n - 1 fr)."""
    _need(f, 32 * n, "f")
    if q_out is not None:
        _need(q_out, 32 * max(n - 1, 0), "quotient")
    out = bytearray(32)
    check(lib.gg_bls12_381_fr_horner(ptr(f), n, ptr(a), ptr(q_out), ptr(out), ptr(stream)))
    return bytes(out)


def evaluate_many(polys, lens, a: bytes, curve: int = None, stream=None):
    """[f_k(a)] for up to 16 canonical regular device polynomials (one batched
    pass, gg_fr_evaluate_many); curve: GG_CURVE_BLS12_381 (default) or GG_CURVE_BN254."""
    import ctypes as _c
    from ._lib import GG_CURVE_BLS12_381
    k = len(polys)
    for f, n in zip(polys, lens):
        _need(f, 32 * n, "f")
    arr = (_c.c_void_p * k)(*[ptr(f).value for f in polys])
    ln = (_c.c_size_t * k)(*lens)
    out = bytearray(32 * k)
    check(lib.gg_fr_evaluate_many(GG_CURVE_BLS12_381 if curve is None else curve, arr, ln, k, ptr(a), ptr(out),
                                  ptr(stream)))
    return [bytes(out[32 * i:32 * i + 32]) for i in range(k)]


def fold_h(h, n_small: int, zeta_pow_np2: bytes, out, stream=None):
    _need(h, 3 * 32 * (n_small + 2), "h")
    _need(out, 32 * (n_small + 2), "folded h")
    check(lib.gg_plonk_fold_h(ptr(h), n_small, ptr(zeta_pow_np2), ptr(out), ptr(stream)))


def linearized_scalars(l_zeta: int, r_zeta: int, o_zeta: int, alpha: int, beta: int, gamma: int,
                       zeta: int, zu: int, s1_zeta: int, s2_zeta: int, coset_shift: int, n: int):
    """The eight scalars of computeLinearizedPolynomial (prove.go:1293-1336), as
    canonical integers mod r: s1, s2, alpha, l, r, l*r, o, alpha^2 L1(zeta) / n."""
    from .fr import BLS_R as R
    s1 = (s1_zeta * beta + l_zeta + gamma) % R
    t = (s2_zeta * beta + r_zeta + gamma) % R
    s1 = s1 * t % R * zu % R * beta % R
    uz = zeta * coset_shift % R
    uuz = uz * coset_shift % R
    s2 = (beta * zeta + l_zeta + gamma) % R
    s2 = s2 * ((beta * uz + r_zeta + gamma) % R) % R
    s2 = s2 * ((beta * uuz + o_zeta + gamma) % R) % R
    s2 = (-s2) % R
    lag = (pow(zeta, n, R) - 1) * pow(zeta - 1, -1, R) % R
    lag = lag * alpha % R * alpha % R * pow(n, -1, R) % R
    return [s1, s2, alpha % R, l_zeta % R, r_zeta % R, l_zeta * r_zeta % R, o_zeta % R, lag]


def linearized(blinded_z, nz: int, s3, ns3: int, q5, nq: int, scalars, pi2=(), qcp_zeta=(),
               stream=None):
    """computeLinearizedPolynomial in place on blinded_z (device, canonical).
    scalars: the 8 values of linearized_scalars (ints); q5 = (Ql, Qr, Qm, Qo, Qk)."""
    from .fr import bls_fr_mont
    _need(blinded_z, 32 * nz, "blinded Z")
    _need(s3, 32 * ns3, "S3")
    for q in list(q5) + list(pi2):
        _need(q, 32 * nq, "selector")
    qa = (ctypes.c_void_p * 5)(*[ptr(x).value for x in q5])
    pa = (ctypes.c_void_p * max(1, len(pi2)))(*[ptr(x).value for x in pi2]) if pi2 else None
    qc = b"".join(bls_fr_mont(v) for v in qcp_zeta) if qcp_zeta else None
    sc = b"".join(bls_fr_mont(v) for v in scalars)
    check(lib.gg_plonk_linearized(ptr(blinded_z), nz, ptr(s3), ns3, qa, nq, pa, ptr(qc), len(pi2),
                                  ptr(sc), ptr(stream)))
