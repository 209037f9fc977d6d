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
