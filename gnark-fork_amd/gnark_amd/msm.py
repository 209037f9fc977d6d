"""Resident MSM bases + multi-scalar multiplication (replaces iciclegnark
CopyPointsToDevice / MsmOnDevice / MsmG2OnDevice, icicle.go:88-126, 302-382,
and G1Jac/G2Jac.MultiExp at prove.go:201-290)."""
from __future__ import annotations

import ctypes

from ._lib import GG_BLS12_381_G1, GG_BLS12_381_G2, GG_G1, GG_G2, check, lib, ptr

G1, G2, BLS12_381_G1, BLS12_381_G2 = GG_G1, GG_G2, GG_BLS12_381_G1, GG_BLS12_381_G2
_JAC = {G1: 96, G2: 192, BLS12_381_G1: 144, BLS12_381_G2: 288}
_AFF = {G1: 64, G2: 128, BLS12_381_G1: 96, BLS12_381_G2: 192}
_TO_AFF = {G1: "gg_g1_jac_to_affine", G2: "gg_g2_jac_to_affine",
           BLS12_381_G1: "gg_bls12_381_g1_jac_to_affine", BLS12_381_G2: "gg_bls12_381_g2_jac_to_affine"}
_ADD = {G1: "gg_g1_jac_add", G2: "gg_g2_jac_add", BLS12_381_G1: "gg_bls12_381_g1_jac_add",
        BLS12_381_G2: "gg_bls12_381_g2_jac_add"}


class MsmBase:
    """n affine points (gnark layout) uploaded once, precomputed, kept in HBM.
    group: G1 / G2 (BN254), BLS12_381_G1 (PlonK KZG commitments, BLS12-381 Groth16)
    or BLS12_381_G2 (BLS12-381 Groth16)."""

    def __init__(self, group: int, points, n: int, on_device=False, scalar_index=None,
                 window_bits: int = 0):
        import numpy as np
        self.group = group
        h = ctypes.c_void_p()
        idx = None
        if scalar_index is not None:
            idx = np.ascontiguousarray(np.asarray(scalar_index, dtype=np.uint32))
        check(lib.gg_msm_base_create(group, ptr(points), n, int(on_device),
                                     ptr(idx), window_bits, ctypes.byref(h)))
        self.handle = h

    def info(self):
        n = ctypes.c_size_t()
        c = ctypes.c_int()
        w = ctypes.c_int()
        check(lib.gg_msm_base_info(self.handle, ctypes.byref(n), ctypes.byref(c), ctypes.byref(w)))
        return n.value, c.value, w.value

    def layout(self):
        """(groups, stored_windows, table_bytes) of the precomputed table."""
        return _layout(lib.gg_msm_base_layout, self.handle)

    def msm_jac(self, scalars, n_scalars: int, on_device=False, stream=None) -> bytes:
        out = bytearray(_JAC[self.group])
        check(lib.gg_msm(self.handle, ptr(scalars), n_scalars, int(on_device), ptr(out), ptr(stream)))
        return bytes(out)

    def msm_stripe_jac(self, scalars, n_scalars: int, stripe_log: int, part: int, on_device=False,
                       stream=None) -> bytes:
        """Bucket stripe `part` of 2^stripe_log of the MSM (gg_msm_stripe): the
        stripes' Jacobian results add up to msm_jac's."""
        out = bytearray(_JAC[self.group])
        check(lib.gg_msm_stripe(self.handle, ptr(scalars), n_scalars, int(on_device), stripe_log, part,
                                ptr(out), ptr(stream)))
        return bytes(out)

    def msm_batch_jac(self, scalar_vectors, n_scalars: int, on_device=False, stream=None) -> list:
        """1..4 MSMs over this base as one (gg_msm_batch: one sort, accumulation
        and reduction; PlonK's same-base commitments): one Jacobian result per
        scalar vector, equal to msm_jac of each."""
        k = len(scalar_vectors)
        outs = [bytearray(_JAC[self.group]) for _ in range(k)]
        keep = [ptr(v) for v in scalar_vectors] + [ptr(o) for o in outs]  # alive across the call
        sv = (ctypes.c_void_p * k)(*[p.value if p is not None else None for p in keep[:k]])
        ov = (ctypes.c_void_p * k)(*[p.value for p in keep[k:]])
        check(lib.gg_msm_batch(self.handle, sv, k, n_scalars, int(on_device), ov, ptr(stream)))
        return [bytes(o) for o in outs]

    def msm(self, scalars, n_scalars: int, on_device=False, stream=None) -> bytes:
        """Affine result (Montgomery, gnark layout; infinity = zeros)."""
        return jac_to_affine(self.group, self.msm_jac(scalars, n_scalars, on_device, stream))

    def close(self):
        if self.handle:
            lib.gg_msm_base_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def jac_to_affine(group: int, jac: bytes) -> bytes:
    out = bytearray(_AFF[group])
    check(getattr(lib, _TO_AFF[group])(ptr(jac), ptr(out)))
    return bytes(out)


def jac_add(group: int, a: bytes, b: bytes) -> bytes:
    out = bytearray(_JAC[group])
    check(getattr(lib, _ADD[group])(ptr(a), ptr(b), ptr(out)))
    return bytes(out)


def scalar_mul(group: int, p_aff: bytes, k_mont: bytes) -> bytes:
    out = bytearray(_JAC[group])
    fn = {G1: lib.gg_g1_scalar_mul, G2: lib.gg_g2_scalar_mul,
          BLS12_381_G1: lib.gg_bls12_381_g1_scalar_mul, BLS12_381_G2: lib.gg_bls12_381_g2_scalar_mul}[group]
    check(fn(ptr(p_aff), ptr(k_mont), ptr(out)))
    return bytes(out)


def batch_scalar_mul(group: int, base_aff: bytes, scalars, n: int, scalars_on_device=False,
                     out=None):
    """out[i] = k_i * base (curve.BatchScalarMultiplicationG1/G2, setup.go:240-318).
    Returns host bytes unless `out` (a device buffer) is given."""
    if out is not None:
        check(lib.gg_batch_scalar_mul(group, ptr(base_aff), ptr(scalars), n,
                                      int(scalars_on_device), ptr(out), 1))
        return out
    res = bytearray(_AFF[group] * n)
    check(lib.gg_batch_scalar_mul(group, ptr(base_aff), ptr(scalars), n, int(scalars_on_device),
                                  ptr(res), 0))
    return bytes(res)


def _layout(fn, *args):
    g, w, b = ctypes.c_int(), ctypes.c_int(), ctypes.c_size_t()
    check(fn(*args, ctypes.byref(g), ctypes.byref(w), ctypes.byref(b)))
    return g.value, w.value, b.value


def set_hbm_budget(nbytes: int) -> None:
    """Cap (bytes per device) on what new precomputed tables may take; 0 = the
    free HBM less a reserve.  Keys built afterwards pick their precompute groups
    (gg_msm_base_layout) to fit it."""
    check(lib.gg_set_hbm_budget(int(nbytes)))


def get_hbm_budget() -> int:
    return int(lib.gg_get_hbm_budget())
