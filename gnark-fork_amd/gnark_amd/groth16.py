"""Groth16 BN254 on MI355X: mirror of gnark's icicle_bn254 package
(backend/groth16/bn254/icicle/{icicle.go,provingkey.go}).

    pk_dev = ProvingKey(pk_data)                      # setupDevicePointers, once
    proof  = prove(pk_dev, solution, opts=[with_amd_acceleration()])

``solution`` is the output of gnark's R1CS solver (cs.R1CSSolution{W, A, B, C},
constraint/bn254/system.go:269-272); the solver itself is out of scope (host
feeder).  As in icicle.go:141-143 the accelerated prover is only taken when the
accelerator option is set; there is no CPU prover in this package, so a call
without it raises instead of silently computing elsewhere.
"""
from __future__ import annotations

import ctypes
import dataclasses
import secrets
import struct
from typing import Optional, Sequence

import numpy as np

from . import backend, fr
from ._lib import check, lib, ptr

HasAMD = True  # mirrors icicle_bn254.HasIcicle (noicicle.go:16 / icicle.go:29)


@dataclasses.dataclass
class ProvingKeyData:
    """Host copy of groth16_bn254.ProvingKey (setup.go:35-58), gnark byte layouts."""
    log_n: int
    g1_A: bytes
    g1_B: bytes
    g1_Z: bytes
    g1_K: bytes
    alpha1: bytes
    beta1: bytes
    delta1: bytes
    g2_B: bytes
    beta2: bytes
    delta2: bytes
    infinity_A: bytes  # n_wires bytes (1 = infinity)
    infinity_B: bytes
    nb_public: int
    domain_generator: Optional[bytes] = None        # pk.Domain.Generator (Montgomery)
    domain_mul_gen: Optional[bytes] = None          # pk.Domain.FrMultiplicativeGen
    k_wire_index: Optional[Sequence[int]] = None    # filterHeap result; None = nb_public + i

    @property
    def n_wires(self):
        return len(self.infinity_A)


@dataclasses.dataclass
class Solution:
    """cs.R1CSSolution: W (wires), A, B, C (per-constraint L.w, R.w, O.w)."""
    W: object
    A: object
    B: object
    C: object
    n_wires: int
    n_constraints: int
    on_device: bool = False


@dataclasses.dataclass
class Proof:
    """groth16_bn254.Proof (prove.go:45-50): affine points, gnark memory layout."""
    Ar: bytes
    Bs: bytes
    Krs: bytes

    def write_raw(self) -> bytes:
        """WriteRawTo (marshal.go:41-66): Ar | Bs | Krs | Commitments | CommitmentPok,
        uncompressed; no commitments -> u32 length 0 and an infinity PoK [ext enc]."""
        return (fr.g1_raw(self.Ar) + fr.g2_raw(self.Bs) + fr.g1_raw(self.Krs)
                + struct.pack(">I", 0) + fr.g1_raw(bytes(64)))


class ProvingKey:
    """icicle_bn254.ProvingKey {ProvingKey; *deviceInfo}: device-resident key."""

    def __init__(self, data: ProvingKeyData):
        self.data = data
        n_wires = data.n_wires
        nA, nB = len(data.g1_A) // 64, len(data.g1_B) // 64
        nZ, nK = len(data.g1_Z) // 64, len(data.g1_K) // 64
        omega = data.domain_generator or fr.fr_mont(fr.domain_generator(data.log_n))
        gen = data.domain_mul_gen or fr.fr_mont(fr.FR_MULTIPLICATIVE_GEN)
        kidx = None
        if data.k_wire_index is not None:
            kidx = np.ascontiguousarray(np.asarray(data.k_wire_index, dtype=np.uint32))
        h = ctypes.c_void_p()
        check(lib.gg_groth16_pk_create(
            data.log_n, ptr(omega), ptr(gen),
            ptr(data.g1_A), nA, ptr(data.g1_B), nB, ptr(data.g1_Z), nZ, ptr(data.g1_K), nK,
            ptr(data.alpha1), ptr(data.beta1), ptr(data.delta1),
            ptr(data.g2_B), ptr(data.beta2), ptr(data.delta2),
            ptr(bytes(data.infinity_A)), ptr(bytes(data.infinity_B)), n_wires, data.nb_public,
            ptr(kidx), ctypes.byref(h)))
        self.handle = h
        self.n_wires = n_wires
        self.log_n = data.log_n

    def close(self):
        if self.handle:
            lib.gg_groth16_pk_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _rand_fr_mont() -> bytes:
    # fr.Element.SetRandom (prove.go:180-185)
    return fr.fr_mont(secrets.randbelow(fr.R))


def prove(pk: ProvingKey, solution: Solution, *opts, r: bytes = None, s: bytes = None,
          h_out=None) -> Proof:
    """icicle_bn254.Prove after Solve (icicle.go:198-422)."""
    cfg = backend.new_prover_config(*opts)
    if not backend.accelerated(cfg):
        raise RuntimeError("accelerated prover requested without with_amd_acceleration(); "
                           "the CPU prover is gnark's groth16_bn254.Prove (prove.go:63)")
    r = r if r is not None else _rand_fr_mont()
    s = s if s is not None else _rand_fr_mont()
    ar, bs, krs = bytearray(64), bytearray(128), bytearray(64)
    check(lib.gg_groth16_prove(pk.handle, ptr(solution.W), solution.n_wires, ptr(solution.A),
                               ptr(solution.B), ptr(solution.C), solution.n_constraints,
                               int(solution.on_device), ptr(r), ptr(s), ptr(ar), ptr(bs),
                               ptr(krs), ptr(h_out)))
    return Proof(bytes(ar), bytes(bs), bytes(krs))


def last_timings() -> dict:
    arr = (ctypes.c_double * 9)()
    check(lib.gg_groth16_last_timings(arr))
    keys = ["upload", "compute_h", "msm_A", "msm_B1", "msm_K", "msm_Z", "msm_G2", "epilogue", "total"]
    return dict(zip(keys, list(arr)))
