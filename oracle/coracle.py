"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of the C restatement (oracle/c/oracle_bn254.c).  Importable only
from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
All buffers are bytes in gnark memory layout (Montgomery, LE limbs).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "liboracle_bn254.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        c_sz, c_p, c_i = ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int
        L.oc_msm_g1.argtypes = [c_p, c_p, c_sz, c_i, c_p]
        L.oc_msm_g2.argtypes = [c_p, c_p, c_sz, c_i, c_p]
        L.oc_g1_batch_mul.argtypes = [c_p, c_p, c_sz, c_i, c_p]
        L.oc_g2_batch_mul.argtypes = [c_p, c_p, c_sz, c_i, c_p]
        L.oc_ntt.argtypes = [c_p, c_i, c_i, c_i, c_i, c_i]
        L.oc_compute_h.argtypes = [c_p, c_p, c_p, c_sz, c_i, c_i, c_p]
        L.oc_groth16_prove.argtypes = [
            c_i, c_p, c_sz, c_p, c_sz, c_p, c_p, c_sz, c_p, c_p, c_p, c_p, c_p, c_p,
            c_p, c_p, c_p, c_sz, c_sz, c_p, c_p, c_p, c_sz, c_p, c_p, c_i, c_p, c_p, c_p, c_p]
        L.oc_g1_add.argtypes = [c_p, c_p, c_p]
        L.oc_r1cs_create_mimc.argtypes = [c_sz, c_sz, c_sz]
        L.oc_r1cs_create_mimc.restype = c_p
        L.oc_r1cs_free.argtypes = [c_p]
        L.oc_r1cs_info.argtypes = [c_p, c_p, c_p, c_p]
        L.oc_r1cs_solve.argtypes = [c_p, c_p, c_p]
        L.oc_r1cs_abc.argtypes = [c_p, c_p, c_p, c_p, c_p, c_i]
        L.oc_r1cs_abc.restype = ctypes.c_long
        L.oc_groth16_key_scalars.argtypes = [c_p, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                             c_p, c_p, c_i]
        L.oc_groth16_expected.argtypes = [c_p, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i]
        L.oc_eval_bitrev.argtypes = [c_p, c_i, c_p, c_p, c_i]
        L.oc_eval_lagrange.argtypes = [c_p, c_sz, c_i, c_p, c_p, c_i]
        L.oc_fr_dot.argtypes = [c_p, c_p, c_sz, c_p, c_i]
        _lib = L
    return _lib


def _buf(b):
    if b is None:
        return None
    if isinstance(b, (bytes, bytearray)):
        return ctypes.c_char_p(bytes(b)) if isinstance(b, bytes) else (ctypes.c_char * len(b)).from_buffer(b)
    return b


def _ptr(b):
    """Return a ctypes pointer for bytes / bytearray / numpy arrays."""
    if b is None:
        return None
    if hasattr(b, "ctypes"):
        return b.ctypes.data_as(ctypes.c_void_p)
    if isinstance(b, bytearray):
        return ctypes.cast((ctypes.c_char * len(b)).from_buffer(b), ctypes.c_void_p)
    return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p)


def msm_g1(points: bytes, scalars: bytes, n: int, nthreads: int = 0) -> bytes:
    out = bytearray(64)
    lib().oc_msm_g1(_ptr(points), _ptr(scalars), n, nthreads, _ptr(out))
    return bytes(out)


def msm_g2(points: bytes, scalars: bytes, n: int, nthreads: int = 0) -> bytes:
    out = bytearray(128)
    lib().oc_msm_g2(_ptr(points), _ptr(scalars), n, nthreads, _ptr(out))
    return bytes(out)


def g1_batch_mul(base: bytes, scalars: bytes, n: int, nthreads: int = 0) -> bytearray:
    out = bytearray(64 * n)
    lib().oc_g1_batch_mul(_ptr(base), _ptr(scalars), n, nthreads, _ptr(out))
    return out


def g2_batch_mul(base: bytes, scalars: bytes, n: int, nthreads: int = 0) -> bytearray:
    out = bytearray(128 * n)
    lib().oc_g2_batch_mul(_ptr(base), _ptr(scalars), n, nthreads, _ptr(out))
    return out


def ntt(data: bytes, log_n: int, inverse: bool, dif: bool, coset: bool, nthreads: int = 0) -> bytes:
    buf = bytearray(data)
    lib().oc_ntt(_ptr(buf), log_n, int(inverse), int(dif), int(coset), nthreads)
    return bytes(buf)


def compute_h(a: bytes, b: bytes, c: bytes, length: int, log_n: int, nthreads: int = 0) -> bytes:
    out = bytearray(32 << log_n)
    rc = lib().oc_compute_h(_ptr(a), _ptr(b), _ptr(c), length, log_n, nthreads, _ptr(out))
    assert rc == 0
    return bytes(out)


def g1_add(a: bytes, b: bytes) -> bytes:
    out = bytearray(64)
    lib().oc_g1_add(_ptr(a), _ptr(b), _ptr(out))
    return bytes(out)


def groth16_prove(log_n, g1A, nA, g1B, nB, g1Z, g1K, nK, alpha1, beta1, delta1,
                  g2B, beta2, delta2, infA, infB, wires, nWires, nbPublic,
                  solA, solB, solC, nCons, r, s, nthreads=0, want_h=False):
    ar, bs, krs = bytearray(64), bytearray(128), bytearray(64)
    h = bytearray(32 << log_n) if want_h else None
    rc = lib().oc_groth16_prove(
        log_n, _ptr(g1A), nA, _ptr(g1B), nB, _ptr(g1Z), _ptr(g1K), nK,
        _ptr(alpha1), _ptr(beta1), _ptr(delta1), _ptr(g2B), _ptr(beta2), _ptr(delta2),
        _ptr(infA), _ptr(infB), _ptr(wires), nWires, nbPublic,
        _ptr(solA), _ptr(solB), _ptr(solC), nCons, _ptr(r), _ptr(s), nthreads,
        _ptr(ar), _ptr(bs), _ptr(krs), _ptr(h))
    if rc != 0:
        raise RuntimeError(f"oc_groth16_prove failed: {rc}")
    return bytes(ar), bytes(bs), bytes(krs), (bytes(h) if want_h else None)


# ------------------------------------------------------------------ R1CS
class MimcR1CS:
    """Synthetic MiMC x^5 chain R1CS (oracle/c/oracle_r1cs.c): nb_chains chains of
    `rounds` rounds (3 constraints each); wire 0 = ONE, wires 1..nb_chains the
    chain inputs (the first nb_public_inputs public)."""

    def __init__(self, nb_chains: int, rounds: int, nb_public_inputs: int = 0):
        self.h = lib().oc_r1cs_create_mimc(nb_chains, rounds, nb_public_inputs)
        if not self.h:
            raise ValueError("bad MiMC R1CS shape")
        a, b, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        lib().oc_r1cs_info(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        self.ncons, self.nw, self.nb_public = a.value, b.value, c.value
        self.nb_chains = nb_chains

    def solve(self, inputs: bytes) -> bytearray:
        """wires (Montgomery) from the nb_chains chain inputs (Montgomery)."""
        assert len(inputs) == 32 * self.nb_chains
        w = bytearray(32 * self.nw)
        if lib().oc_r1cs_solve(self.h, _ptr(inputs), _ptr(w)) != 0:
            raise RuntimeError("solve failed")
        return w

    def abc(self, wires, nthreads: int = 0):
        """(A, B, C, n_unsatisfied): the solution vectors (solver.go:532-560)."""
        A, B, C = (bytearray(32 * self.ncons) for _ in range(3))
        bad = lib().oc_r1cs_abc(self.h, _ptr(wires), _ptr(A), _ptr(B), _ptr(C), nthreads)
        return A, B, C, bad

    def key_scalars(self, log_n, tau, alpha, beta, delta, nthreads: int = 0):
        """Discrete logs of the proving key in pk order (setup.go:212-275)."""
        n = 1 << log_n
        infA, infB = bytearray(self.nw), bytearray(self.nw)
        A, B = bytearray(32 * self.nw), bytearray(32 * self.nw)
        K = bytearray(32 * (self.nw - self.nb_public))
        Z = bytearray(32 * (n - 1))
        nA, nB = ctypes.c_size_t(), ctypes.c_size_t()
        rc = lib().oc_groth16_key_scalars(self.h, log_n, _ptr(tau), _ptr(alpha), _ptr(beta), _ptr(delta),
                                          _ptr(infA), _ptr(infB), _ptr(A), ctypes.byref(nA), _ptr(B),
                                          ctypes.byref(nB), _ptr(K), _ptr(Z), nthreads)
        if rc != 0:
            raise RuntimeError("key_scalars failed")
        return dict(infA=bytes(infA), infB=bytes(infB), A=bytes(A[:32 * nA.value]),
                    B=bytes(B[:32 * nB.value]), K=bytes(K), Z=bytes(Z))

    def expected(self, log_n, tau, alpha, beta, delta, wires, r, s, nthreads: int = 0):
        """Discrete logs (a, b, c) of (Ar, Bs, Krs), 32-B Montgomery each."""
        out = bytearray(96)
        rc = lib().oc_groth16_expected(self.h, log_n, _ptr(tau), _ptr(alpha), _ptr(beta), _ptr(delta),
                                       _ptr(wires), _ptr(r), _ptr(s), _ptr(out), nthreads)
        if rc != 0:
            raise RuntimeError("expected failed")
        return bytes(out[:32]), bytes(out[32:64]), bytes(out[64:])

    def close(self):
        if self.h:
            lib().oc_r1cs_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def eval_bitrev(coeffs: bytes, log_n: int, x: bytes, nthreads: int = 0) -> bytes:
    out = bytearray(32)
    lib().oc_eval_bitrev(_ptr(coeffs), log_n, _ptr(x), _ptr(out), nthreads)
    return bytes(out)


def eval_lagrange(vals: bytes, length: int, log_n: int, x: bytes, nthreads: int = 0) -> bytes:
    out = bytearray(32)
    lib().oc_eval_lagrange(_ptr(vals), length, log_n, _ptr(x), _ptr(out), nthreads)
    return bytes(out)


def fr_dot(a, b, n: int, nthreads: int = 0) -> bytes:
    """sum_i a_i b_i (fr Montgomery bytes)."""
    out = bytearray(32)
    lib().oc_fr_dot(_ptr(a), _ptr(b), n, _ptr(out), nthreads)
    return bytes(out)
