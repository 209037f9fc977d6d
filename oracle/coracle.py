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
