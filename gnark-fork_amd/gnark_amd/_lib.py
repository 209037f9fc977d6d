"""ctypes binding of libgnark_amd.so (include/gnark_amd.h).

The HIP library is the product: there is no CPU fallback.  If the shared
object is missing or cannot be loaded this module raises immediately.
"""
from __future__ import annotations

import ctypes
import os

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("GNARK_AMD_LIB", os.path.join(_PKG_DIR, "lib", "libgnark_amd.so"))

GG_OK = 0
GG_BUILD_ACCUM_PROBE = 1  # gg_build_flags(): a traffic-attribution build, MSM sums wrong by design
GG_REHEARSAL = 7  # a multi-GPU timing rehearsal: the proof written is not valid
GG_ERR_UNSUPPORTED = 4
GG_ERR_TIMEOUT = 8  # a host wait of the library passed its deadline (gg_set_wait_timeout)
GG_MPK_TIMING_SLOTS = 18
GG_PLONK_PART_SLOTS = 14
GG_G1, GG_G2, GG_BLS12_381_G1, GG_BLS12_381_G2 = 1, 2, 3, 4
GG_CURVE_BN254, GG_CURVE_BLS12_381 = 0, 1
PEER_ACCESS = {0: "same_device", 1: "enabled", 2: "unavailable", 3: "enable_failed"}  # GG_PEER_*
GG_DIF, GG_DIT = 0, 1


# gg_exchange_fn (include/gnark_amd.h): all-to-all supplied by the caller
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_size_t)


# gg_hash_fn / gg_g1_reduce_fn (include/gnark_amd.h): PlonK transcript hash, KZG partial reduce
HASH_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                           ctypes.POINTER(ctypes.c_size_t))
REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)


class GnarkAmdError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"gnark_amd error {code}: {msg}")
        self.code = code


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libgnark_amd.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    PP = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "gg_last_error": ([], ctypes.c_char_p),
        "gg_version": ([], I),
        "gg_build_flags": ([], I),
        "gg_device_count": ([ctypes.POINTER(I)], I),
        "gg_set_device": ([I], I),
        "gg_malloc": ([PP, S], I),
        "gg_free": ([P], I),
        "gg_copy_to_device": ([P, P, S], I),
        "gg_copy_to_host": ([P, P, S], I),
        "gg_synchronize": ([], I),
        "gg_copy_device": ([P, P, S], I),
        "gg_fr_from_canonical_be": ([I, P, P, S, ctypes.POINTER(ctypes.c_uint64), P], I),
        "gg_fr_to_canonical_be": ([I, P, P, S, P], I),
        "gg_memset_device": ([P, I, S], I),
        "gg_bls12_381_fr_bit_reverse": ([P, P, S, P], I),
        "gg_bls12_381_fr_axpy": ([P, P, S, P, P], I),
        "gg_domain_create": ([I, P, P, PP], I),
        "gg_domain_create_ex": ([I, I, P, P, PP], I),
        "gg_domain_release": ([P], I),
        "gg_domain_log_n": ([P, ctypes.POINTER(I)], I),
        "gg_ntt": ([P, P, I, I, I, P], I),
        "gg_groth16_compute_h": ([P, P, P, P, S, I, P, P], I),
        "gg_msm_base_create": ([I, P, S, I, P, I, PP], I),
        "gg_msm_base_release": ([P], I),
        "gg_msm_base_info": ([P, ctypes.POINTER(S), ctypes.POINTER(I), ctypes.POINTER(I)], I),
        "gg_msm_base_layout": ([P, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(S)], I),
        "gg_groth16_pk_base_layout": ([P, I, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(S)], I),
        "gg_set_hbm_budget": ([S], I),
        "gg_get_hbm_budget": ([], S),
        "gg_msm": ([P, P, S, I, P, P], I),
        "gg_msm_stripe": ([P, P, S, I, I, I, P, P], I),
        "gg_msm_batch": ([P, P, I, S, I, P, P], I),
        "gg_msm_batch_shape": ([S, I, I, I, I], I),
        "gg_set_wait_timeout": ([ctypes.c_double], I),
        "gg_get_wait_timeout": ([], ctypes.c_double),
        "gg_wait_selftest": ([I, I, ctypes.c_double], I),
        "gg_wait_selftest_device": ([ctypes.c_uint32, ctypes.c_double], I),
        "gg_task_selftest": ([I], I),
        "gg_release_task_queues": ([], I),
        "gg_groth16_pk_create_stripe_ex": ([I, I, P, P, P, S, P, S, P, S, S, P, S, P, P, P, P, P, P, P, P, S,
                                            S, P, I, I, PP], I),
        "gg_groth16_pk_stripe": ([P, ctypes.POINTER(I), ctypes.POINTER(I)], I),
        "gg_groth16_mpk_split": ([P, ctypes.POINTER(I)], I),
        "gg_g1_jac_to_affine": ([P, P], I),
        "gg_g2_jac_to_affine": ([P, P], I),
        "gg_g1_jac_add": ([P, P, P], I),
        "gg_g2_jac_add": ([P, P, P], I),
        "gg_g1_scalar_mul": ([P, P, P], I),
        "gg_g2_scalar_mul": ([P, P, P], I),
        "gg_bls12_381_g1_jac_to_affine": ([P, P], I),
        "gg_bls12_381_g1_jac_add": ([P, P, P], I),
        "gg_bls12_381_g1_scalar_mul": ([P, P, P], I),
        "gg_groth16_pk_create": ([I, P, P, P, S, P, S, P, S, P, S, P, P, P, P, P, P, P, P, S, S, P, PP], I),
        "gg_groth16_pk_release": ([P], I),
        "gg_groth16_pk_create_ex": ([I, I, P, P, P, S, P, S, P, S, P, S, P, P, P, P, P, P, P, P, S, S, P, PP], I),
        "gg_groth16_finalize_ex": ([I, P, P, P, P, P, P, P, P, P, P, P], I),
        "gg_groth16_finalize_begin": ([I, P, P, P, P, PP], I),
        "gg_groth16_finalize_end": ([P, P, P, P, P, P, P, P], I),
        "gg_bls12_381_g2_jac_to_affine": ([P, P], I),
        "gg_bls12_381_g2_jac_add": ([P, P, P], I),
        "gg_bls12_381_g2_scalar_mul": ([P, P, P], I),
        "gg_groth16_prove": ([P, P, S, P, P, P, S, I, P, P, P, P, P, P], I),
        "gg_groth16_last_timings": ([ctypes.POINTER(ctypes.c_double)], I),
        "gg_groth16_last_timings_ex": ([ctypes.POINTER(ctypes.c_double), I], I),
        "gg_groth16_pk_base_info": ([P, I, P, P, P], I),
        "gg_groth16_pk_create_shard": ([I, P, P, P, S, P, S, P, S, S, P, S, P, P, P, P, P, P, P, P, S,
                                        S, P, S, S, PP], I),
        "gg_groth16_prove_partial": ([P, P, S, P, P, P, S, I, P, P], I),
        "gg_groth16_finalize": ([P, P, P, P, P, P, P, P, P, P, P], I),
        "gg_plonk_ratio_copy_constraint": ([P, P, P, P, S, P, P, P, P, P, P], I),
        "gg_bls12_381_fr_prefix_product": ([P, S, P], I),
        "gg_bls12_381_fr_horner": ([P, S, P, P, P, P], I),
        "gg_fr_evaluate_many": ([I, PP, ctypes.POINTER(S), I, P, P, P], I),
        "gg_plonk_fold_h": ([P, S, P, P, P], I),
        "gg_plonk_linearized": ([P, S, P, S, ctypes.POINTER(ctypes.c_void_p), S,
                                 ctypes.POINTER(ctypes.c_void_p), P, I, P, P], I),
        "gg_hshard_create": ([I, P, P, I, I, PP], I),
        "gg_hshard_create_ex": ([I, I, P, P, I, I, PP], I),
        "gg_hshard_exchange_bytes": ([P, I, ctypes.POINTER(S)], I),
        "gg_hshard_release": ([P], I),
        "gg_hshard_info": ([P, ctypes.POINTER(S), ctypes.POINTER(S)], I),
        "gg_hshard_phase": ([P, I, P, P, P, S, I, P, P, P], I),
        "gg_groth16_prove_partial_dist": ([P, P, P, S, P, P, P, S, I, EXCHANGE_FN, P, P, P, P], I),
        "gg_groth16_mpk_create": ([I, P, P, P, S, P, S, P, S, P, S, P, P, P, P, P, P, P, P, S, S, P, I,
                                   ctypes.POINTER(ctypes.c_int), PP], I),
        "gg_groth16_mpk_create_ex": ([I, I, P, P, P, S, P, S, P, S, P, S, P, P, P, P, P, P, P, P, S, S, P, I,
                                      ctypes.POINTER(ctypes.c_int), PP], I),
        "gg_groth16_mpk_prove_ex": ([P, I, PP, S, PP, PP, PP, S, P, P, P, P, P], I),
        "gg_groth16_mpk_devices": ([P, ctypes.POINTER(ctypes.c_int), I], I),
        "gg_groth16_mpk_base_info": ([P, I, I, P, P, P], I),
        "gg_groth16_pk_create_shard_ex": ([I, I, P, P, P, S, P, S, P, S, S, P, S, P, P, P, P, P, P, P, P, S,
                                           S, P, S, S, PP], I),
        "gg_groth16_mpk_release": ([P], I),
        "gg_groth16_mpk_info": ([P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], I),
        "gg_groth16_mpk_prove": ([P, P, S, P, P, P, S, P, P, P, P, P], I),
        "gg_groth16_mpk_last_timings": ([P, ctypes.POINTER(ctypes.c_double)], I),
        "gg_groth16_mpk_shard_timings": ([P, I, ctypes.POINTER(ctypes.c_double), I], I),
        "gg_groth16_mpk_set_rehearsal": ([P, I], I),
        "gg_groth16_mpk_peer_access": ([P, ctypes.POINTER(I), I], I),
        "gg_plonk_pk_peer_access": ([P, ctypes.POINTER(I), I, ctypes.POINTER(I)], I),
        "gg_batch_scalar_mul": ([I, P, P, S, I, P, I], I),
        "gg_plonk_numerator_coset": ([ctypes.POINTER(ctypes.c_void_p), I, P, ctypes.POINTER(I), P,
                                      P, P, P, P, S, I, I, P, P], I),
        "gg_plonk_divide_by_xn_minus_one": ([P, S, P, P], I),
        "gg_bls12_381_fr_batch_invert": ([P, S, P], I),
        "gg_plonk_pk_create": ([I, I, P, P, P, P, S, P, PP, PP, I, P, S, P, P, PP], I),
        "gg_plonk_pk_create_shard": ([I, I, P, P, P, P, S, P, PP, PP, I, P, S, P, P, I, I, REDUCE_FN, P, PP], I),
        "gg_plonk_pk_create_multi": ([I, I, P, P, P, P, S, P, PP, PP, I, P, S, P, P, I,
                                      ctypes.POINTER(ctypes.c_int), PP], I),
        "gg_plonk_pk_devices": ([P, ctypes.POINTER(ctypes.c_int), I, ctypes.POINTER(ctypes.c_int)], I),
        "gg_plonk_pk_set_rehearsal": ([P, I], I),
        "gg_plonk_pk_set_rehearsal_part": ([P, I], I),
        "gg_plonk_pk_part_timings": ([P, I, ctypes.POINTER(ctypes.c_double), I], I),
        "gg_plonk_pk_create_ex": ([I, I, I, P, P, P, P, S, P, PP, PP, I, P, S, P, P, I,
                                   ctypes.POINTER(ctypes.c_int), PP], I),
        "gg_plonk_pk_create_shard_ex": ([I, I, I, P, P, P, P, S, P, PP, PP, I, P, S, P, P, I, I, REDUCE_FN, P,
                                         PP], I),
        "gg_plonk_pk_info": ([P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                              ctypes.POINTER(ctypes.c_int)], I),
        "gg_plonk_proof_size_ex": ([I, I], S),
        "gg_plonk_pk_release": ([P], I),
        "gg_plonk_pk_vk": ([P, P, S], I),
        "gg_plonk_commit_lagrange": ([P, P, I, P], I),
        "gg_plonk_proof_size": ([I], S),
        "gg_plonk_prove": ([P, P, P, P, I, P, S, PP, P, P, I, P, HASH_FN, P, HASH_FN, P, P, S], I),
        "gg_plonk_last_timings": ([ctypes.POINTER(ctypes.c_double), I], I),
        "gg_r1cs_create": ([S, S, P, P, P, P, S, P, P, S, PP], I),
        "gg_r1cs_create_ex": ([I, S, S, P, P, P, P, S, P, P, S, PP], I),
        "gg_r1cs_release": ([P], I),
        "gg_r1cs_info": ([P, ctypes.POINTER(S), ctypes.POINTER(S), ctypes.POINTER(S)], I),
        "gg_r1cs_solve": ([P, P, S, I, P, P, P, P, I, ctypes.POINTER(ctypes.c_int64)], I),
        "gg_r1cs_solution_dev": ([P, PP, PP, PP, PP], I),
        "gg_r1cs_set_inputs": ([P, S, S], I),
        "gg_scs_set_inputs": ([P, S, S], I),
        "gg_scs_create": ([I, S, S, S, P, P, P, P, S, P, P, S, PP], I),
        "gg_scs_release": ([P], I),
        "gg_scs_info": ([P, ctypes.POINTER(S), ctypes.POINTER(S), ctypes.POINTER(S)], I),
        "gg_scs_solve": ([P, P, S, I, P, P, P, P, I, ctypes.POINTER(ctypes.c_int64)], I),
        "gg_scs_solution_dev": ([P, PP, PP, PP, PP], I),
        "gg_r1cs_schedule": ([P, ctypes.POINTER(I), ctypes.POINTER(S), ctypes.POINTER(S)], I),
        "gg_scs_schedule": ([P, ctypes.POINTER(I), ctypes.POINTER(S), ctypes.POINTER(S)], I),
        "gg_profile_enable": ([I], I),
        "gg_profile_get": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                            ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)], I),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)  # AttributeError == missing export: fail loudly
        fn.argtypes = args
        fn.restype = res
    return L


lib = _load()


def _release_queues_at_exit():
    # the dedicated queues no key holds any more, while the runtime (and a
    # profiler's hooks) are still up (gg_release_task_queues)
    try:
        lib.gg_release_task_queues()
    except Exception:  # pragma: no cover - exiting anyway
        pass


import atexit  # noqa: E402
atexit.register(_release_queues_at_exit)
# a diagnostic build (GG_BUILD_ACCUM_PROBE: wrong MSM sums) is loaded only when
# asked for by name; its provers return GG_REHEARSAL
BUILD_FLAGS = lib.gg_build_flags()
if BUILD_FLAGS and os.environ.get("GNARK_AMD_ALLOW_PROBE") != "1":
    raise ImportError(f"{LIB_PATH} is a diagnostic build (flags {BUILD_FLAGS}): its MSM sums are wrong; "
                      "set GNARK_AMD_ALLOW_PROBE=1 to load it for traffic attribution")
EXPORTED = [
    "gg_last_error", "gg_version", "gg_build_flags", "gg_device_count", "gg_set_device", "gg_malloc", "gg_free",
    "gg_copy_to_device", "gg_copy_to_host", "gg_synchronize", "gg_domain_create",
    "gg_domain_create_ex", "gg_bls12_381_g1_jac_to_affine", "gg_bls12_381_g1_jac_add",
    "gg_domain_release", "gg_domain_log_n", "gg_ntt", "gg_groth16_compute_h",
    "gg_msm_base_create", "gg_msm_base_release", "gg_msm_base_info", "gg_msm", "gg_msm_base_layout",
    "gg_groth16_pk_base_layout", "gg_set_hbm_budget", "gg_get_hbm_budget",
    "gg_g1_jac_to_affine", "gg_g2_jac_to_affine", "gg_g1_jac_add", "gg_g2_jac_add",
    "gg_g1_scalar_mul", "gg_g2_scalar_mul", "gg_groth16_pk_create", "gg_groth16_pk_release",
    "gg_groth16_prove", "gg_groth16_last_timings", "gg_batch_scalar_mul", "gg_profile_enable",
    "gg_plonk_numerator_coset", "gg_plonk_divide_by_xn_minus_one", "gg_bls12_381_fr_batch_invert",
    "gg_profile_get", "gg_groth16_pk_create_shard", "gg_groth16_prove_partial",
    "gg_groth16_finalize", "gg_hshard_create", "gg_hshard_release", "gg_hshard_info",
    "gg_hshard_phase", "gg_groth16_prove_partial_dist", "gg_plonk_ratio_copy_constraint",
    "gg_bls12_381_fr_prefix_product", "gg_bls12_381_fr_horner", "gg_plonk_fold_h",
    "gg_plonk_linearized", "gg_copy_device", "gg_memset_device", "gg_bls12_381_fr_bit_reverse",
    "gg_bls12_381_fr_axpy", "gg_bls12_381_g1_scalar_mul", "gg_fr_from_canonical_be",
    "gg_fr_to_canonical_be", "gg_groth16_last_timings_ex",
    "gg_groth16_pk_base_info", "gg_plonk_pk_create", "gg_plonk_pk_create_shard", "gg_plonk_pk_release", "gg_plonk_pk_create_multi", "gg_plonk_pk_devices",
    "gg_plonk_pk_create_ex", "gg_plonk_pk_create_shard_ex", "gg_plonk_pk_info", "gg_plonk_proof_size_ex",
    "gg_plonk_pk_vk", "gg_plonk_commit_lagrange", "gg_plonk_proof_size", "gg_plonk_prove",
    "gg_plonk_last_timings", "gg_groth16_pk_create_ex", "gg_groth16_finalize_ex",
    "gg_groth16_finalize_begin", "gg_groth16_finalize_end",
    "gg_bls12_381_g2_jac_to_affine", "gg_bls12_381_g2_jac_add", "gg_bls12_381_g2_scalar_mul",
    "gg_groth16_mpk_create", "gg_groth16_mpk_release", "gg_groth16_mpk_info", "gg_groth16_mpk_prove",
    "gg_groth16_mpk_last_timings", "gg_groth16_mpk_create_ex", "gg_groth16_mpk_prove_ex",
    "gg_groth16_mpk_devices", "gg_groth16_mpk_base_info", "gg_groth16_pk_create_shard_ex", "gg_r1cs_create", "gg_r1cs_create_ex", "gg_r1cs_release", "gg_r1cs_info", "gg_r1cs_solve",
    "gg_r1cs_solution_dev", "gg_scs_create", "gg_scs_release", "gg_scs_info", "gg_scs_solve",
    "gg_scs_solution_dev", "gg_r1cs_set_inputs", "gg_scs_set_inputs", "gg_r1cs_schedule", "gg_scs_schedule",
    "gg_msm_stripe", "gg_msm_batch", "gg_groth16_pk_create_stripe_ex", "gg_groth16_pk_stripe", "gg_groth16_mpk_split",
    "gg_hshard_create_ex", "gg_hshard_exchange_bytes", "gg_groth16_mpk_shard_timings",
    "gg_groth16_mpk_set_rehearsal", "gg_plonk_pk_set_rehearsal", "gg_plonk_pk_set_rehearsal_part",
    "gg_plonk_pk_part_timings", "gg_groth16_mpk_peer_access", "gg_plonk_pk_peer_access",
    "gg_fr_evaluate_many", "gg_msm_batch_shape", "gg_set_wait_timeout", "gg_get_wait_timeout",
    "gg_wait_selftest", "gg_wait_selftest_device", "gg_task_selftest", "gg_release_task_queues",
]


def check(rc):
    if rc != GG_OK:
        msg = lib.gg_last_error()
        raise GnarkAmdError(rc, msg.decode() if msg else "")


def ptr(obj):
    """Pointer to a host or device buffer: bytes/bytearray/numpy/torch/int/None."""
    if obj is None:
        return None
    if isinstance(obj, ctypes.c_void_p):
        return obj
    if isinstance(obj, int):
        return ctypes.c_void_p(obj)
    if hasattr(obj, "data_ptr"):  # torch tensor (device or host)
        return ctypes.c_void_p(obj.data_ptr())
    if hasattr(obj, "ctypes"):  # numpy
        return obj.ctypes.data_as(ctypes.c_void_p)
    if isinstance(obj, bytearray):
        return ctypes.cast((ctypes.c_char * len(obj)).from_buffer(obj), ctypes.c_void_p)
    if isinstance(obj, (bytes, memoryview)):
        return ctypes.cast(ctypes.c_char_p(bytes(obj)), ctypes.c_void_p)
    if isinstance(obj, DeviceBuffer):
        return ctypes.c_void_p(obj.ptr)
    raise TypeError(f"cannot take a pointer of {type(obj)}")


class DeviceBuffer:
    """HBM buffer owned through gg_malloc / gg_free."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        check(lib.gg_malloc(ctypes.byref(p), nbytes))
        self.ptr = p.value
        self.nbytes = nbytes

    @classmethod
    def from_host(cls, data):
        b = cls(len(data))
        check(lib.gg_copy_to_device(ctypes.c_void_p(b.ptr), ptr(data), len(data)))
        return b

    def to_host(self, nbytes=None) -> bytes:
        nbytes = self.nbytes if nbytes is None else nbytes
        out = bytearray(nbytes)
        check(lib.gg_copy_to_host(ptr(out), ctypes.c_void_p(self.ptr), nbytes))
        return bytes(out)

    def free(self):
        if self.ptr:
            lib.gg_free(ctypes.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def device_count() -> int:
    n = ctypes.c_int()
    check(lib.gg_device_count(ctypes.byref(n)))
    return n.value


def profile_enable(on: bool = True):
    check(lib.gg_profile_enable(int(on)))


def profile_get(name: str):
    ms = ctypes.c_double()
    cnt = ctypes.c_int64()
    units = ctypes.c_double()
    check(lib.gg_profile_get(name.encode(), ctypes.byref(ms), ctypes.byref(cnt), ctypes.byref(units)))
    return ms.value, cnt.value, units.value
