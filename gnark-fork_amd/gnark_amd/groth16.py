"""Groth16 (BN254, BLS12-381) on MI355X: mirror of gnark's icicle_bn254 package
(backend/groth16/bn254/icicle/{icicle.go,provingkey.go}); ProvingKeyData(curve=
"bls12-381") is backend/groth16/bls12-381's key (same prover over BLS12-381).

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
from . import dist as gdist
from ._lib import BUILD_FLAGS, check, lib, ptr, GG_CURVE_BN254, GG_CURVE_BLS12_381, GG_MPK_TIMING_SLOTS, GG_REHEARSAL

# (G1 affine, G2 affine) bytes per curve
_SIZES = {"bn254": (64, 128), "bls12-381": (96, 192)}

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
    curve: str = "bn254"                            # or "bls12-381"
    commitment_keys: Optional[Sequence] = None      # pk.CommitmentKeys (pedersen.ProvingKey), BN254

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
    """groth16_bn254.Proof (prove.go:45-50): affine points, gnark memory layout;
    Commitments / CommitmentPok are set by BSB22 circuits (pedersen.Bsb22Hints)."""
    Ar: bytes
    Bs: bytes
    Krs: bytes
    Commitments: Sequence[bytes] = ()
    CommitmentPok: bytes = bytes(64)

    def write_raw(self) -> bytes:
        """WriteRawTo (marshal.go:41-66): Ar | Bs | Krs | u32 len(Commitments) |
        Commitments | CommitmentPok, uncompressed (infinity PoK without commitments)."""
        return (fr.g1_raw(self.Ar) + fr.g2_raw(self.Bs) + fr.g1_raw(self.Krs)
                + struct.pack(">I", len(self.Commitments)) + b"".join(fr.g1_raw(c) for c in self.Commitments)
                + fr.g1_raw(self.CommitmentPok))


BASE_A, BASE_B1, BASE_K, BASE_Z, BASE_B2 = range(5)


class ProvingKey:
    """icicle_bn254.ProvingKey {ProvingKey; *deviceInfo}: device-resident key."""

    def __init__(self, data: ProvingKeyData):
        self.data = data
        n_wires = data.n_wires
        self.curve = data.curve
        g1b, self.g2b = _SIZES[data.curve]
        self.g1b = g1b
        nA, nB = len(data.g1_A) // g1b, len(data.g1_B) // g1b
        nZ, nK = len(data.g1_Z) // g1b, len(data.g1_K) // g1b
        if data.curve == "bn254":
            cid = GG_CURVE_BN254
            omega = data.domain_generator or fr.fr_mont(fr.domain_generator(data.log_n))
            gen = data.domain_mul_gen or fr.fr_mont(fr.FR_MULTIPLICATIVE_GEN)
        else:
            cid = GG_CURVE_BLS12_381
            omega = data.domain_generator or fr.bls_fr_mont(fr.bls_domain_generator(data.log_n))
            gen = data.domain_mul_gen or fr.bls_fr_mont(fr.BLS_FR_MULTIPLICATIVE_GEN)
        kidx = None
        if data.k_wire_index is not None:
            kidx = np.ascontiguousarray(np.asarray(data.k_wire_index, dtype=np.uint32))
        h = ctypes.c_void_p()
        check(lib.gg_groth16_pk_create_ex(
            cid, data.log_n, ptr(omega), ptr(gen),
            ptr(data.g1_A), nA, ptr(data.g1_B), nB, ptr(data.g1_Z), nZ, ptr(data.g1_K), nK,
            ptr(data.alpha1), ptr(data.beta1), ptr(data.delta1),
            ptr(data.g2_B), ptr(data.beta2), ptr(data.delta2),
            ptr(bytes(data.infinity_A)), ptr(bytes(data.infinity_B)), n_wires, data.nb_public,
            ptr(kidx), ctypes.byref(h)))
        self.handle = h
        self.n_wires = n_wires
        self.log_n = data.log_n
        # pk.CommitmentKeys: both Pedersen bases resident next to the key
        self.commitment_keys = []
        if data.commitment_keys:
            if data.curve != "bn254":
                raise ValueError("BSB22 commitment keys: BN254 only")
            from . import pedersen
            self.commitment_keys = [pedersen.DevicePedersenKey(k) for k in data.commitment_keys]

    def base_info(self, which: int):
        """(resident points, window bits, windows) of MSM base `which` (BASE_*)."""
        n, c, w = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_int()
        check(lib.gg_groth16_pk_base_info(self.handle, which, ctypes.byref(n), ctypes.byref(c),
                                          ctypes.byref(w)))
        return n.value, c.value, w.value

    def base_layout(self, which: int):
        """(groups, stored_windows, table_bytes) of base `which` (0 A, 1 B, 2 K, 3 Z, 4 G2.B)."""
        from .msm import _layout
        return _layout(lib.gg_groth16_pk_base_layout, self.handle, which)

    def close(self):
        for k in getattr(self, "commitment_keys", ()):
            k.close()
        self.commitment_keys = []
        if self.handle:
            lib.gg_groth16_pk_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiGpuProvingKey:
    """One-process multi-GPU key (gg_groth16_mpk_create_ex): shard r of the whole
    key on devices[r] (ids may repeat: several shards per GPU); proofs run one
    host thread per shard with the distributed computeH's all-to-alls done as
    peer copies inside the library -- the shape a Go caller uses, no
    torch.distributed.  BN254 (distributed computeH) or BLS12-381 (computeH on
    every shard, MSMs sharded).  Host inputs, or a solution resident on every
    device (`replicate_solution` / per-device GPU solves)."""

    def __init__(self, data: ProvingKeyData, devices):
        self.data = data
        self.curve = data.curve
        g1b, g2b = _SIZES[data.curve]
        self.g1b, self.g2b = g1b, g2b
        devs = (ctypes.c_int * len(devices))(*devices)
        if data.curve == "bn254":
            cid = GG_CURVE_BN254
            omega = data.domain_generator or fr.fr_mont(fr.domain_generator(data.log_n))
            gen = data.domain_mul_gen or fr.fr_mont(fr.FR_MULTIPLICATIVE_GEN)
        else:
            cid = GG_CURVE_BLS12_381
            omega = data.domain_generator or fr.bls_fr_mont(fr.bls_domain_generator(data.log_n))
            gen = data.domain_mul_gen or fr.bls_fr_mont(fr.BLS_FR_MULTIPLICATIVE_GEN)
        kidx = None
        if data.k_wire_index is not None:
            kidx = np.ascontiguousarray(np.asarray(data.k_wire_index, dtype=np.uint32))
        h = ctypes.c_void_p()
        check(lib.gg_groth16_mpk_create_ex(
            cid, data.log_n, ptr(omega), ptr(gen),
            ptr(data.g1_A), len(data.g1_A) // g1b, ptr(data.g1_B), len(data.g1_B) // g1b,
            ptr(data.g1_Z), len(data.g1_Z) // g1b, ptr(data.g1_K), len(data.g1_K) // g1b,
            ptr(data.alpha1), ptr(data.beta1), ptr(data.delta1),
            ptr(data.g2_B), ptr(data.beta2), ptr(data.delta2),
            ptr(bytes(data.infinity_A)), ptr(bytes(data.infinity_B)), data.n_wires, data.nb_public,
            ptr(kidx), len(devices), devs, ctypes.byref(h)))
        self.handle = h
        self.devices = list(devices)
        self.n_wires = data.n_wires
        self.log_n = data.log_n

    def info(self):
        """(world, distributed computeH?)"""
        w, d = ctypes.c_int(), ctypes.c_int()
        check(lib.gg_groth16_mpk_info(self.handle, ctypes.byref(w), ctypes.byref(d)))
        return w.value, bool(d.value)

    def split(self) -> str:
        """'stripes' (bucket stripes over whole per-device wire tables) or 'wires'."""
        v = ctypes.c_int()
        check(lib.gg_groth16_mpk_split(self.handle, ctypes.byref(v)))
        return "stripes" if v.value else "wires"

    def base_info(self, which: int, shard: int = 0):
        """(resident points, window bits, windows) of MSM base `which` of a shard"""
        n, c, w = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_int()
        check(lib.gg_groth16_mpk_base_info(self.handle, shard, which, ctypes.byref(n), ctypes.byref(c),
                                           ctypes.byref(w)))
        return n.value, c.value, w.value

    def shard_devices(self):
        """device id of every shard (gg_groth16_mpk_devices)"""
        arr = (ctypes.c_int * len(self.devices))()
        check(lib.gg_groth16_mpk_devices(self.handle, arr, len(self.devices)))
        return list(arr)

    def set_rehearsal(self, solo_shard: int = -1):
        """Timing rehearsal (gg_groth16_mpk_set_rehearsal): solo_shard >= 0 makes
        later proves run that shard ALONE (the per-GPU work of an N-GPU node on
        one GPU); those proofs are NOT valid and prove() refuses them unless
        called with rehearsal_ok=True.  -1 restores real proofs."""
        check(lib.gg_groth16_mpk_set_rehearsal(self.handle, int(solo_shard)))
        self._solo = int(solo_shard)

    def peer_access(self) -> list:
        """[i][j]: how shard i's device reaches shard j's ('same_device', 'enabled',
        'unavailable', 'enable_failed'; gg_groth16_mpk_peer_access)"""
        from ._lib import PEER_ACCESS
        w = len(self.devices)
        arr = (ctypes.c_int * (w * w))()
        check(lib.gg_groth16_mpk_peer_access(self.handle, arr, w * w))
        return [[PEER_ACCESS.get(arr[i * w + j], str(arr[i * w + j])) for j in range(w)] for i in range(w)]

    def shard_timings(self) -> list:
        """Per shard, the last proof: prove ms and, per exchange of the distributed
        computeH, the wait at the first barrier, the peer-copy push time, the wait
        at the second barrier and the MB pushed (gg_groth16_mpk_shard_timings)."""
        out = []
        for r in range(len(self.devices)):
            v = (ctypes.c_double * GG_MPK_TIMING_SLOTS)()
            check(lib.gg_groth16_mpk_shard_timings(self.handle, r, v, GG_MPK_TIMING_SLOTS))
            nx = int(v[1])
            ex = [{"wait_before_ms": v[2 + 4 * e], "push_ms": v[3 + 4 * e], "wait_after_ms": v[4 + 4 * e],
                   "pushed_MB": v[5 + 4 * e]} for e in range(nx)]
            out.append({"shard": r, "device": self.devices[r], "prove_ms": v[0], "exchanges": ex})
        return out

    def prove(self, solution, *opts, r: bytes = None, s: bytes = None, rehearsal_ok: bool = False) -> "Proof":
        """`solution`: a host Solution (every shard reads it), or a DeviceSolutions
        (one resident copy per device, see replicate_solution)."""
        cfg = backend.new_prover_config(*opts)
        if not backend.accelerated(cfg):
            raise RuntimeError("accelerated prover requested without with_amd_acceleration()")
        rnd = _rand_fr_mont if self.curve == "bn254" else (lambda: fr.bls_fr_mont(secrets.randbelow(fr.BLS_R)))
        r = r if r is not None else rnd()
        s = s if s is not None else rnd()
        world = len(self.devices)
        if isinstance(solution, DeviceSolutions):
            per = [solution.for_device(d) for d in self.devices]
            on_dev = 1
        elif solution.on_device:
            if len(set(self.devices)) != 1:
                raise ValueError("a device-resident Solution serves one GPU; use replicate_solution(...)")
            per, on_dev = [solution] * world, 1
        else:
            per, on_dev = [solution] * world, 0
        n_wires, n_cons = per[0].n_wires, per[0].n_constraints

        def arr(field):
            return (ctypes.c_void_p * world)(*[ptr(getattr(x, field)).value for x in per])
        ar, bs, krs = bytearray(self.g1b), bytearray(self.g2b), bytearray(self.g1b)
        rc = lib.gg_groth16_mpk_prove_ex(self.handle, on_dev, arr("W"), n_wires, arr("A"), arr("B"), arr("C"),
                                         n_cons, ptr(r), ptr(s), ptr(ar), ptr(bs), ptr(krs))
        if not (rc == GG_REHEARSAL and rehearsal_ok):
            check(rc)
        return Proof(bytes(ar), bytes(bs), bytes(krs))

    def last_timings(self) -> dict:
        t = (ctypes.c_double * 3)()
        check(lib.gg_groth16_mpk_last_timings(self.handle, t))
        return {"shards": t[0], "combine": t[1], "total": t[2]}

    def close(self):
        if self.handle:
            lib.gg_groth16_mpk_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclasses.dataclass
class DeviceSolutions:
    """One HBM-resident copy of a Solution per GPU (device id -> Solution with
    on_device=True), for MultiGpuProvingKey.prove."""
    by_device: dict

    def for_device(self, d):
        if d not in self.by_device:
            raise ValueError("no resident solution on device %d" % d)
        return self.by_device[d]


def replicate_solution(solution: Solution, devices) -> DeviceSolutions:
    """Upload a host Solution once to every distinct device of `devices`."""
    from ._lib import DeviceBuffer
    out = {}
    for d in dict.fromkeys(devices):
        check(lib.gg_set_device(int(d)))
        bufs = [DeviceBuffer.from_host(bytes(getattr(solution, f))) for f in ("W", "A", "B", "C")]
        out[d] = Solution(*bufs, solution.n_wires, solution.n_constraints, on_device=True)
    check(lib.gg_set_device(int(devices[0])))
    return DeviceSolutions(out)


def _rand_fr_mont() -> bytes:
    # fr.Element.SetRandom (prove.go:180-185)
    return fr.fr_mont(secrets.randbelow(fr.R))


def prove(pk: ProvingKey, solution: Solution, *opts, r: bytes = None, s: bytes = None,
          h_out=None, bsb22=None) -> Proof:
    """icicle_bn254.Prove after Solve (icicle.go:198-422).  BSB22 circuits pass
    the solved hints (pedersen.Bsb22Hints): their commitments go into the proof
    and the proof of knowledge is pedersen.BatchProve on the resident bases
    (prove.go:128-136); the key's K points must then exclude the committed and
    commitment wires (k_wire_index = pedersen.k_wire_index(...), prove.go:238-248)."""
    cfg = backend.new_prover_config(*opts)
    if not backend.accelerated(cfg):
        raise RuntimeError("accelerated prover requested without with_amd_acceleration(); "
                           "the CPU prover is gnark's groth16_bn254.Prove (prove.go:63)")
    ncom = len(getattr(pk, "commitment_keys", ()))
    if ncom and (bsb22 is None or len(bsb22.keys) != ncom):
        raise ValueError("key has %d commitment keys: pass the solved pedersen.Bsb22Hints" % ncom)
    if bsb22 is not None and not ncom and bsb22.keys:
        raise ValueError("BSB22 hints for a key without commitment keys")
    rnd = _rand_fr_mont if getattr(pk, "curve", "bn254") == "bn254" else \
        (lambda: fr.bls_fr_mont(secrets.randbelow(fr.BLS_R)))
    r = r if r is not None else rnd()
    s = s if s is not None else rnd()
    g1b, g2b = _SIZES[getattr(pk, "curve", "bn254")]
    ar, bs, krs = bytearray(g1b), bytearray(g2b), bytearray(g1b)
    rc = lib.gg_groth16_prove(pk.handle, ptr(solution.W), solution.n_wires, ptr(solution.A),
                              ptr(solution.B), ptr(solution.C), solution.n_constraints,
                              int(solution.on_device), ptr(r), ptr(s), ptr(ar), ptr(bs),
                              ptr(krs), ptr(h_out))
    if not (rc == GG_REHEARSAL and BUILD_FLAGS):  # a probe build (opted into at import) proves nothing valid
        check(rc)
    if ncom:
        return Proof(bytes(ar), bytes(bs), bytes(krs), list(bsb22.commitments), bsb22.pok())
    return Proof(bytes(ar), bytes(bs), bytes(krs))


def last_timings() -> dict:
    """Per-stage wall times (ms) of this thread's last prove: upload = host staging
    of the wires (before the MSMs start); upload_abc = host staging of A, B, C
    inside the computeH task (overlapped with the MSMs, included in compute_h)."""
    arr = (ctypes.c_double * 12)()
    check(lib.gg_groth16_last_timings_ex(arr, 12))
    keys = ["upload", "compute_h", "msm_A", "msm_B1", "msm_K", "msm_Z", "msm_G2", "epilogue", "total",
            "upload_abc", "t_enter", "t_exit"]
    return dict(zip(keys, list(arr)))


# ---------------------------------------------------------------- multi-GPU
# One key shard per GPU: the MSM point sets partition by wire (A,
# B1, K, G2) and by domain position (Z); every GPU computes h itself, so the
# only cross-GPU traffic is the all-gather of the 576-B partials.

PARTIALS_BYTES = 4 * 96 + 192  # G1Jac A | B1 | K | Z, G2Jac B2


@dataclasses.dataclass
class KeyShard:
    """Slices of a ProvingKeyData owned by one shard (host bytes, key order)."""
    wire_lo: int
    wire_hi: int
    z_lo: int
    g1_A: bytes
    g1_B: bytes
    g2_B: bytes
    g1_K: bytes
    g1_Z: bytes
    k_wire_index: Optional[np.ndarray]  # absolute wire ids of g1_K (None = default numbering)


def dist_h_supported(n: int, world: int) -> bool:
    """The distributed computeH (gg_hshard_*) needs world a power of two <= 16
    and n >= world^2."""
    return 1 <= world <= 16 and world & (world - 1) == 0 and n >= 2 and n >= world * world


def shard_ranges(n_wires: int, n: int, rank: int, world: int):
    """(wire_lo, wire_hi, z_lo, z_hi) of `rank`: contiguous balanced slices of the
    wires; Z positions [rank m, (rank+1) m) (m = n / world, the h block the
    distributed computeH leaves on this rank) when dist_h_supported, else a
    balanced slice of the n - 1 positions."""
    from .dist import shard_range
    lo, hi = shard_range(n_wires, rank, world)
    if dist_h_supported(n, world):
        m = n // world
        zl, zh = min(rank * m, n - 1), min((rank + 1) * m, n - 1)
    else:
        zl, zh = shard_range(max(n - 1, 0), rank, world)
    return lo, hi, zl, zh


def slice_key(data: ProvingKeyData, rank: int, world: int) -> KeyShard:
    """Cut the key arrays of `data` for shard `rank` of `world` (pk order kept:
    A/B are the non-infinity points in wire order, setup.go:259-275)."""
    n = 1 << data.log_n
    lo, hi, zl, zh = shard_ranges(data.n_wires, n, rank, world)
    infA = np.frombuffer(bytes(data.infinity_A), dtype=np.uint8)
    infB = np.frombuffer(bytes(data.infinity_B), dtype=np.uint8)
    a0, a1 = int((infA[:lo] == 0).sum()), int((infA[:hi] == 0).sum())
    b0, b1 = int((infB[:lo] == 0).sum()), int((infB[:hi] == 0).sum())
    if data.k_wire_index is None:
        k0 = max(lo, data.nb_public) - data.nb_public
        k1 = max(hi, data.nb_public) - data.nb_public
        k1 = min(k1, len(data.g1_K) // 64)
        k0 = min(k0, k1)
        g1K, kidx = data.g1_K[64 * k0:64 * k1], None
    else:
        kw = np.asarray(data.k_wire_index, dtype=np.uint32)
        sel = np.nonzero((kw >= lo) & (kw < hi))[0]
        kp = np.frombuffer(bytes(data.g1_K), dtype=np.uint8).reshape(-1, 64)
        g1K, kidx = kp[sel].tobytes(), np.ascontiguousarray(kw[sel])
    return KeyShard(lo, hi, zl, data.g1_A[64 * a0:64 * a1], data.g1_B[64 * b0:64 * b1],
                    data.g2_B[128 * b0:128 * b1], g1K, data.g1_Z[64 * zl:64 * zh], kidx)


class ProvingKeyShard:
    """Device-resident shard `rank` of `world` of a proving key (gg_groth16_pk_create_shard).
    `shard` may be given directly (slices already cut, e.g. generated per GPU)."""

    def __init__(self, data: ProvingKeyData, rank: int = 0, world: int = 1,
                 shard: Optional[KeyShard] = None):
        sh = shard if shard is not None else slice_key(data, rank, world)
        self.data, self.shard, self.rank, self.world = data, sh, rank, world
        omega = data.domain_generator or fr.fr_mont(fr.domain_generator(data.log_n))
        gen = data.domain_mul_gen or fr.fr_mont(fr.FR_MULTIPLICATIVE_GEN)
        h = ctypes.c_void_p()
        check(lib.gg_groth16_pk_create_shard(
            data.log_n, ptr(omega), ptr(gen),
            ptr(sh.g1_A), len(sh.g1_A) // 64, ptr(sh.g1_B), len(sh.g1_B) // 64,
            ptr(sh.g1_Z), sh.z_lo, len(sh.g1_Z) // 64, ptr(sh.g1_K), len(sh.g1_K) // 64,
            ptr(data.alpha1), ptr(data.beta1), ptr(data.delta1),
            ptr(sh.g2_B), ptr(data.beta2), ptr(data.delta2),
            ptr(bytes(data.infinity_A)), ptr(bytes(data.infinity_B)), data.n_wires,
            data.nb_public, ptr(sh.k_wire_index), sh.wire_lo, sh.wire_hi, ctypes.byref(h)))
        self.handle = h
        self.n_wires = data.n_wires
        self.log_n = data.log_n

    base_info = ProvingKey.base_info
    close = ProvingKey.close
    __del__ = ProvingKey.__del__


class ProvingKeyStripe:
    """Bucket-stripe shard `rank` of `world` (a power of two) of a proving key
    (gg_groth16_pk_create_stripe_ex): the WHOLE A, B, K and G2 B tables, whose
    A, B1, K and G2 MSMs this shard computes over the buckets b = rank mod world,
    and the Z slice of shard_ranges (the h block the distributed computeH leaves
    on this rank).  Proves with prove_partial / prove_distributed_h like a
    ProvingKeyShard; the partials of all ranks add up to the proof's.
    g1_Z / z_lo: this rank's Z slice when `data` does not hold the whole Z."""

    def __init__(self, data: ProvingKeyData, rank: int = 0, world: int = 1, g1_Z: bytes = None,
                 z_lo: int = None):
        assert world >= 1 and world & (world - 1) == 0, "world must be a power of two"
        n = 1 << data.log_n
        _, _, zl, zh = shard_ranges(data.n_wires, n, rank, world)
        if g1_Z is None:
            g1_Z, z_lo = data.g1_Z[64 * zl:64 * zh], zl
        assert z_lo == zl and len(g1_Z) == 64 * (zh - zl), "Z slice differs from shard_ranges"
        self.data, self.rank, self.world = data, rank, world
        omega = data.domain_generator or fr.fr_mont(fr.domain_generator(data.log_n))
        gen = data.domain_mul_gen or fr.fr_mont(fr.FR_MULTIPLICATIVE_GEN)
        kidx = None if data.k_wire_index is None else np.ascontiguousarray(data.k_wire_index, dtype=np.uint32)
        h = ctypes.c_void_p()
        check(lib.gg_groth16_pk_create_stripe_ex(
            GG_CURVE_BN254, data.log_n, ptr(omega), ptr(gen),
            ptr(data.g1_A), len(data.g1_A) // 64, ptr(data.g1_B), len(data.g1_B) // 64,
            ptr(g1_Z), z_lo, len(g1_Z) // 64, ptr(data.g1_K), len(data.g1_K) // 64,
            ptr(data.alpha1), ptr(data.beta1), ptr(data.delta1),
            ptr(data.g2_B), ptr(data.beta2), ptr(data.delta2),
            ptr(bytes(data.infinity_A)), ptr(bytes(data.infinity_B)), data.n_wires,
            data.nb_public, ptr(kidx), world.bit_length() - 1, rank, ctypes.byref(h)))
        self.handle = h
        self.n_wires = data.n_wires
        self.log_n = data.log_n

    def stripe(self):
        """(stripe_log, stripe_part) of the key."""
        a, b = ctypes.c_int(), ctypes.c_int()
        check(lib.gg_groth16_pk_stripe(self.handle, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    base_info = ProvingKey.base_info
    close = ProvingKey.close
    __del__ = ProvingKey.__del__


def prove_partial(pk: ProvingKeyShard, solution: Solution, h_out=None) -> bytes:
    """computeH + this shard's five MSMs (gg_groth16_prove_partial): 576-B partials."""
    out = bytearray(PARTIALS_BYTES)
    check(lib.gg_groth16_prove_partial(pk.handle, ptr(solution.W), solution.n_wires,
                                       ptr(solution.A), ptr(solution.B), ptr(solution.C),
                                       solution.n_constraints, int(solution.on_device), ptr(out),
                                       ptr(h_out)))
    return bytes(out)


def add_partials(parts: Sequence[bytes]) -> bytes:
    """Sum of shard partials with the library's exact group law."""
    from . import msm
    acc = bytearray(parts[0])
    for p in parts[1:]:
        for k in range(4):
            acc[96 * k:96 * k + 96] = msm.jac_add(msm.G1, bytes(acc[96 * k:96 * k + 96]), p[96 * k:96 * k + 96])
        acc[384:576] = msm.jac_add(msm.G2, bytes(acc[384:576]), p[384:576])
    return bytes(acc)


class FixedTerms:
    """gg_groth16_finalize_begin / _end: the fixed-point terms of prove.go:177-192
    (r.delta, s.delta, kr.delta, s.delta2) computed on host threads while the
    sharded prove runs; finish() combines them with the summed partials."""

    def __init__(self, data: ProvingKeyData, r: bytes, s: bytes):
        cid = GG_CURVE_BN254 if data.curve == "bn254" else GG_CURVE_BLS12_381
        h = ctypes.c_void_p()
        check(lib.gg_groth16_finalize_begin(cid, ptr(data.delta1), ptr(data.delta2), ptr(r), ptr(s),
                                            ctypes.byref(h)))
        self.data, self.handle = data, h

    def finish(self, partials: bytes) -> Proof:
        g1b, g2b = _SIZES[self.data.curve]
        ar, bs, krs = bytearray(g1b), bytearray(g2b), bytearray(g1b)
        h, self.handle = self.handle, None
        d = self.data
        check(lib.gg_groth16_finalize_end(h, ptr(d.alpha1), ptr(d.beta1), ptr(d.beta2), ptr(partials),
                                          ptr(ar), ptr(bs), ptr(krs)))
        return Proof(bytes(ar), bytes(bs), bytes(krs))

    def close(self):
        if self.handle:
            h, self.handle = self.handle, None
            lib.gg_groth16_finalize_end(h, None, None, None, None, None, None, None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def finalize(data: ProvingKeyData, partials: bytes, r: bytes, s: bytes) -> Proof:
    """Combination of prove.go:177-299 on the summed partials (host, gg_groth16_finalize_ex)."""
    g1b, g2b = _SIZES[data.curve]
    ar, bs, krs = bytearray(g1b), bytearray(g2b), bytearray(g1b)
    cid = GG_CURVE_BN254 if data.curve == "bn254" else GG_CURVE_BLS12_381
    check(lib.gg_groth16_finalize_ex(cid, ptr(data.alpha1), ptr(data.beta1), ptr(data.delta1),
                                  ptr(data.beta2), ptr(data.delta2), ptr(partials), ptr(r), ptr(s),
                                  ptr(ar), ptr(bs), ptr(krs)))
    return Proof(bytes(ar), bytes(bs), bytes(krs))


def prove_distributed(pk: ProvingKeyShard, solution: Solution, *opts, r: bytes = None,
                      s: bytes = None, device=None) -> Proof:
    """Multi-GPU Prove, one process per GPU (torch.distributed, RCCL on ROCm):
    shard partials -> all-gather (576 B per rank) -> exact sum -> combination.
    r and s come from rank 0 (broadcast) unless given; every rank returns the proof."""
    import torch
    import torch.distributed as tdist
    cfg = backend.new_prover_config(*opts)
    if not backend.accelerated(cfg):
        raise RuntimeError("accelerated prover requested without with_amd_acceleration()")
    world = tdist.get_world_size() if tdist.is_initialized() else 1
    if r is None or s is None:
        rs = torch.frombuffer(bytearray(_rand_fr_mont() + _rand_fr_mont()), dtype=torch.uint8)
        if world > 1:
            rs = rs.to(device) if device is not None else rs
            tdist.broadcast(rs, 0)
        rsb = bytes(rs.cpu().numpy())
        r, s = rsb[:32], rsb[32:]
    # errgroup across ranks (prove.go:198-209): a rank whose partial fails makes
    # every rank raise at the status step before the gather (dist.RankGuard)
    guard = gdist.RankGuard(device, "Groth16 prove (shard partials)")
    fixed = guard.run(FixedTerms, pk.data, r, s)  # host threads, overlapped with the GPU work
    try:
        part = guard.run(prove_partial, pk, solution)
    except BaseException:
        fixed.close()
        raise
    return gather_and_finalize(pk.data, part, r, s, device, fixed=fixed, guard=guard)


def gather_and_finalize(data: ProvingKeyData, part: bytes, r: bytes, s: bytes, device=None,
                        fixed: "FixedTerms" = None, guard=None) -> Proof:
    """All-gather every rank's 576-B partials, add them exactly, combine (all ranks).
    fixed: the fixed-point terms already started (FixedTerms) for this r, s.
    guard: the proof's dist.RankGuard (its status step comes first: a failed
    rank makes every rank raise instead of waiting in the gather)."""
    import torch
    import torch.distributed as tdist
    world = tdist.get_world_size() if tdist.is_initialized() else 1
    try:
        if guard is not None:
            guard.check("partial all-gather")
        if world > 1:
            t = torch.frombuffer(bytearray(part), dtype=torch.uint8)
            if device is not None:
                t = t.to(device)
            bufs = [torch.empty_like(t) for _ in range(world)]
            tdist.all_gather(bufs, t)
            part = add_partials([bytes(b.cpu().numpy()) for b in bufs])
    except BaseException:
        if fixed is not None:
            fixed.close()
        raise
    if fixed is not None:
        return fixed.finish(part)
    return finalize(data, part, r, s)


# ------------------------------------------------- distributed computeH
class HShard:
    """This rank's part of the distributed computeH (gg_hshard_*): three
    all-to-alls per proof instead of h computed on every GPU."""

    def __init__(self, log_n: int, rank: int, world: int, omega: bytes = None, gen: bytes = None,
                 curve: str = "bn254"):
        if curve == "bn254":
            omega = omega or fr.fr_mont(fr.domain_generator(log_n))
            gen = gen or fr.fr_mont(fr.FR_MULTIPLICATIVE_GEN)
            cid = GG_CURVE_BN254
        else:
            omega = omega or fr.bls_fr_mont(fr.bls_domain_generator(log_n))
            gen = gen or fr.bls_fr_mont(fr.BLS_FR_MULTIPLICATIVE_GEN)
            cid = GG_CURVE_BLS12_381
        h = ctypes.c_void_p()
        check(lib.gg_hshard_create_ex(cid, log_n, ptr(omega), ptr(gen), rank, world, ctypes.byref(h)))
        self.handle, self.log_n, self.rank, self.world = h, log_n, rank, world
        m, xb = ctypes.c_size_t(), ctypes.c_size_t()
        check(lib.gg_hshard_info(h, ctypes.byref(m), ctypes.byref(xb)))
        self.m, self.exchange_bytes = m.value, xb.value

    def exchange_bytes_after(self, phase: int) -> int:
        """bytes per rank pair of the all-to-all after phase 1, 2 or 3"""
        v = ctypes.c_size_t()
        check(lib.gg_hshard_exchange_bytes(self.handle, phase, ctypes.byref(v)))
        return v.value

    def phase(self, k: int, a=None, b=None, c=None, length: int = 0, on_device: bool = False,
              recv=None, out=None):
        check(lib.gg_hshard_phase(self.handle, k, ptr(a), ptr(b), ptr(c), length, int(on_device),
                                  ptr(recv), ptr(out), None))

    def close(self):
        if self.handle:
            lib.gg_hshard_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def prove_partial_dist(pk: ProvingKeyShard, hs: HShard, solution: Solution, exchange, send, recv) -> bytes:
    """gg_groth16_prove_partial_dist: shard partials with the distributed computeH.
    exchange(send_ptr, recv_ptr, bytes_per_rank) performs the all-to-all."""
    import traceback
    from ._lib import EXCHANGE_FN

    def _cb(ctx, s_ptr, r_ptr, nbytes):
        try:
            exchange(s_ptr, r_ptr, nbytes)
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    cb = EXCHANGE_FN(_cb)
    out = bytearray(PARTIALS_BYTES)
    check(lib.gg_groth16_prove_partial_dist(
        pk.handle, hs.handle, ptr(solution.W), solution.n_wires, ptr(solution.A), ptr(solution.B),
        ptr(solution.C), solution.n_constraints, int(solution.on_device), cb, None, ptr(send),
        ptr(recv), ptr(out)))
    return bytes(out)


class TorchExchange:
    """All-to-all over torch.distributed for the distributed computeH: RCCL
    (backend "nccl") on device buffers, or gloo through host staging.

    Failure semantics: while prove_distributed_h runs, `guard` is its
    dist.RankGuard and every all-to-all is preceded by a status step: a rank
    whose prove fails before an exchange joins that step with its error
    (RankGuard.fail), so its peers raise RankFailure there instead of waiting in
    all_to_all_single until the group's timeout.  (A collective that fails
    half-way, e.g. a dead peer, still ends by the transport's own timeout.)"""

    def __init__(self, nbytes: int, device):
        import torch
        import torch.distributed as tdist
        self.dev = torch.device(device)
        self.send = torch.empty(nbytes, dtype=torch.uint8, device=self.dev)
        self.recv = torch.empty(nbytes, dtype=torch.uint8, device=self.dev)
        self.gloo = tdist.get_backend() != "nccl"
        self.world = tdist.get_world_size()
        # the collective is joined on a stream of the greatest priority: its
        # own hardware queue, so the host's wait for it never sits behind an MSM
        # kernel of the library's streams on a shared queue
        self.stream = torch.cuda.Stream(device=self.dev, priority=-1)
        self.guard = None

    def __call__(self, s_ptr, r_ptr, nbytes):
        import torch
        import torch.distributed as tdist
        if self.guard is not None:
            self.guard.check("computeH all-to-all")
        total = nbytes * self.world
        s, r = self.send[:total], self.recv[:total]
        with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):
            if self.gloo:
                rc = torch.empty(total, dtype=torch.uint8)
                tdist.all_to_all_single(rc, s.cpu())
                r.copy_(rc)
            else:
                tdist.all_to_all_single(r, s)
            self.stream.synchronize()


def prove_distributed_h(pk: ProvingKeyShard, hs: HShard, xchg: TorchExchange, solution: Solution,
                        *opts, r: bytes, s: bytes, device=None) -> Proof:
    """Multi-GPU Prove with the distributed computeH: per-rank partials (three
    all-to-alls inside), all-gather of the 576-B partials, exact sum, combination."""
    cfg = backend.new_prover_config(*opts)
    if not backend.accelerated(cfg):
        raise RuntimeError("accelerated prover requested without with_amd_acceleration()")
    guard = gdist.RankGuard(device, "Groth16 prove (distributed computeH)")
    fixed = guard.run(FixedTerms, pk.data, r, s)  # host threads, overlapped with the GPU work
    xchg.guard = guard  # a status step before each of the three all-to-alls
    try:
        part = guard.run(prove_partial_dist, pk, hs, solution, xchg, xchg.send.data_ptr(), xchg.recv.data_ptr())
    except BaseException:
        fixed.close()
        raise
    finally:
        xchg.guard = None
    return gather_and_finalize(pk.data, part, r, s, device, fixed=fixed, guard=guard)
