"""PlonK BLS12-381 prover: ctypes mirror of gnark's backend/plonk/bls12-381
ProvingKey / Prove (setup.go:88-106, prove.go:116-1079) over the C-ABI prover
(csrc/plonk_prover.hip: gg_plonk_pk_create, gg_plonk_prove).

The whole prove.go flow runs inside libgnark_amd.so -- commitToLRO, completeQk,
deriveGammaAndBeta (bindPublicData), buildRatioCopyConstraint, computeNumerator
per coset, divideByXMinusOne, commitToQuotient, openZ, foldH,
computeLinearizedPolynomial, batchOpening -- with the errgroup DAG mapped onto
HIP streams and the Fiat-Shamir transcripts in C++ (SHA-256 by default, or the
caller's hash through gg_hash_fn).  This module only marshals arguments, so a Go
shim (go/backend/plonk/bls12-381/amd) and these tests drive the same code.

Public inputs (completeQk, prove.go:397-423) and BSB22 commitments
(initBSB22Commitments / bsb22Hint, prove.go:304-352) are supported: the
solver's hint commits the committed values through `ProvingKey.commit_lagrange`
and hashes the digest to the field (hash_to_field, a gnark-crypto [ext]
algorithm the caller supplies); `prove` receives the committed-value vectors,
digests and hashed values.
"""
from __future__ import annotations

import ctypes
import dataclasses
import secrets
from typing import Callable, List, Optional, Sequence, Tuple

from . import fr, ntt
from ._lib import DeviceBuffer, check, lib, ptr, GG_CURVE_BLS12_381, GG_PLONK_PART_SLOTS, GG_REHEARSAL, HASH_FN, REDUCE_FN

R = fr.BLS_R
ORDER_BLINDING = (1, 1, 1, 2)  # order_blinding_L, _R, _O, _Z (prove.go:88-93)


class _Field:
    """The scalar field and G1 point size of a PlonK curve (backend/plonk/bls12-381,
    backend/plonk/bn254)."""

    def __init__(self, curve):
        from ._lib import GG_CURVE_BN254
        self.curve = curve
        if curve == "bn254":
            self.cid, self.R, self.pt = GG_CURVE_BN254, fr.R, 64
            self.mont, self.unmont = fr.fr_mont, fr.fr_unmont
            self.gen, self.domain_generator = fr.FR_MULTIPLICATIVE_GEN, fr.domain_generator
        elif curve == "bls12-381":
            self.cid, self.R, self.pt = GG_CURVE_BLS12_381, fr.BLS_R, 96
            self.mont, self.unmont = fr.bls_fr_mont, fr.bls_fr_unmont
            self.gen, self.domain_generator = fr.BLS_FR_MULTIPLICATIVE_GEN, fr.bls_domain_generator
        else:
            raise ValueError("curve must be 'bls12-381' or 'bn254'")


def fr_int(b: bytes) -> int:
    return fr.bls_fr_unmont(b)


def fr_b(x: int) -> bytes:
    return fr.bls_fr_mont(x % R)


def _host(v, nbytes: int) -> bytes:
    """bytes of a host buffer or a DeviceBuffer (copied back)."""
    if isinstance(v, DeviceBuffer):
        return v.to_host(nbytes)
    b = bytes(v)
    assert len(b) >= nbytes, "buffer too short"
    return b[:nbytes]


@dataclasses.dataclass
class VerifyingKey:
    """backend/plonk/bls12-381 VerifyingKey (setup.go:37-60) minus the KZG G2 part."""
    size: int
    generator: int
    coset_shift: int
    S: List[bytes]
    Ql: bytes
    Qr: bytes
    Qm: bytes
    Qo: bytes
    Qk: bytes
    Qcp: List[bytes]
    nb_public: int
    commitment_indexes: List[int]


@dataclasses.dataclass
class Proof:
    """backend/plonk/bls12-381 Proof (prove.go:96-114), affine points (Montgomery bytes)."""
    LRO: List[bytes]
    Z: bytes
    H: List[bytes]
    bsb22: List[bytes]
    batched_H: bytes
    claimed_values: List[int]
    z_shifted_H: bytes
    z_shifted_value: int

    @classmethod
    def parse(cls, b: bytes, n_cmt: int, curve: str = "bls12-381") -> "Proof":
        o = 0
        F = _Field(curve)

        def take(k):
            nonlocal o
            o += k
            return b[o - k:o]
        pt = F.pt
        lro = [take(pt) for _ in range(3)]
        z = take(pt)
        h = [take(pt) for _ in range(3)]
        bsb = [take(pt) for _ in range(n_cmt)]
        bh = take(pt)
        cv = [F.unmont(take(32)) for _ in range(7 + n_cmt)]
        zh = take(pt)
        zv = F.unmont(take(32))
        return cls(lro, z, h, bsb, bh, cv, zh, zv)


def _hash_cb(h):
    """gg_hash_fn over a hashlib-style constructor (None = the library's SHA-256)."""
    if h is None:
        return HASH_FN()

    def cb(_ctx, data, ln, out, out_len):
        try:
            d = h(ctypes.string_at(data, ln)).digest()
            if len(d) > out_len[0]:
                return 1
            ctypes.memmove(out, d, len(d))
            out_len[0] = len(d)
            return 0
        except Exception:  # pragma: no cover - reported as a library error
            return 1
    return HASH_FN(cb)


class ProvingKey:
    """Device-resident PlonK proving key (setup.go:88-106).

    kzg_g1: >= n+3 affine points [tau^i]G (pk.Kzg.G1); kzg_lagrange_g1: n points
    [L_i(tau)]G (pk.KzgLagrange.G1); ql..qk, s1..s3 and qcp: the trace
    polynomials, in Lagrange regular form (BuildTrace / computePermutationPolynomials
    output, basis="lagrange", converted on the GPU) or canonical (gnark's pk.trace
    after Setup, basis="canonical"); Qk is the incomplete one.  perm: 3n int64
    (pk.trace.S).  Buffers: bytes or DeviceBuffers.

    Multi-GPU: shard=(rank, world) keeps this rank's slice of each
    KZG base; `reduce(jac144) -> jac144` (e.g. gnark_amd.dist.allgather_partial)
    completes every partial commitment; the library calls it in one fixed order.
    One process, N GPUs: devices=[d0, d1, ...] splits the key over the devices
    inside the library (gg_plonk_pk_create_multi: KZG base slices, numerator
    cosets; ids may repeat); d0 runs the prover, device inputs live there."""

    def __init__(self, log_n: int, kzg_g1, kzg_lagrange_g1, ql, qr, qm, qo, qk, s1, s2, s3, perm,
                 qcp: Sequence = (), nb_public: int = 0, commitment_indexes: Sequence[int] = (),
                 basis: str = "lagrange", big_log: Optional[int] = None, shard=None, reduce=None,
                 vk: Optional[VerifyingKey] = None, devices: Optional[Sequence[int]] = None,
                 curve: str = "bls12-381"):
        F = self.field = _Field(curve)
        self.curve = curve
        mont = F.mont
        self.log_n = log_n
        self.n = n = 1 << log_n
        self.big_log = big_log if big_log is not None else log_n + (2 if n >= 6 else 3)
        self.omega = F.domain_generator(log_n)
        self.omega_big = F.domain_generator(self.big_log)
        self.g = F.gen
        self.n_cmt = len(qcp)
        self.nb_public = nb_public
        nb = 32 * n
        polys = [ql, qr, qm, qo, qk, s1, s2, s3] + list(qcp)
        if basis == "lagrange":
            d0 = ntt.Domain(log_n, mont(self.omega), mont(self.g), curve=F.cid)
            canon = []
            for v in polys:
                b = DeviceBuffer(nb)
                if isinstance(v, DeviceBuffer):
                    check(lib.gg_copy_device(ptr(b), ptr(v), nb))
                else:
                    check(lib.gg_copy_to_device(ptr(b), ptr(v), nb))
                d0.fft_inverse(b, ntt.DIF)  # Lagrange regular -> canonical bit-reversed
                reg = DeviceBuffer(nb)
                # a permutation of 32-B elements: the same kernel serves both scalar fields
                check(lib.gg_bls12_381_fr_bit_reverse(ptr(b), ptr(reg), n, None))
                canon.append(reg.to_host(nb))
            del d0
        else:
            canon = [_host(v, nb) for v in polys]
        keep = [ctypes.create_string_buffer(c, len(c)) for c in canon]  # alive for the call
        tr = (ctypes.c_void_p * 8)(*[ctypes.addressof(c) for c in keep[:8]])
        qa = (ctypes.c_void_p * max(1, self.n_cmt))(*[ctypes.addressof(c) for c in keep[8:]])
        idx = (ctypes.c_uint64 * max(1, self.n_cmt))(*commitment_indexes)
        kz = _host(kzg_g1, F.pt * (n + 3))
        kl = _host(kzg_lagrange_g1, F.pt * n)
        pm = _host(perm, 24 * n)
        vkd = None
        if vk is not None:
            vkd = b"".join(vk.S + [vk.Ql, vk.Qr, vk.Qm, vk.Qo, vk.Qk] + list(vk.Qcp))
        h = ctypes.c_void_p()
        args = (F.cid, log_n, self.big_log, mont(self.omega), mont(self.omega_big), mont(self.g), kz, n + 3, kl, tr,
                qa, self.n_cmt, pm, nb_public, idx, vkd)
        self._reduce_cb = None
        if shard is not None and shard[1] > 1:
            rank, world = shard

            def cb(_ctx, jac):
                try:
                    out = reduce(ctypes.string_at(jac, 144))
                    ctypes.memmove(jac, out, 144)
                    return 0
                except Exception:  # pragma: no cover - surfaced as GG_ERR_DEVICE
                    return 1
            self._reduce_cb = REDUCE_FN(cb)
            check(lib.gg_plonk_pk_create_shard_ex(*args, rank, world, self._reduce_cb, None, ctypes.byref(h)))
        else:
            devs = list(devices) if devices is not None and len(devices) > 1 else []
            check(lib.gg_plonk_pk_create_ex(*args, len(devs), (ctypes.c_int * max(1, len(devs)))(*devs),
                                            ctypes.byref(h)))
        self.handle = h
        del keep
        pt = F.pt
        out = bytearray(pt * (8 + self.n_cmt))
        check(lib.gg_plonk_pk_vk(h, ptr(out), len(out)))
        d = [bytes(out[pt * i:pt * (i + 1)]) for i in range(8 + self.n_cmt)]
        self.vk = VerifyingKey(n, self.omega, self.g, d[0:3], d[3], d[4], d[5], d[6], d[7], d[8:], nb_public,
                               list(commitment_indexes))

    def devices(self) -> List[int]:
        """the key's device parts, primary first (gg_plonk_pk_devices)"""
        k = ctypes.c_int()
        check(lib.gg_plonk_pk_devices(self.handle, None, 0, ctypes.byref(k)))
        arr = (ctypes.c_int * k.value)()
        check(lib.gg_plonk_pk_devices(self.handle, arr, k.value, ctypes.byref(k)))
        return list(arr)

    def set_rehearsal(self, on: bool = True, part: int = 0):
        """Timing rehearsal (gg_plonk_pk_set_rehearsal_part): only device part
        `part` (0 = primary) of a multi-part key does its work in later proves
        (one part's work timed on one GPU); those proofs are NOT valid and
        prove() refuses them unless called with rehearsal_ok=True."""
        check(lib.gg_plonk_pk_set_rehearsal_part(self.handle, int(part) if on else -1))

    def peer_access(self) -> list:
        """[i][j]: how device part i reaches part j ('same_device', 'enabled',
        'unavailable', 'enable_failed'; gg_plonk_pk_peer_access)"""
        from ._lib import PEER_ACCESS
        k = ctypes.c_int()
        check(lib.gg_plonk_pk_peer_access(self.handle, None, 0, ctypes.byref(k)))
        w = k.value
        arr = (ctypes.c_int * (w * w))()
        check(lib.gg_plonk_pk_peer_access(self.handle, arr, w * w, ctypes.byref(k)))
        return [[PEER_ACCESS.get(arr[i * w + j], str(arr[i * w + j])) for j in range(w)] for i in range(w)]

    def part_timings(self) -> list:
        """Per device part (0 = primary), the last proof: MSM slices and their ms,
        scalar-slice copies (ms, MB), quotient units (ms, copies in / out, MB),
        part 0's wait for its peers, the part's slice of the ratio, and its
        canonical-form tasks (count, ms, MB pushed) (gg_plonk_pk_part_timings)."""
        names = ["msm_slices", "msm_ms", "scalar_copy_ms", "scalar_MB", "quotient_units", "unit_ms",
                 "unit_in_copy_ms", "unit_out_copy_ms", "unit_MB", "wait_for_peers_ms", "ratio_ms",
                 "canon_tasks", "canon_ms", "canon_MB"]
        out = []
        for p in range(len(self.devices())):
            v = (ctypes.c_double * GG_PLONK_PART_SLOTS)()
            check(lib.gg_plonk_pk_part_timings(self.handle, p, v, GG_PLONK_PART_SLOTS))
            out.append(dict(zip(names, list(v))))
        return out

    def commit_lagrange(self, values) -> bytes:
        """kzg.Commit(values, pk.KzgLagrange) -- the commitment of bsb22Hint (prove.go:336)."""
        out = bytearray(self.field.pt)
        on_dev = isinstance(values, DeviceBuffer)
        check(lib.gg_plonk_commit_lagrange(self.handle, ptr(values), int(on_dev), ptr(out)))
        return bytes(out)

    def close(self):
        if getattr(self, "handle", None):
            lib.gg_plonk_pk_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def prove(pk: ProvingKey, L, R_, O, rng=None, timings: Optional[dict] = None, public: Sequence[int] = (),
          commitments: Sequence[Tuple[bytes, bytes, int]] = (), challenge_hash: Optional[Callable] = None,
          folding_hash: Optional[Callable] = None, rehearsal_ok: bool = False) -> Proof:
    """Prove after Solve (prove.go:116-176).  L, R_, O: the solver's Lagrange-regular
    vectors (bytes or DeviceBuffers of n fr); public: fullWitness[:nb_public] (ints);
    commitments: per BSB22 commitment (committed values, Lagrange, n fr bytes;
    digest, affine bytes; hashed value, int) as bsb22Hint produced them; rng: the
    blinding coefficients' source (random.Random for reproducible proofs, default
    secrets); challenge_hash / folding_hash: hashlib constructors (default SHA-256)."""
    assert len(public) == pk.nb_public and len(commitments) == pk.n_cmt
    F = pk.field
    rnd = rng or secrets.SystemRandom()
    blind = b"".join(F.mont(rnd.randrange(F.R)) for o in ORDER_BLINDING for _ in range(o + 1))
    on_dev = isinstance(L, DeviceBuffer)
    nb = 32 * pk.n
    lro = [x if on_dev else _host(x, nb) for x in (L, R_, O)]
    pub = b"".join(F.mont(v % F.R) for v in public)
    cv = [ctypes.create_string_buffer(_host(c[0], nb), nb) for c in commitments]  # alive for the call
    cva = (ctypes.c_void_p * max(1, len(cv)))(*[ctypes.addressof(c) for c in cv])
    dig = b"".join(c[1] for c in commitments)
    hashed = b"".join(F.mont(c[2] % F.R) for c in commitments)
    size = lib.gg_plonk_proof_size_ex(F.cid, pk.n_cmt)
    out = bytearray(size)
    hc, hf = _hash_cb(challenge_hash), _hash_cb(folding_hash)
    rc = lib.gg_plonk_prove(pk.handle, ptr(lro[0]), ptr(lro[1]), ptr(lro[2]), int(on_dev), ptr(pub) if pub else None,
                            len(public), cva, ptr(dig) if dig else None, ptr(hashed) if hashed else None,
                            pk.n_cmt, ptr(blind), hc, None, hf, None, ptr(out), size)
    if not (rc == GG_REHEARSAL and rehearsal_ok):
        check(rc)
    if timings is not None:
        ms = (ctypes.c_double * 8)()
        check(lib.gg_plonk_last_timings(ms, 8))
        names = ["commit_lro", "ratio_z", "numerator_enqueued", "commit_h", "open_z_linearize",
                 "commit_linearized", "batch_open"]
        prev = 0.0
        for k, nm in enumerate(names):
            timings[nm] = ms[k] - prev
            prev = ms[k]
        timings["total"] = prev
    return Proof.parse(bytes(out), pk.n_cmt, pk.curve)


class GroupProvingKey:
    """PlonK under a process-per-GPU launch (torch.distributed.run, one rank per
    GPU; SURVEY 8(e), BASELINE configs[4] "8 x MI355X").

    Rank 0 ("leader") holds a one-process multi-part key whose device parts are
    the GPUs of all ranks, in rank order (gg_plonk_pk_create_ex with devices =
    every rank's device): its proof runs the whole device-part split -- KZG
    shares, quotient units, ratio slices, canonical forms -- with
    the cross-part hand-offs as in-library peer copies over xGMI, exactly as a
    one-process (Go) caller's key does.  The other ranks hold no PlonK state;
    they take part in the process group's collectives (the device all-gather
    here, the proof broadcast in prove_group).  Why not a callback per hand-off
    (as gg_hshard does for Groth16's three all-to-alls): a PlonK proof has ~20
    dependent cross-part hand-offs (Z slices to the Z owner, canonical forms to
    every unit, unit blocks back, scalar slices ahead of each MSM stage), each a
    device-to-device copy ordered by HIP events; a host round trip through a
    collective per hand-off would serialise what the event graph overlaps.

    `key_args` / `key_kw`: the ProvingKey arguments (significant on rank 0 only;
    other ranks may pass None for the buffers).  local_device: this rank's GPU.

    Preconditions, checked at creation (dist.check_leader_devices): every rank's
    GPU id must name the same GPU on rank 0 (a launcher that isolates
    HIP_VISIBLE_DEVICES per rank breaks the leader design) and, under RCCL, no two
    ranks may share a GPU.  A violation -- or any failure of rank 0's key
    creation -- raises on every rank (RankFailure on the others), never a hang.
    `identity` / `view`: test hooks for the device identities (default
    dist.device_identity)."""

    mode = "leader"  # rank 0 runs the whole device-part split; the others receive the proof

    def __init__(self, *key_args, local_device: int = 0, comm_device=None, identity=None, view=None, **key_kw):
        import torch.distributed as dist
        from . import dist as gdist
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        backend = dist.get_backend() if dist.is_initialized() else None
        self.devices = gdist.group_devices(local_device, comm_device)
        ident = identity(local_device) if identity else gdist.device_identity(local_device)
        self.identities = gdist.group_identities(ident, comm_device)
        self.comm_device = comm_device
        self.pk = None
        err = None
        if self.rank == 0:
            try:
                probs = gdist.check_leader_devices(self.devices, self.identities, view or gdist.device_identity,
                                                   backend)
                if probs:
                    raise ValueError("PlonK leader key refused: " + "; ".join(probs))
                self.pk = ProvingKey(*key_args, devices=self.devices, **key_kw)
            except BaseException as e:
                err = e
        gdist.broadcast_status(err is None, f"{type(err).__name__}: {err}" if err else "", b"", 0, 0, comm_device,
                               "PlonK leader key creation")
        if err is not None:
            raise err
        curve = key_kw.get("curve", "bls12-381")
        self.curve = curve
        self.n_cmt = len(key_kw.get("qcp", ()))

    def close(self):
        if self.pk is not None:
            self.pk.close()
            self.pk = None


def prove_group(gpk: GroupProvingKey, L, R_, O, **kw) -> Proof:
    """prove() on the leader's multi-part key; every rank returns the proof
    (broadcast from rank 0).  Inputs and options are significant on rank 0."""
    from . import dist as gdist
    size = lib.gg_plonk_proof_size_ex(_Field(gpk.curve).cid, gpk.n_cmt)
    raw, err = b"", None
    if gpk.rank == 0:
        try:
            pr = prove(gpk.pk, L, R_, O, **kw)
            raw = proof_bytes(pr, gpk.curve)
        except BaseException as e:  # errgroup (prove.go:132-173): the proof ends on every rank
            err = e
    # the leader's status with the proof: a failed prove raises on every rank
    raw = gdist.broadcast_status(err is None, f"{type(err).__name__}: {err}" if err else "", raw, size, 0,
                                 gpk.comm_device, "PlonK prove (leader)")
    if err is not None:
        raise err
    return Proof.parse(raw, gpk.n_cmt, gpk.curve)


def proof_bytes(pr: Proof, curve: str = "bls12-381") -> bytes:
    """the library's proof layout (Proof.parse's inverse)"""
    F = _Field(curve)
    return b"".join(pr.LRO + [pr.Z] + pr.H + pr.bsb22 + [pr.batched_H] +
                    [F.mont(v) for v in pr.claimed_values] + [pr.z_shifted_H, F.mont(pr.z_shifted_value)])

