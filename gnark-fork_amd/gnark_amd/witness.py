"""Witness binary format (backend/witness/witness.go:15-36, WriteTo :103-138,
ReadFrom :140-190) to / from the prover's device layout:

    Witness  -> [uint32(nbPublic) | uint32(nbSecret) | fr.Vector]
    fr.Vector -> [uint32(len) | len x 32-byte big-endian canonical elements]

Public variables first, then secret ones.  The header is parsed on the host;
the element conversion (big-endian canonical <-> Montgomery little-endian limbs,
with fr.Vector.ReadFrom's range check) runs on the GPU
(gg_fr_from_canonical_be / gg_fr_to_canonical_be)."""
from __future__ import annotations

import ctypes
import dataclasses
import struct

from ._lib import GG_CURVE_BN254, DeviceBuffer, check, lib, ptr


@dataclasses.dataclass
class Witness:
    nb_public: int
    nb_secret: int
    vector: DeviceBuffer  # (nb_public + nb_secret) fr, Montgomery, on the device
    curve: int = GG_CURVE_BN254

    @property
    def n(self) -> int:
        return self.nb_public + self.nb_secret

    def public(self) -> "Witness":
        """witness.Public() (witness.go:92-101): the public part only."""
        v = DeviceBuffer(max(32 * self.nb_public, 32))
        if self.nb_public:
            check(lib.gg_copy_device(ptr(v), ptr(self.vector), 32 * self.nb_public))
        return Witness(self.nb_public, 0, v, self.curve)


def parse_header(data: bytes):
    """(nbPublic, nbSecret, len, offset of the first element)."""
    if len(data) < 12:
        raise ValueError("witness: truncated header")
    nb_public, nb_secret, n = struct.unpack(">III", data[:12])
    if len(data) < 12 + 32 * n:
        raise ValueError("witness: truncated vector")
    # witness.ReadFrom (witness.go:140-190) reads the header and then the
    # fr.Vector as-is, without checking len == nbPublic + nbSecret; neither do we
    return nb_public, nb_secret, n, 12


def read(data: bytes, curve: int = GG_CURVE_BN254) -> Witness:
    """witness.ReadFrom / UnmarshalBinary into device memory (Montgomery)."""
    nb_public, nb_secret, n, off = parse_header(data)
    buf = DeviceBuffer(max(32 * n, 32))
    if n:
        check(lib.gg_copy_to_device(ctypes.c_void_p(buf.ptr), ptr(data[off:off + 32 * n]), 32 * n))
        bad = ctypes.c_uint64()
        check(lib.gg_fr_from_canonical_be(curve, ptr(buf), ptr(buf), n, ctypes.byref(bad), None))
    return Witness(nb_public, nb_secret, buf, curve)


def write(w: Witness) -> bytes:
    """witness.WriteTo / MarshalBinary from device memory."""
    n = w.n
    out = bytearray(12 + 32 * n)
    out[:12] = struct.pack(">III", w.nb_public, w.nb_secret, n)
    if n:
        tmp = DeviceBuffer(32 * n)
        check(lib.gg_fr_to_canonical_be(w.curve, ptr(w.vector), ptr(tmp), n, None))
        body = tmp.to_host(32 * n)
        out[12:] = body
    return bytes(out)
