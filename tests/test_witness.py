"""Witness binary format (backend/witness/witness.go:15-36): header parsing on the
host (CPU), element conversion on the GPU, pinned by the reference's own KAT
(Y = 35 public, X = 3, Z = 2 secret)."""
import random

import pytest

import bn254_oracle as o

KAT = ("00000001000000020000000300000000000000000000000000000000000000000000000000000000000000"
       "2300000000000000000000000000000000000000000000000000000000000000030000000000000000000000"
       "000000000000000000000000000000000000000002")


def test_header_kat():
    from gnark_amd import witness
    data = bytes.fromhex(KAT)
    assert witness.parse_header(data) == (1, 2, 3, 12)
    assert o.witness_encode([35], [3, 2]) == data
    with pytest.raises(ValueError):
        witness.parse_header(data[:40])
    bad = bytearray(data)
    bad[11] = 4  # len != nbPublic + nbSecret: ReadFrom (witness.go:140-190) does not check it
    assert witness.parse_header(bytes(bad) + bytes(32)) == (1, 2, 4, 12)
    with pytest.raises(ValueError):  # but the vector must be there
        witness.parse_header(bytes(bad))


@pytest.mark.gpu
def test_read_write_kat_gpu():
    from gnark_amd import witness, fr
    w = witness.read(bytes.fromhex(KAT))
    assert (w.nb_public, w.nb_secret) == (1, 2)
    vals = w.vector.to_host(96)
    assert [fr.fr_unmont(vals[32 * i:32 * i + 32]) for i in range(3)] == [35, 3, 2]
    assert witness.write(w).hex() == KAT
    assert witness.write(w.public()) == bytes.fromhex("00000001000000000000000100") + bytes(30) + bytes([0x23])


@pytest.mark.gpu
@pytest.mark.parametrize("curve_name", ["bn254", "bls12_381"])
def test_roundtrip_and_range_check_gpu(curve_name):
    from gnark_amd import witness, GnarkAmdError
    from gnark_amd._lib import GG_CURVE_BN254, GG_CURVE_BLS12_381
    import bls12_381_oracle as bo
    curve = GG_CURVE_BN254 if curve_name == "bn254" else GG_CURVE_BLS12_381
    r = o.R if curve_name == "bn254" else bo.R
    to_mont = o.fr_to_bytes if curve_name == "bn254" else bo.fr_to_bytes
    rnd = random.Random(4)
    vals = [0, 1, r - 1] + [rnd.randrange(r) for _ in range(5000)]
    data = bytes.fromhex("%08x%08x%08x" % (3, len(vals) - 3, len(vals))) + \
        b"".join(v.to_bytes(32, "big") for v in vals)
    w = witness.read(data, curve)
    assert w.vector.to_host(32 * len(vals)) == b"".join(to_mont(v) for v in vals)
    assert witness.write(w) == data
    # an element >= r is refused, as fr.Vector.ReadFrom does
    bad = bytearray(data)
    bad[12 + 32 * 7:12 + 32 * 8] = r.to_bytes(32, "big")
    with pytest.raises(GnarkAmdError):
        witness.read(bytes(bad), curve)
