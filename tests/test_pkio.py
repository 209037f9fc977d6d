"""gnark's BN254 Groth16 proving-key byte format (marshal.go:246-374) in the
Python mirror (gnark_amd.pkio): WriteRawTo / WriteTo -> ReadFrom round trips of
the golden keys, the field layout byte by byte (domain header, u32 lengths,
u64 counters, flag-bearing point encodings), rejection of malformed input, and
(GPU) a proof from a key that went through the codec.  The reference holds no
serialized key, so the format itself is "parity unpinned" (module docstring)."""
import struct

import pytest

import bn254_oracle as o
from helpers import b, golden


def _data(idx):
    from gnark_amd import groth16
    g = golden()["groth16"][idx]
    return g, groth16.ProvingKeyData(
        log_n=g["log_n"], g1_A=b(g["g1_A"]), g1_B=b(g["g1_B"]), g1_Z=b(g["g1_Z"]),
        g1_K=b(g["g1_K"]), alpha1=b(g["alpha1"]), beta1=b(g["beta1"]), delta1=b(g["delta1"]),
        g2_B=b(g["g2_B"]), beta2=b(g["beta2"]), delta2=b(g["delta2"]),
        infinity_A=b(g["infA"]), infinity_B=b(g["infB"]), nb_public=g["nb_public"])


def _same(a, d):
    for f in ("log_n", "g1_A", "g1_B", "g1_Z", "g1_K", "alpha1", "beta1", "delta1", "g2_B", "beta2",
              "delta2", "nb_public"):
        assert getattr(a, f) == getattr(d, f), f
    assert bytes(a.infinity_A) == bytes(d.infinity_A) and bytes(a.infinity_B) == bytes(d.infinity_B)


@pytest.mark.parametrize("idx", [0, 1])
@pytest.mark.parametrize("raw", [True, False])
def test_pk_roundtrip(idx, raw):
    from gnark_amd import pkio
    g, d = _data(idx)
    blob = pkio.write_proving_key(d, raw=raw, commitment_keys=[(d.g1_A[:128], d.g1_B[:64])])
    back, cks = pkio.read_proving_key(blob, nb_public=d.nb_public)
    _same(back, d)
    assert cks == [(d.g1_A[:128], d.g1_B[:64])]
    # the domain the reader reports is the one the prover uses by default
    from gnark_amd import fr
    assert back.domain_generator == fr.fr_mont(fr.domain_generator(d.log_n))
    assert back.domain_mul_gen == fr.fr_mont(5)
    # re-encoding is byte-identical
    assert pkio.write_proving_key(back, raw=raw, commitment_keys=cks) == blob


def test_pk_layout():
    """Field-by-field offsets of WriteRawTo (marshal.go:255-283)."""
    from gnark_amd import pkio
    g, d = _data(1)
    blob = pkio.write_proving_key(d, raw=True)
    n = 1 << d.log_n
    assert struct.unpack(">Q", blob[:8])[0] == n
    assert int.from_bytes(blob[8:40], "big") == pow(n, -1, o.R)
    off = 168
    ax, ay = o.g1_from_bytes(d.alpha1)
    assert blob[off:off + 64] == ax.to_bytes(32, "big") + ay.to_bytes(32, "big")
    off += 3 * 64
    nA = len(d.g1_A) // 64
    assert struct.unpack(">I", blob[off:off + 4])[0] == nA
    # compressed alpha: x with the y-order flag in the two top bits
    cblob = pkio.write_proving_key(d, raw=False)
    flag = cblob[168] & 0xC0
    assert flag == (0xC0 if ay > (o.P - 1) // 2 else 0x80)
    assert (cblob[168] & 0x3F) == ax.to_bytes(32, "big")[0] and cblob[169:200] == ax.to_bytes(32, "big")[1:]
    # tail: nbWires, NbInfinityA, NbInfinityB, the two flag arrays, 0 commitment keys
    nw = d.n_wires
    tail = blob[-(24 + 2 * nw + 4):]
    assert struct.unpack(">QQQ", tail[:24]) == (nw, sum(d.infinity_A), sum(d.infinity_B))
    assert tail[24:24 + nw] == bytes(d.infinity_A) and tail[-4:] == bytes(4)


def test_pk_infinity_and_g2_encodings():
    from gnark_amd import pkio
    inf1, inf2 = bytes(64), bytes(128)
    assert pkio._g1_encode(inf1, raw=False) == b"\x40" + bytes(31)
    assert pkio._g1_decode(b"\x40" + bytes(31), 0, False) == (inf1, 32)
    assert pkio._g1_decode(bytes(64), 0, True) == (inf1, 64)
    assert pkio._g2_decode(b"\x40" + bytes(63), 0, False) == (inf2, 64)
    _, d = _data(1)
    for i in range(0, len(d.g2_B), 128):
        p = d.g2_B[i:i + 128]
        for raw in (True, False):
            enc = pkio._g2_encode(p, raw)
            assert pkio._g2_decode(enc, 0, raw)[0] == p


def test_pk_rejects_malformed():
    from gnark_amd import pkio
    _, d = _data(1)
    blob = pkio.write_proving_key(d, raw=True)
    with pytest.raises(ValueError):
        pkio.read_proving_key(blob[:100], 0)
    with pytest.raises(ValueError):
        pkio.read_proving_key(blob[:-30], 0)
    bad = bytearray(blob)
    bad[:8] = struct.pack(">Q", 3)  # not a power of two
    with pytest.raises(ValueError):
        pkio.read_proving_key(bytes(bad), 0)
    bad = bytearray(blob)
    bad[168 + 63] ^= 1  # alpha1.y off the curve
    with pytest.raises(ValueError):
        pkio.read_proving_key(bytes(bad), 0)
    cblob = bytearray(pkio.write_proving_key(d, raw=False))
    cblob[168] &= 0x3F  # compressed key whose first point lost its flag: misparsed -> error
    with pytest.raises(ValueError):
        pkio.read_proving_key(bytes(cblob), 0)


@pytest.mark.gpu
def test_pk_codec_then_prove():
    from gnark_amd import backend, groth16, pkio
    g, d = _data(1)
    back, _ = pkio.read_proving_key(pkio.write_proving_key(d, raw=False), nb_public=d.nb_public)
    pk = groth16.ProvingKey(back)
    sol = groth16.Solution(b(g["wires"]), b(g["solA"]), b(g["solB"]), b(g["solC"]), back.n_wires,
                           len(b(g["solA"])) // 32)
    pr = groth16.prove(pk, sol, backend.with_amd_acceleration(), r=b(g["r"]), s=b(g["s"]))
    assert (pr.Ar.hex(), pr.Bs.hex(), pr.Krs.hex()) == (g["Ar"], g["Bs"], g["Krs"])
    pk.close()
