"""Minimal host-side BN254 Fr/Fp helpers for byte layouts (not a compute path).

gnark-crypto stores fr.Element / fp.Element as Montgomery form (R = 2^256),
[4]uint64 little-endian.  These helpers exist so Python callers can build the
domain parameters gnark keeps in pk.Domain (Generator, FrMultiplicativeGen) and
encode proofs; all bulk arithmetic runs in libgnark_amd.so.
"""
from __future__ import annotations

# backend/groth16/bn254/solidity.go:41-42
P = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
R = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
FR_MULTIPLICATIVE_GEN = 5  # gnark-crypto fft.Domain.FrMultiplicativeGen [ext]
FR_TWO_ADICITY = 28


def fr_mont(x: int) -> bytes:
    return (((x % R) << 256) % R).to_bytes(32, "little")


def fr_unmont(b: bytes) -> int:
    return int.from_bytes(b[:32], "little") * pow(1 << 256, -1, R) % R


def fp_mont(x: int) -> bytes:
    return (((x % P) * (1 << 256)) % P).to_bytes(32, "little")


def fp_unmont(b: bytes) -> int:
    return int.from_bytes(b[:32], "little") * pow(1 << 256, -1, P) % P


def domain_generator(log_n: int) -> int:
    """omega_n = 5^((r-1)/2^log_n): gnark-crypto fft.NewDomain's Generator
    (pinned by std/commitments/fri/fri_test.go:35)."""
    assert 0 <= log_n <= FR_TWO_ADICITY
    return pow(FR_MULTIPLICATIVE_GEN, (R - 1) >> log_n, R)


def g1_raw(aff: bytes) -> bytes:
    """gnark RawEncoding of a G1Affine (64 B Montgomery in) -> X|Y big-endian."""
    if aff == bytes(64):
        out = bytearray(64)
        out[0] |= 0x40  # mUncompressedInfinity
        return bytes(out)
    return fp_unmont(aff[0:32]).to_bytes(32, "big") + fp_unmont(aff[32:64]).to_bytes(32, "big")


def g2_raw(aff: bytes) -> bytes:
    """G2Affine (128 B {X.A0,X.A1,Y.A0,Y.A1}) -> X.A1|X.A0|Y.A1|Y.A0 big-endian
    (test/assert_solidity.go:60-69)."""
    if aff == bytes(128):
        out = bytearray(128)
        out[0] |= 0x40
        return bytes(out)
    x0, x1, y0, y1 = (fp_unmont(aff[i:i + 32]) for i in range(0, 128, 32))
    return b"".join(v.to_bytes(32, "big") for v in (x1, x0, y1, y0))


# ---- BLS12-381 (PlonK path): std/math/emulated/emparams/emparams.go:145-171
BLS_P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
BLS_R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
BLS_FR_MULTIPLICATIVE_GEN = 7  # gnark-crypto bls12-381 fr [ext]
BLS_FR_TWO_ADICITY = 32


def bls_fr_mont(x: int) -> bytes:
    """bls12-381 fr.Element bytes: Montgomery R = 2^256, [4]uint64 LE."""
    return (((x % BLS_R) << 256) % BLS_R).to_bytes(32, "little")


def bls_fr_unmont(b: bytes) -> int:
    return int.from_bytes(b[:32], "little") * pow(1 << 256, -1, BLS_R) % BLS_R


def bls_fp_mont(x: int) -> bytes:
    """bls12-381 fp.Element bytes: Montgomery R = 2^384, [6]uint64 LE."""
    return (((x % BLS_P) << 384) % BLS_P).to_bytes(48, "little")


def bls_fp_unmont(b: bytes) -> int:
    return int.from_bytes(b[:48], "little") * pow(1 << 384, -1, BLS_P) % BLS_P


def bls_domain_generator(log_n: int) -> int:
    """7^((r-1)/2^log_n) -- gnark-crypto's choice for bls12-381 (unpinned by any
    reference fixture; pass pk.Domain.Generator to mirror a real key)."""
    assert 0 <= log_n <= BLS_FR_TWO_ADICITY
    return pow(BLS_FR_MULTIPLICATIVE_GEN, (BLS_R - 1) >> log_n, BLS_R)
