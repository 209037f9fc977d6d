"""gnark's BN254 Groth16 proving-key byte format (backend/groth16/bn254/marshal.go:
writeTo 246-307, readFrom 309-374), so keys written by gnark's `WriteTo` /
`WriteRawTo` load straight into `groth16.ProvingKeyData` (and from there into
HBM), and keys made here can be handed back to gnark.

Layout, in marshal.go's order, through gnark-crypto's curve.Encoder
(github.com/consensys/gnark-crypto v0.12.2-0.20231117165148-e77308824822, not
vendored in the reference; its published encoding is restated here):

    Domain.WriteTo: Cardinality u64 BE, CardinalityInv, Generator, GeneratorInv,
                    FrMultiplicativeGen, FrMultiplicativeGenInv (fr: 32-B BE canonical)
    G1.Alpha, G1.Beta, G1.Delta                      (points)
    G1.A, G1.B, G1.Z, G1.K                            (u32 BE length + points)
    G2.Beta, G2.Delta, G2.B
    nbWires u64, NbInfinityA u64, NbInfinityB u64     (BE)
    InfinityA, InfinityB                              (nbWires bytes each, no length)
    len(CommitmentKeys) u32, then per key: Basis, BasisExpSigma (u32 length + points)

Points: raw (WriteRawTo) = X|Y big-endian canonical, G1 64 B, G2 128 B as
X.A1|X.A0|Y.A1|Y.A0; (0, 0) is infinity.  Compressed (WriteTo) = X only with the
top two bits of the first byte as flags: 0b10 y is the smaller root, 0b11 the
larger (E2: compare A1, then A0 if A1 = 0), 0b01 infinity.

Parity: the reference holds no serialized key, so the byte format is "parity
unpinned" beyond the round trips in tests/test_pkio.py; the point encoding
rules are those pinned for BLS12-381 by bellman_test.go in test_oracle_bls.
"""
from __future__ import annotations

import io
import struct
from typing import BinaryIO, List, Optional, Tuple, Union

from . import fr

P = fr.P
R = fr.R
_M_UNCOMPRESSED, _M_INFINITY, _M_SMALLEST, _M_LARGEST = 0x00, 0x40, 0x80, 0xC0
_MASK = 0xC0
_DOMAIN_BYTES = 8 + 5 * 32


# ------------------------------------------------------------- field helpers
def _fp_sqrt(a: int) -> Optional[int]:
    r = pow(a, (P + 1) // 4, P)  # p = 3 mod 4
    return r if r * r % P == a % P else None


def _f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def _f2_pow(a, e):
    r, b = (1, 0), a
    while e:
        if e & 1:
            r = _f2_mul(r, b)
        b = _f2_mul(b, b)
        e >>= 1
    return r


def _f2_sqrt(a) -> Optional[Tuple[int, int]]:
    """Square root in Fp2 = Fp[u]/(u^2+1), p = 3 mod 4 (Adj-Rodriguez-Henriquez Alg. 9)."""
    if a == (0, 0):
        return (0, 0)
    a1 = _f2_pow(a, (P - 3) // 4)
    alpha = _f2_mul(a1, _f2_mul(a1, a))
    x0 = _f2_mul(a1, a)
    if alpha == (P - 1, 0):
        x = _f2_mul((0, 1), x0)
    else:
        b = _f2_pow(((1 + alpha[0]) % P, alpha[1]), (P - 1) // 2)
        x = _f2_mul(b, x0)
    return x if _f2_mul(x, x) == (a[0] % P, a[1] % P) else None


def _lex_largest(y: int) -> bool:
    return y > (P - 1) // 2


def _lex_largest2(y) -> bool:
    return _lex_largest(y[1]) if y[1] else _lex_largest(y[0])


def _be(x: int) -> bytes:
    return x.to_bytes(32, "big")


def _mont(x: int) -> bytes:
    return fr.fp_mont(x)


def _unmont(b: bytes) -> int:
    return fr.fp_unmont(b)


# ------------------------------------------------------------- point codecs
def _g1_encode(aff: bytes, raw: bool) -> bytes:
    x, y = _unmont(aff[:32]), _unmont(aff[32:64])
    inf = x == 0 and y == 0
    if raw:
        return _be(x) + _be(y)
    if inf:
        return bytes([_M_INFINITY]) + bytes(31)
    b = bytearray(_be(x))
    b[0] |= _M_LARGEST if _lex_largest(y) else _M_SMALLEST
    return bytes(b)


def _g1_decode(buf: bytes, off: int, raw: bool) -> Tuple[bytes, int]:
    if raw:
        flag = buf[off] & _MASK
        if flag != _M_UNCOMPRESSED:
            raise ValueError("pk: expected an uncompressed G1 point")
        x = int.from_bytes(buf[off:off + 32], "big")
        y = int.from_bytes(buf[off + 32:off + 64], "big")
        if x >= P or y >= P:
            raise ValueError("pk: G1 coordinate not reduced")
        if (x, y) != (0, 0) and (y * y - x * x * x - 3) % P:
            raise ValueError("pk: G1 point not on the curve")
        return _mont(x) + _mont(y), off + 64
    flag = buf[off] & _MASK
    if flag == _M_INFINITY:
        return bytes(64), off + 32
    if flag not in (_M_SMALLEST, _M_LARGEST):
        raise ValueError("pk: bad G1 compression flag")
    xb = bytearray(buf[off:off + 32])
    xb[0] &= ~_MASK & 0xFF
    x = int.from_bytes(xb, "big")
    y = _fp_sqrt((x * x * x + 3) % P)
    if x >= P or y is None:
        raise ValueError("pk: G1 x not on the curve")
    if _lex_largest(y) != (flag == _M_LARGEST):
        y = (P - y) % P
    return _mont(x) + _mont(y), off + 32


_B2 = (19485874751759354771024239261021720505790618469301721065564631296452457478373 % P,
       266929791119991161246907387137283842545076965332900288569378510910307636690 % P)  # 3/(9+u)


def _g2_encode(aff: bytes, raw: bool) -> bytes:
    x = (_unmont(aff[0:32]), _unmont(aff[32:64]))
    y = (_unmont(aff[64:96]), _unmont(aff[96:128]))
    if raw:
        return _be(x[1]) + _be(x[0]) + _be(y[1]) + _be(y[0])
    if x == (0, 0) and y == (0, 0):
        return bytes([_M_INFINITY]) + bytes(63)
    b = bytearray(_be(x[1]) + _be(x[0]))
    b[0] |= _M_LARGEST if _lex_largest2(y) else _M_SMALLEST
    return bytes(b)


def _g2_decode(buf: bytes, off: int, raw: bool) -> Tuple[bytes, int]:
    def coord(o):
        return int.from_bytes(buf[o:o + 32], "big")
    if raw:
        if buf[off] & _MASK != _M_UNCOMPRESSED:
            raise ValueError("pk: expected an uncompressed G2 point")
        x = (coord(off + 32), coord(off))
        y = (coord(off + 96), coord(off + 64))
        if max(x + y) >= P:
            raise ValueError("pk: G2 coordinate not reduced")
        if (x, y) != ((0, 0), (0, 0)):
            lhs = _f2_mul(y, y)
            rhs = _f2_mul(x, _f2_mul(x, x))
            if ((lhs[0] - rhs[0] - _B2[0]) % P, (lhs[1] - rhs[1] - _B2[1]) % P) != (0, 0):
                raise ValueError("pk: G2 point not on the curve")
        return _mont(x[0]) + _mont(x[1]) + _mont(y[0]) + _mont(y[1]), off + 128
    flag = buf[off] & _MASK
    if flag == _M_INFINITY:
        return bytes(128), off + 64
    if flag not in (_M_SMALLEST, _M_LARGEST):
        raise ValueError("pk: bad G2 compression flag")
    hb = bytearray(buf[off:off + 32])
    hb[0] &= ~_MASK & 0xFF
    x = (coord(off + 32), int.from_bytes(hb, "big"))
    x3 = _f2_mul(x, _f2_mul(x, x))
    y = _f2_sqrt(((x3[0] + _B2[0]) % P, (x3[1] + _B2[1]) % P))
    if y is None:
        raise ValueError("pk: G2 x not on the curve")
    if _lex_largest2(y) != (flag == _M_LARGEST):
        y = ((P - y[0]) % P, (P - y[1]) % P)
    return _mont(x[0]) + _mont(x[1]) + _mont(y[0]) + _mont(y[1]), off + 64


# ------------------------------------------------------------- key codec
def write_proving_key(data, raw: bool = True, commitment_keys: Optional[List[Tuple[bytes, bytes]]] = None,
                      out: Optional[BinaryIO] = None) -> bytes:
    """ProvingKey.WriteRawTo (raw=True) / WriteTo (marshal.go:246-307) of a
    `groth16.ProvingKeyData` (BN254).  commitment_keys: (basis, basis_exp_sigma)
    G1 arrays (gnark layout) of the pedersen keys, default none."""
    if data.curve != "bn254":
        raise ValueError("pk codec: BN254 only")
    n = 1 << data.log_n
    omega = fr.fr_unmont(data.domain_generator) if data.domain_generator else fr.domain_generator(data.log_n)
    g = fr.fr_unmont(data.domain_mul_gen) if data.domain_mul_gen else fr.FR_MULTIPLICATIVE_GEN
    w = io.BytesIO()
    w.write(struct.pack(">Q", n))
    for v in (pow(n, -1, R), omega, pow(omega, -1, R), g, pow(g, -1, R)):
        w.write(_be(v))

    def g1s(b):
        return [b[i:i + 64] for i in range(0, len(b), 64)]

    def vec1(b):
        pts = g1s(b)
        w.write(struct.pack(">I", len(pts)))
        for p_ in pts:
            w.write(_g1_encode(p_, raw))

    for p_ in (data.alpha1, data.beta1, data.delta1):
        w.write(_g1_encode(p_, raw))
    for v in (data.g1_A, data.g1_B, data.g1_Z, data.g1_K):
        vec1(v)
    w.write(_g2_encode(data.beta2, raw))
    w.write(_g2_encode(data.delta2, raw))
    g2 = [data.g2_B[i:i + 128] for i in range(0, len(data.g2_B), 128)]
    w.write(struct.pack(">I", len(g2)))
    for p_ in g2:
        w.write(_g2_encode(p_, raw))
    infA, infB = bytes(data.infinity_A), bytes(data.infinity_B)
    w.write(struct.pack(">QQQ", len(infA), sum(1 for c in infA if c), sum(1 for c in infB if c)))
    w.write(bytes(1 if c else 0 for c in infA))
    w.write(bytes(1 if c else 0 for c in infB))
    cks = commitment_keys or []
    w.write(struct.pack(">I", len(cks)))
    for basis, sigma in cks:
        vec1(basis)
        vec1(sigma)
    b = w.getvalue()
    if out is not None:
        out.write(b)
    return b


def read_proving_key(src: Union[bytes, BinaryIO], nb_public: int, k_wire_index=None):
    """ProvingKey.ReadFrom (marshal.go:309-374) into a `groth16.ProvingKeyData`
    (BN254); raw or compressed points, detected per point from the flag bits.
    nb_public comes from the R1CS (it is not part of the key).  Returns
    (ProvingKeyData, commitment_keys)."""
    from .groth16 import ProvingKeyData
    buf = src if isinstance(src, (bytes, bytearray)) else src.read()
    if len(buf) < _DOMAIN_BYTES:
        raise ValueError("pk: truncated domain")
    n = struct.unpack(">Q", buf[:8])[0]
    if n == 0 or n & (n - 1):
        raise ValueError("pk: domain cardinality is not a power of two")
    vals = [int.from_bytes(buf[8 + 32 * i:40 + 32 * i], "big") for i in range(5)]
    if any(v >= R for v in vals):
        raise ValueError("pk: domain element not reduced")
    _, omega, _, gen, _ = vals
    off = _DOMAIN_BYTES
    # raw keys have no compression flags on the first point; gnark decodes the
    # same way (per-point flag)
    raw = (buf[off] & _MASK) == _M_UNCOMPRESSED

    def need(k):
        if off + k > len(buf):
            raise ValueError("pk: truncated")

    def pt1():
        nonlocal off
        need(64 if raw else 32)
        p_, off = _g1_decode(buf, off, raw)
        return p_

    def pt2():
        nonlocal off
        need(128 if raw else 64)
        p_, off = _g2_decode(buf, off, raw)
        return p_

    def u32():
        nonlocal off
        need(4)
        v = struct.unpack(">I", buf[off:off + 4])[0]
        off += 4
        return v

    def vec(f):
        return b"".join(f() for _ in range(u32()))

    alpha1, beta1, delta1 = pt1(), pt1(), pt1()
    gA, gB, gZ, gK = vec(pt1), vec(pt1), vec(pt1), vec(pt1)
    beta2, delta2 = pt2(), pt2()
    g2B = vec(pt2)
    need(24)
    nw, ninfA, ninfB = struct.unpack(">QQQ", buf[off:off + 24])
    off += 24
    need(2 * nw)
    infA, infB = bytes(buf[off:off + nw]), bytes(buf[off + nw:off + 2 * nw])
    off += 2 * nw
    if any(c > 1 for c in infA + infB):
        raise ValueError("pk: infinity flags must be 0/1")
    if sum(infA) != ninfA or sum(infB) != ninfB:
        raise ValueError("pk: NbInfinityA/B disagree with the flags")
    if len(gA) // 64 != nw - ninfA or len(gB) // 64 != nw - ninfB or len(g2B) // 128 != nw - ninfB:
        raise ValueError("pk: point counts disagree with the infinity flags")
    cks = []
    for _ in range(u32()):
        cks.append((vec(pt1), vec(pt1)))
    log_n = n.bit_length() - 1
    data = ProvingKeyData(
        log_n=log_n, g1_A=gA, g1_B=gB, g1_Z=gZ, g1_K=gK, alpha1=alpha1, beta1=beta1, delta1=delta1,
        g2_B=g2B, beta2=beta2, delta2=delta2, infinity_A=infA, infinity_B=infB, nb_public=nb_public,
        domain_generator=fr.fr_mont(omega), domain_mul_gen=fr.fr_mont(gen), k_wire_index=k_wire_index)
    return data, cks
