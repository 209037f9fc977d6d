"""Constants of the reduced-radix Montgomery configurations in
gnark-fork_amd/csrc/field29.cuh (printed as C++ initialisers):
BN254 Fp in 9 x 29-bit limbs (R' = 2^261) and BLS12-381 Fp in 14 x 28-bit
limbs (R' = 2^392).  KP[k-1] = k p with limbs 0..N-2 borrowed into [2^B, 2^(B+1))."""
import sys


def limbs(x, n, b):
    m = (1 << b) - 1
    return [(x >> (b * i)) & m for i in range(n - 1)] + [x >> (b * (n - 1))]


def words(x, n):
    return [(x >> (32 * i)) & 0xffffffff for i in range(n)]


def cfg(name, p, n, b, r32_words):
    M = 1 << (n * b)
    R32 = 1 << (32 * r32_words)
    h = lambda v: "0x%08xu" % v
    out = [f"// {name}: N = {n}, B = {b}, M / p = {M / p:.2f}"]
    out.append("P = {" + ", ".join(h(v) for v in limbs(p, n, b)) + "}")
    out.append("INV = " + h((-pow(p, -1, 1 << b)) % (1 << b)))
    out.append("PINV = " + h(pow(p, -1, 1 << b)))
    out.append("ONE = {" + ", ".join(h(v) for v in limbs(M % p, n, b)) + "}")
    out.append("C_OUT = {" + ", ".join(h(v) for v in limbs(R32 % p, n, b)) + "}")
    out.append("C_IN = {" + ", ".join(h(v) for v in words(M % p, r32_words)) + "}")
    for k in range(1, 9):
        d = limbs(k * p, n, b)
        kb = [d[i] + (1 << b) - (0 if i == 0 else 1) for i in range(n - 1)] + [d[n - 1] - 1]
        assert sum(v << (b * i) for i, v in enumerate(kb)) == k * p
        assert all((1 << b) <= v < (1 << (b + 1)) for v in kb[:-1])
        out.append("KP[%d] = {" % (k - 1) + ", ".join(h(v) for v in kb) + "}")
    return "\n".join(out)


if __name__ == "__main__":
    bn = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
    bls = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
    print(cfg("BN254 Fp", bn, 9, 29, 8))
    print(cfg("BLS12-381 Fp", bls, 14, 28, 12))
    sys.exit(0)
