// BN254 base field Fp, scalar field Fr and Fp2 for CDNA4 (gfx950) and host.
//
// Representation: 8 x u32 little-endian limbs, Montgomery form with R = 2^256.
// This is bit-identical in memory to gnark-crypto's fp.Element / fr.Element
// ([4]uint64 little-endian, R = 2^256), so buffers handed over by the Go side
// (icicle.go:44-126 call sites) are used without any conversion.
// Moduli: backend/groth16/bn254/solidity.go:41-42.
//
// Multiplication is CIOS with 32x32->64 products (v_mad_u64_u32 on gfx950);
// add/sub are v_add_co/v_addc chains via __builtin_addc/__builtin_subc.
// Both moduli are < 2^254, so a+b never overflows 256 bits and the CIOS
// accumulator never needs a 10th word.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#define GG_HD __host__ __device__ __forceinline__

namespace gg {

struct FpCfg {
    static constexpr int N = 8;
    static constexpr uint32_t P[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                      0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
    static constexpr uint32_t INV = 0xe4866389u;  // -p^-1 mod 2^32
    static constexpr uint64_t INV64 = 0x87d20782e4866389ull;  // -p^-1 mod 2^64
    static constexpr uint32_t ONE[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                        0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
    static constexpr uint32_t R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                       0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
};

struct FrCfg {
    static constexpr int N = 8;
    static constexpr uint32_t P[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                      0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
    static constexpr uint32_t INV = 0xefffffffu;
    static constexpr uint64_t INV64 = 0xc2e1f593efffffffull;
    static constexpr uint32_t ONE[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                        0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
    static constexpr uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                       0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
};

// BLS12-381 base field (381-bit, 12 x u32, R = 2^384) and scalar field (255-bit,
// 8 x u32, R = 2^256): gnark-crypto ecc/bls12-381 fp.Element ([6]uint64) /
// fr.Element ([4]uint64) layouts.  Moduli: std/math/emulated/emparams/emparams.go:145-171.
struct FpBlsCfg {
    static constexpr int N = 12;
    static constexpr uint32_t P[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu,
                                       0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u,
                                       0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
    static constexpr uint32_t INV = 0xfffcfffdu;
    static constexpr uint64_t INV64 = 0x89f3fffcfffcfffdull;
    static constexpr uint32_t ONE[12] = {0x0002fffdu, 0x76090000u, 0xc40c0002u, 0xebf4000bu,
                                         0x53c758bau, 0x5f489857u, 0x70525745u, 0x77ce5853u,
                                         0xa256ec6du, 0x5c071a97u, 0xfa80e493u, 0x15f65ec3u};
    static constexpr uint32_t R2[12] = {0x1c341746u, 0xf4df1f34u, 0x09d104f1u, 0x0a76e6a6u,
                                        0x4c95b6d5u, 0x8de5476cu, 0x939d83c0u, 0x67eb88a9u,
                                        0xb519952du, 0x9a793e85u, 0x92cae3aau, 0x11988fe5u};
};

struct FrBlsCfg {
    static constexpr int N = 8;
    static constexpr uint32_t P[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                      0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
    static constexpr uint32_t INV = 0xffffffffu;
    static constexpr uint64_t INV64 = 0xfffffffeffffffffull;
    static constexpr uint32_t ONE[8] = {0xfffffffeu, 0x00000001u, 0x00034802u, 0x5884b7fau,
                                        0xecbc4ff5u, 0x998c4fefu, 0xacc5056fu, 0x1824b159u};
    static constexpr uint32_t R2[8] = {0xf3f29c6du, 0xc999e990u, 0x87925c23u, 0x2b6cedcbu,
                                       0x7254398fu, 0x05d31496u, 0x9f59ff11u, 0x0748d9d9u};
};

template <class C>
struct Fe {
    uint32_t v[C::N];

    static GG_HD Fe zero() {
        Fe r;
#pragma unroll
        for (int i = 0; i < C::N; i++) r.v[i] = 0;
        return r;
    }
    static GG_HD Fe one() {
        Fe r;
#pragma unroll
        for (int i = 0; i < C::N; i++) r.v[i] = C::ONE[i];
        return r;
    }
    static GG_HD Fe r2() {
        Fe r;
#pragma unroll
        for (int i = 0; i < C::N; i++) r.v[i] = C::R2[i];
        return r;
    }
    static GG_HD Fe modulus() {
        Fe r;
#pragma unroll
        for (int i = 0; i < C::N; i++) r.v[i] = C::P[i];
        return r;
    }
    GG_HD bool is_zero() const {
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < C::N; i++) x |= v[i];
        return x == 0;
    }
    GG_HD bool operator==(const Fe& o) const {
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < C::N; i++) x |= v[i] ^ o.v[i];
        return x == 0;
    }
    GG_HD bool operator!=(const Fe& o) const { return !(*this == o); }
};

// r = a + b mod p   (inputs < p; p < 2^(32N-1), so no overflow)
template <class C>
GG_HD Fe<C> operator+(const Fe<C>& a, const Fe<C>& b) {
    Fe<C> r, s;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < C::N; i++) r.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < C::N; i++) s.v[i] = __builtin_subc(r.v[i], C::P[i], br, &br);
    // br == 0  <=>  r >= p
#pragma unroll
    for (int i = 0; i < C::N; i++) r.v[i] = br ? r.v[i] : s.v[i];
    return r;
}

template <class C>
GG_HD Fe<C> operator-(const Fe<C>& a, const Fe<C>& b) {
    Fe<C> r, s;
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < C::N; i++) r.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < C::N; i++) s.v[i] = __builtin_addc(r.v[i], C::P[i], c, &c);
#pragma unroll
    for (int i = 0; i < C::N; i++) r.v[i] = br ? s.v[i] : r.v[i];
    return r;
}

template <class C>
GG_HD Fe<C> operator-(const Fe<C>& a) {
    return Fe<C>::zero() - a;
}

template <class C>
GG_HD Fe<C> dbl(const Fe<C>& a) {
    return a + a;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Host side (epilogue, bucket-reduction tail): same Montgomery product on
// 4 x 64-bit limbs with 128-bit intermediates -- identical bytes, ~4x fewer
// host instructions than the 32-bit device formulation.
template <class C>
inline Fe<C> mont_mul_host(const Fe<C>& a, const Fe<C>& b) {
    typedef unsigned __int128 u128;
    constexpr int K = C::N / 2;  // 64-bit limbs
    uint64_t A[K], B[K], P[K], t[K + 2];
    for (int i = 0; i < K + 2; i++) t[i] = 0;
    for (int i = 0; i < K; i++) {
        A[i] = (uint64_t)a.v[2 * i] | ((uint64_t)a.v[2 * i + 1] << 32);
        B[i] = (uint64_t)b.v[2 * i] | ((uint64_t)b.v[2 * i + 1] << 32);
        P[i] = (uint64_t)C::P[2 * i] | ((uint64_t)C::P[2 * i + 1] << 32);
    }
    for (int i = 0; i < K; i++) {
        uint64_t carry = 0;
        for (int j = 0; j < K; j++) {
            u128 x = (u128)A[j] * B[i] + t[j] + carry;
            t[j] = (uint64_t)x;
            carry = (uint64_t)(x >> 64);
        }
        u128 x = (u128)t[K] + carry;
        t[K] = (uint64_t)x;
        t[K + 1] = (uint64_t)(x >> 64);
        uint64_t m = t[0] * C::INV64;
        x = (u128)m * P[0] + t[0];
        carry = (uint64_t)(x >> 64);
        for (int j = 1; j < K; j++) {
            x = (u128)m * P[j] + t[j] + carry;
            t[j - 1] = (uint64_t)x;
            carry = (uint64_t)(x >> 64);
        }
        x = (u128)t[K] + carry;
        t[K - 1] = (uint64_t)x;
        t[K] = t[K + 1] + (uint64_t)(x >> 64);
    }
    // conditional subtraction
    uint64_t s[K];
    uint64_t br = 0;
    for (int i = 0; i < K; i++) {
        u128 x = (u128)t[i] - P[i] - br;
        s[i] = (uint64_t)x;
        br = (uint64_t)(x >> 64) & 1;
    }
    bool ge = t[K] || !br;
    Fe<C> r;
    for (int i = 0; i < K; i++) {
        uint64_t v = ge ? s[i] : t[i];
        r.v[2 * i] = (uint32_t)v;
        r.v[2 * i + 1] = (uint32_t)(v >> 32);
    }
    return r;
}
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// acc(96 bit = {acc64, c2}) += x * y : one v_mad_u64_u32 with its carry-out in
// VCC folded into the third word by one v_addc (2 instructions per product).
__device__ __forceinline__ void mac96(uint64_t& acc, uint32_t& c2, uint32_t x, uint32_t y) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
        "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(acc), "+v"(c2)
        : "v"(x), "v"(y)
        : "vcc");
}
__device__ __forceinline__ void mac96s(uint64_t& acc, uint32_t& c2, uint32_t x, uint32_t y_sgpr) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
        "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(acc), "+v"(c2)
        : "v"(x), "s"(y_sgpr)
        : "vcc");
}

// Montgomery product by operand-interleaved product scanning (column-wise):
// column k accumulates a_i*b_{k-i} and m_i*p_{k-i} into a 96-bit accumulator;
// for k < 8 the new digit m_k = lo * (-p^-1) zeroes the column.  128
// v_mad_u64_u32 + 128 v_addc and no per-product 64-bit add/move chains (the
// CIOS form needs ~500 instructions, this one ~330).
template <class C>
__device__ __forceinline__ Fe<C> mont_mul_ps8(const Fe<C>& a, const Fe<C>& b) {
    const uint32_t a0 = a.v[0], a1 = a.v[1], a2 = a.v[2], a3 = a.v[3], a4 = a.v[4], a5 = a.v[5],
                   a6 = a.v[6], a7 = a.v[7];
    const uint32_t b0 = b.v[0], b1 = b.v[1], b2 = b.v[2], b3 = b.v[3], b4 = b.v[4], b5 = b.v[5],
                   b6 = b.v[6], b7 = b.v[7];
    const uint32_t P0 = C::P[0], P1 = C::P[1], P2 = C::P[2], P3 = C::P[3], P4 = C::P[4],
                   P5 = C::P[5], P6 = C::P[6], P7 = C::P[7], INV = C::INV;
    uint32_t m0, m1, m2, m3, m4, m5, m6, m7;
    uint32_t t[8];
    uint64_t acc = 0;
    uint32_t c2 = 0;
#include "mont_ps.inc"
    Fe<C> r, s;
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = __builtin_subc(t[i], C::P[i], br, &br);
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = br ? t[i] : s.v[i];
    return r;
}
// The same product without the final subtraction: t = (a b + m p) / R < a b / R + p,
// so a < 4p, b < p gives t < 2p whenever 4p < R (BN254 fr) -- the lazily reduced
// NTT butterflies (ntt.hip) keep their values below 2p
template <class C>
__device__ __forceinline__ Fe<C> mont_mul_ps8_nored(const Fe<C>& a, const Fe<C>& b) {
    const uint32_t a0 = a.v[0], a1 = a.v[1], a2 = a.v[2], a3 = a.v[3], a4 = a.v[4], a5 = a.v[5],
                   a6 = a.v[6], a7 = a.v[7];
    const uint32_t b0 = b.v[0], b1 = b.v[1], b2 = b.v[2], b3 = b.v[3], b4 = b.v[4], b5 = b.v[5],
                   b6 = b.v[6], b7 = b.v[7];
    const uint32_t P0 = C::P[0], P1 = C::P[1], P2 = C::P[2], P3 = C::P[3], P4 = C::P[4],
                   P5 = C::P[5], P6 = C::P[6], P7 = C::P[7], INV = C::INV;
    uint32_t m0, m1, m2, m3, m4, m5, m6, m7;
    uint32_t t[8];
    uint64_t acc = 0;
    uint32_t c2 = 0;
#include "mont_ps.inc"
    Fe<C> r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = t[i];
    return r;
}
// 12-limb (BLS12-381 Fp) product scanning: 288 v_mad_u64_u32 + 288 v_addc
template <class C>
__device__ __forceinline__ Fe<C> mont_mul_ps12(const Fe<C>& a, const Fe<C>& b) {
    const uint32_t a0 = a.v[0], a1 = a.v[1], a2 = a.v[2], a3 = a.v[3], a4 = a.v[4], a5 = a.v[5],
                   a6 = a.v[6], a7 = a.v[7], a8 = a.v[8], a9 = a.v[9], a10 = a.v[10], a11 = a.v[11];
    const uint32_t b0 = b.v[0], b1 = b.v[1], b2 = b.v[2], b3 = b.v[3], b4 = b.v[4], b5 = b.v[5],
                   b6 = b.v[6], b7 = b.v[7], b8 = b.v[8], b9 = b.v[9], b10 = b.v[10], b11 = b.v[11];
    const uint32_t P0 = C::P[0], P1 = C::P[1], P2 = C::P[2], P3 = C::P[3], P4 = C::P[4],
                   P5 = C::P[5], P6 = C::P[6], P7 = C::P[7], P8 = C::P[8], P9 = C::P[9],
                   P10 = C::P[10], P11 = C::P[11], INV = C::INV;
    uint32_t m0, m1, m2, m3, m4, m5, m6, m7, m8, m9, m10, m11;
    uint32_t t[12];
    uint64_t acc = 0;
    uint32_t c2 = 0;
#include "mont_ps12.inc"
    Fe<C> r, s;
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) s.v[i] = __builtin_subc(t[i], C::P[i], br, &br);
#pragma unroll
    for (int i = 0; i < 12; i++) r.v[i] = br ? t[i] : s.v[i];
    return r;
}
template <class C>
__device__ __forceinline__ Fe<C> mont_mul_ps(const Fe<C>& a, const Fe<C>& b) {
    if constexpr (C::N == 8) return mont_mul_ps8(a, b);
    else {
        static_assert(C::N == 12, "limb count");
        return mont_mul_ps12(a, b);
    }
}
#endif

// a b mod p as some representative < 2p (see mont_mul_ps8_nored; 8-limb fields)
template <class C>
GG_HD Fe<C> mul_nored(const Fe<C>& a, const Fe<C>& b) {
#if defined(__HIP_DEVICE_COMPILE__)
    static_assert(C::N == 8, "8-limb fields");
    return mont_mul_ps8_nored(a, b);
#else
    return mont_mul_host(a, b);  // canonical, also < 2p
#endif
}

#ifndef GG_MUL_CIOS
#define GG_MUL_CIOS 0
#endif

// Montgomery multiplication: product scanning on the device (GG_MUL_CIOS=1
// selects the portable CIOS form below), 64-bit limbs on the host.
template <class C>
GG_HD Fe<C> operator*(const Fe<C>& a, const Fe<C>& b) {
#if !defined(__HIP_DEVICE_COMPILE__)
    return mont_mul_host(a, b);
#elif !GG_MUL_CIOS
    return mont_mul_ps(a, b);
#else
    uint32_t t[C::N];
#pragma unroll
    for (int j = 0; j < C::N; j++) t[j] = 0;
#pragma unroll
    for (int i = 0; i < C::N; i++) {
        uint64_t acc = 0;
#pragma unroll
        for (int j = 0; j < C::N; j++) {
            acc = (uint64_t)a.v[j] * b.v[i] + t[j] + (acc >> 32);
            t[j] = (uint32_t)acc;
        }
        uint32_t t8 = (uint32_t)(acc >> 32);
        uint32_t m = t[0] * C::INV;
        acc = (uint64_t)m * C::P[0] + t[0];
#pragma unroll
        for (int j = 1; j < C::N; j++) {
            acc = (uint64_t)m * C::P[j] + t[j] + (acc >> 32);
            t[j - 1] = (uint32_t)acc;
        }
        t[C::N - 1] = t8 + (uint32_t)(acc >> 32);
    }
    Fe<C> r, s;
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < C::N; i++) s.v[i] = __builtin_subc(t[i], C::P[i], br, &br);
#pragma unroll
    for (int i = 0; i < C::N; i++) r.v[i] = br ? t[i] : s.v[i];
    return r;
#endif
}

template <class C>
GG_HD Fe<C> sqr(const Fe<C>& a) {
    return a * a;
}

template <class C>
GG_HD Fe<C> to_mont(const Fe<C>& a) {
    return a * Fe<C>::r2();
}

template <class C>
GG_HD Fe<C> from_mont(const Fe<C>& a) {
    Fe<C> one = Fe<C>::zero();
    one.v[0] = 1;
    return a * one;
}

// a^(p-2) (Fermat); a == 0 -> 0
template <class C>
GG_HD Fe<C> inverse(const Fe<C>& a) {
    // exponent p - 2, scanned from the top bit
    uint32_t e[C::N];
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < C::N; i++) e[i] = __builtin_subc(C::P[i], i == 0 ? 2u : 0u, br, &br);
    Fe<C> acc = Fe<C>::one();
    for (int i = 32 * C::N - 1; i >= 0; i--) {
        acc = sqr(acc);
        if ((e[i >> 5] >> (i & 31)) & 1) acc = acc * a;
    }
    return acc;
}

// x^e for a small exponent (host-side table building)
template <class C>
GG_HD Fe<C> pow_u64(const Fe<C>& x, uint64_t e) {
    Fe<C> acc = Fe<C>::one(), b = x;
    while (e) {
        if (e & 1) acc = acc * b;
        b = sqr(b);
        e >>= 1;
    }
    return acc;
}

using Fp = Fe<FpCfg>;
using Fr = Fe<FrCfg>;
using FpBls = Fe<FpBlsCfg>;
using FrBls = Fe<FrBlsCfg>;

// ---------------------------------------------------------------------------
// Fp2 = Fp[u] / (u^2 + 1)   (gnark-crypto bn254 E2 layout: {A0, A1})
// ---------------------------------------------------------------------------
struct Fp2 {
    Fp a0, a1;
    static GG_HD Fp2 zero() { return Fp2{Fp::zero(), Fp::zero()}; }
    static GG_HD Fp2 one() { return Fp2{Fp::one(), Fp::zero()}; }
    GG_HD bool is_zero() const { return a0.is_zero() && a1.is_zero(); }
    GG_HD bool operator==(const Fp2& o) const { return a0 == o.a0 && a1 == o.a1; }
};

GG_HD Fp2 operator+(const Fp2& a, const Fp2& b) { return Fp2{a.a0 + b.a0, a.a1 + b.a1}; }
GG_HD Fp2 operator-(const Fp2& a, const Fp2& b) { return Fp2{a.a0 - b.a0, a.a1 - b.a1}; }
GG_HD Fp2 operator-(const Fp2& a) { return Fp2{-a.a0, -a.a1}; }
GG_HD Fp2 dbl(const Fp2& a) { return Fp2{a.a0 + a.a0, a.a1 + a.a1}; }
#if defined(__HIP_DEVICE_COMPILE__)
#include "wide_redc.inc"
// 512-bit helpers (16 x u32, little endian)
__device__ __forceinline__ void add512(const uint32_t* x, const uint32_t* y, uint32_t* o) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) o[i] = __builtin_addc(x[i], y[i], c, &c);
}
__device__ __forceinline__ void sub512(const uint32_t* x, const uint32_t* y, uint32_t* o) {
    uint32_t b = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) o[i] = __builtin_subc(x[i], y[i], b, &b);
}
#define GG_WIDE_OPERANDS(A, B)                                                                  \
    const uint32_t a0 = (A).v[0], a1 = (A).v[1], a2 = (A).v[2], a3 = (A).v[3], a4 = (A).v[4],     \
                   a5 = (A).v[5], a6 = (A).v[6], a7 = (A).v[7];                                    \
    const uint32_t b0 = (B).v[0], b1 = (B).v[1], b2 = (B).v[2], b3 = (B).v[3], b4 = (B).v[4],     \
                   b5 = (B).v[5], b6 = (B).v[6], b7 = (B).v[7];
// Montgomery reduction T * 2^-256 mod p of T < p * 2^256, canonical result
__device__ __forceinline__ Fp fp_redc(const uint32_t* Tin) {
    const uint32_t T0 = Tin[0], T1 = Tin[1], T2 = Tin[2], T3 = Tin[3], T4 = Tin[4], T5 = Tin[5],
                   T6 = Tin[6], T7 = Tin[7], T8 = Tin[8], T9 = Tin[9], T10 = Tin[10], T11 = Tin[11],
                   T12 = Tin[12], T13 = Tin[13], T14 = Tin[14], T15 = Tin[15];
    const uint32_t P0 = FpCfg::P[0], P1 = FpCfg::P[1], P2 = FpCfg::P[2], P3 = FpCfg::P[3],
                   P4 = FpCfg::P[4], P5 = FpCfg::P[5], P6 = FpCfg::P[6], P7 = FpCfg::P[7],
                   INV = FpCfg::INV;
    uint32_t m0, m1, m2, m3, m4, m5, m6, m7;
    uint32_t r[8];
    GG_REDC_BODY
    Fp o, d;
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d.v[i] = __builtin_subc(r[i], FpCfg::P[i], br, &br);
#pragma unroll
    for (int i = 0; i < 8; i++) o.v[i] = br ? r[i] : d.v[i];
    return o;
}
// Fp2 product with lazy reduction (Karatsuba on 512-bit products, 2 reductions
// instead of 3): c0 = REDC(a0b0 - a1b1 + p^2), c1 = REDC((a0+a1)(b0+b1) - a0b0 - a1b1);
// both arguments are < 2p^2 < p * 2^256 (p < 2^254).  The products' digits are
// folded into the two 512-bit accumulators column by column (no 512-bit temporaries).
__device__ __forceinline__ Fp2 fp2_mul_lazy(const Fp2& x, const Fp2& y) {
    uint32_t S[16], U[16];
    {  // S = (x0 + x1)(y0 + y1), sums unreduced (< 2p < 2^255)
        Fp sa, sb;
        uint32_t ca = 0, cb = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            sa.v[i] = __builtin_addc(x.a0.v[i], x.a1.v[i], ca, &ca);
            sb.v[i] = __builtin_addc(y.a0.v[i], y.a1.v[i], cb, &cb);
        }
        GG_WIDE_OPERANDS(sa, sb)
#define GG_WIDE_COL(k, d) S[k] = (d);
        GG_WIDE_BODY
#undef GG_WIDE_COL
    }
    {  // t0 = x0 y0: S -= t0, U = t0 + p^2
        GG_WIDE_OPERANDS(x.a0, y.a0)
        uint32_t bs = 0, cu = 0;
#define GG_WIDE_COL(k, d)                                          \
    {                                                              \
        const uint32_t d_ = (d);                                   \
        S[k] = __builtin_subc(S[k], d_, bs, &bs);                  \
        U[k] = __builtin_addc(d_, kFpP2[k], cu, &cu);              \
    }
        GG_WIDE_BODY
#undef GG_WIDE_COL
    }
    {  // t1 = x1 y1: S -= t1, U -= t1
        GG_WIDE_OPERANDS(x.a1, y.a1)
        uint32_t bs = 0, bu = 0;
#define GG_WIDE_COL(k, d)                                          \
    {                                                              \
        const uint32_t d_ = (d);                                   \
        S[k] = __builtin_subc(S[k], d_, bs, &bs);                  \
        U[k] = __builtin_subc(U[k], d_, bu, &bu);                  \
    }
        GG_WIDE_BODY
#undef GG_WIDE_COL
    }
    return Fp2{fp_redc(U), fp_redc(S)};
}
// a*b - c*d with one Montgomery reduction: REDC(a*b + p^2 - c*d), the argument
// in (0, 2p^2) < p * 2^256 (inputs canonical, p < 2^254); canonical result.
__device__ __forceinline__ Fp fp_mul_sub_lazy(const Fp& x, const Fp& y, const Fp& z, const Fp& w) {
    uint32_t U[16];
    {
        GG_WIDE_OPERANDS(x, y)
        uint32_t cu = 0;
#define GG_WIDE_COL(k, dd) U[k] = __builtin_addc((dd), kFpP2[k], cu, &cu);
        GG_WIDE_BODY
#undef GG_WIDE_COL
    }
    {
        GG_WIDE_OPERANDS(z, w)
        uint32_t bu = 0;
#define GG_WIDE_COL(k, dd) U[k] = __builtin_subc(U[k], (dd), bu, &bu);
        GG_WIDE_BODY
#undef GG_WIDE_COL
    }
    return fp_redc(U);
}
#endif

// a*b - c*d (lazily reduced for BN254 Fp on the device)
template <class F>
GG_HD F mul_sub(const F& a, const F& b, const F& c, const F& d) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (std::is_same<F, Fp>::value) return fp_mul_sub_lazy(a, b, c, d);
    else
#endif
        return a * b - c * d;
}

#ifndef GG_FP2_PLAIN
#define GG_FP2_PLAIN 0
#endif
GG_HD Fp2 operator*(const Fp2& a, const Fp2& b) {
#if defined(__HIP_DEVICE_COMPILE__) && !GG_FP2_PLAIN
    return fp2_mul_lazy(a, b);
#else
    Fp t0 = a.a0 * b.a0;
    Fp t1 = a.a1 * b.a1;
    Fp t2 = (a.a0 + a.a1) * (b.a0 + b.a1);
    return Fp2{t0 - t1, t2 - t0 - t1};
#endif
}
GG_HD Fp2 sqr(const Fp2& a) {
    Fp t0 = (a.a0 + a.a1) * (a.a0 - a.a1);
    Fp t1 = a.a0 * a.a1;
    return Fp2{t0, t1 + t1};
}
GG_HD Fp2 inverse(const Fp2& a) {
    Fp n = sqr(a.a0) + sqr(a.a1);
    Fp ni = inverse(n);
    return Fp2{a.a0 * ni, -(a.a1 * ni)};
}

// ---------------------------------------------------------------------------
// Fp2 over BLS12-381 Fp = Fp[u] / (u^2 + 1) (gnark-crypto ecc/bls12-381 E2
// layout {A0, A1}: 2 x 48 B): the field of the G2 points of a BLS12-381
// Groth16 key (backend/groth16/bls12-381/setup.go).  Karatsuba product (three
// 12-limb Montgomery products), complex squaring (two).
// ---------------------------------------------------------------------------
struct Fp2Bls {
    FpBls a0, a1;
    static GG_HD Fp2Bls zero() { return Fp2Bls{FpBls::zero(), FpBls::zero()}; }
    static GG_HD Fp2Bls one() { return Fp2Bls{FpBls::one(), FpBls::zero()}; }
    GG_HD bool is_zero() const { return a0.is_zero() && a1.is_zero(); }
    GG_HD bool operator==(const Fp2Bls& o) const { return a0 == o.a0 && a1 == o.a1; }
    GG_HD bool operator!=(const Fp2Bls& o) const { return !(*this == o); }
};
GG_HD Fp2Bls operator+(const Fp2Bls& a, const Fp2Bls& b) { return Fp2Bls{a.a0 + b.a0, a.a1 + b.a1}; }
GG_HD Fp2Bls operator-(const Fp2Bls& a, const Fp2Bls& b) { return Fp2Bls{a.a0 - b.a0, a.a1 - b.a1}; }
GG_HD Fp2Bls operator-(const Fp2Bls& a) { return Fp2Bls{-a.a0, -a.a1}; }
GG_HD Fp2Bls dbl(const Fp2Bls& a) { return Fp2Bls{a.a0 + a.a0, a.a1 + a.a1}; }
GG_HD Fp2Bls operator*(const Fp2Bls& a, const Fp2Bls& b) {
    const FpBls t0 = a.a0 * b.a0, t1 = a.a1 * b.a1;
    const FpBls t2 = (a.a0 + a.a1) * (b.a0 + b.a1);
    return Fp2Bls{t0 - t1, t2 - t0 - t1};
}
GG_HD Fp2Bls sqr(const Fp2Bls& a) {
    const FpBls t0 = (a.a0 + a.a1) * (a.a0 - a.a1);
    const FpBls t1 = a.a0 * a.a1;
    return Fp2Bls{t0, t1 + t1};
}
GG_HD Fp2Bls inverse(const Fp2Bls& a) {
    const FpBls ni = inverse(sqr(a.a0) + sqr(a.a1));
    return Fp2Bls{a.a0 * ni, -(a.a1 * ni)};
}

}  // namespace gg
