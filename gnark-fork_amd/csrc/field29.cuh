// Reduced-radix Montgomery arithmetic for the bucket-accumulation hot loop.
//
// An element of BN254 Fp is held as 9 limbs of 29 bits (261 bits) in
// Montgomery form with R' = 2^261, lazily reduced (value < a small multiple of
// p, tracked per call site).  Why: on gfx950 the 32-bit-limb product-scanning
// multiply (field.cuh) spends one v_addc per v_mad_u64_u32 to fold the column
// carry (128 + 128 instructions plus the final subtraction).  With 29-bit limbs
// a column of the Montgomery product is at most 18 products of < 2^58 (or 9 of
// < 2^60 plus 9 of < 2^58 when one operand is an unnormalised sum), which fits
// a 64-bit accumulator with no carry-out: 162 v_mad_u64_u32 and ~60 shifts /
// masks, no carry chain, no final subtraction.
//
// The representation never leaves the accumulation kernels: base points are
// stored as x * 2^261 mod p (canonical, packed into the 8 x u32 gnark layout,
// prepared once when the base is built) and unpacked with funnel shifts; the
// bucket partials are converted back to gnark's x * 2^256 mod p (canonical)
// before they are written.  Results are therefore bit-identical to the
// 32-bit-limb path.
//
// Bounds (M = 2^261 = 169.28 p):
//   mul(a, b) < a b / M + p      (any a, b < 2^260 with limbs < 2^30)
//   sub<k>(a, b) = a + k p - b   (requires b < (k - 1) p + 2^232, so the
//                                 borrowed limbs of k p dominate b's)
#pragma once
#include "curve.cuh"

// Column schedule of the product-scanning loops.  GG_R29_SPLIT = 1: the
// operand products of a column go to their own accumulator, added once to the
// running (carry + reduction) accumulator -- they do not depend on the
// previous column's reduction digit, so the two chains interleave (ILP 2).
#ifndef GG_R29_SPLIT
#define GG_R29_SPLIT 0
#endif
#if GG_R29_SPLIT
#define GG_COL_BEGIN uint64_t col_ = 0;
#define GG_COL_ACC col_
#define GG_COL_END acc += col_;
#else
#define GG_COL_BEGIN
#define GG_COL_ACC acc
#define GG_COL_END
#endif

namespace gg {

struct Fp29Cfg {
    using Std = FpCfg;  // the gnark (32-bit limb, R = 2^256) layout of the same field
    static constexpr int N = 9;
    static constexpr int B = 29;
    static constexpr uint32_t MASK = (1u << B) - 1;
    static constexpr uint32_t P[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u,
                                      0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
    // 2^261 mod p: one in R' form
    static constexpr uint32_t ONE[9] = {0x157ccc21u, 0x141c2758u, 0x185230d3u, 0x014c0419u, 0x0aa36fb9u,
                                        0x1d4240ceu, 0x11d54c07u, 0x052ac7a8u, 0x000dc836u};
    static constexpr uint32_t INV = 0x04866389u;   // -p^-1 mod 2^29
    static constexpr uint32_t PINV = 0x1b799c77u;  // p^-1 mod 2^29
    // 2^256 mod p as a 29-bit-limb integer: mul(x * 2^261, C_OUT) = x * 2^256
    static constexpr uint32_t C_OUT[9] = {0x058f0d9du, 0x1aea1c6eu, 0x11c2cf74u, 0x11d651ebu, 0x1462c0a7u,
                                          0x11b7bc3cu, 0x1cbd99bau, 0x183340fbu, 0x000e0a77u};
    // 2^266 mod p as limbs: mul(x * 2^256 (unpacked), C_LOAD) = x * 2^261 (from_std)
    static constexpr uint32_t C_LOAD[9] = {0x13349ca1u, 0x1a5d84a8u, 0x0a3e5cacu, 0x100249e0u, 0x12b951e8u,
                                           0x0e92d304u, 0x14cb95b3u, 0x041b9d3du, 0x00058003u};
    // 2^261 mod p in the gnark 32-bit layout: mont256(x * 2^256, C_IN) = x * 2^261
    static constexpr uint32_t C_IN[8] = {0x157ccc21u, 0x4e8384ebu, 0x0ce148c3u, 0xfb90a602u,
                                         0x819caa36u, 0x5301fa84u, 0x563d4475u, 0x0dc83629u};
    // k p (k = 1..8) with limbs 0..7 borrowed into [2^29, 2^30): k p - b limb by
    // limb never goes negative for normalised b < (k - 1) p + 2^232.
    static constexpr uint32_t KP[8][9] = {
        {0x387cfd47u, 0x210460b5u, 0x3c72a34eu, 0x22d522cfu, 0x3585d977u, 0x22db40bfu, 0x20a6e140u, 0x2e5c2633u, 0x0030644du},
        {0x30f9fa8eu, 0x2208c16cu, 0x38e5469du, 0x25aa45a0u, 0x2b0bb2efu, 0x25b68180u, 0x214dc281u, 0x3cb84c67u, 0x0060c89bu},
        {0x2976f7d5u, 0x230d2223u, 0x3557e9ecu, 0x287f6871u, 0x20918c67u, 0x2891c241u, 0x21f4a3c2u, 0x2b14729bu, 0x00912ceau},
        {0x21f3f51cu, 0x241182dau, 0x31ca8d3bu, 0x2b548b42u, 0x361765dfu, 0x2b6d0301u, 0x229b8503u, 0x397098cfu, 0x00c19138u},
        {0x3a70f263u, 0x2515e390u, 0x2e3d308au, 0x2e29ae13u, 0x2b9d3f57u, 0x2e4843c2u, 0x23426644u, 0x27ccbf03u, 0x00f1f587u},
        {0x32edefaau, 0x261a4447u, 0x2aafd3d9u, 0x30fed0e4u, 0x212318cfu, 0x31238483u, 0x23e94785u, 0x3628e537u, 0x012259d5u},
        {0x2b6aecf1u, 0x271ea4feu, 0x27227728u, 0x33d3f3b5u, 0x36a8f247u, 0x33fec543u, 0x249028c6u, 0x24850b6bu, 0x0152be24u},
        {0x23e7ea38u, 0x282305b5u, 0x23951a77u, 0x36a91686u, 0x2c2ecbbfu, 0x36da0604u, 0x25370a07u, 0x32e1319fu, 0x01832272u}};
    // 5 p with limbs 0..7 in [2^31 - 4, 2^31 + 2^29): dominates every limb of an
    // unnormalised sum of three normalised values (< 3 * 2^29), see sqr_subw5
    static constexpr uint32_t KPW5[9] = {0x9a70f263u, 0x8515e38du, 0x8e3d3087u, 0x8e29ae10u, 0x8b9d3f54u,
                                         0x8e4843bfu, 0x83426641u, 0x87ccbf00u, 0x00f1f584u};
};

// BLS12-381 Fp in 14 x 28-bit limbs, R' = 2^392 = 2520 p: a column is at most
// 28 products of < 2^56 (mul4: 70), far inside 64 bits.  tools/gen_field29.py
struct FpBls28Cfg {
    using Std = FpBlsCfg;
    static constexpr int N = 14;
    static constexpr int B = 28;
    static constexpr uint32_t MASK = (1u << B) - 1;
    static constexpr uint32_t P[14] = {0x0fffaaabu, 0x0fefffffu, 0x03ffffb9u, 0x0fffeb15u, 0x06241eabu,
                                       0x0a0f6b0fu, 0x0f6730d2u, 0x0f38512bu, 0x04774b84u, 0x04bacd76u,
                                       0x0ba7b643u, 0x0e69a4b1u, 0x01ea397fu, 0x0001a011u};
    static constexpr uint32_t ONE[14] = {0x0347fcb8u, 0x0d800000u, 0x0002b119u, 0x00cde6d2u, 0x0c7212e0u,
                                         0x083a2090u, 0x0037669fu, 0x0da0f73eu, 0x09b09b42u, 0x01297bb0u,
                                         0x0515d98fu, 0x0012ca7cu, 0x0659fcfau, 0x0000577au};
    static constexpr uint32_t INV = 0x0ffcfffdu;
    static constexpr uint32_t PINV = 0x00030003u;
    static constexpr uint32_t C_OUT[14] = {0x0002fffdu, 0x00900000u, 0x0c000276u, 0x0000bc40u, 0x08baebf4u,
                                           0x05753c75u, 0x055f4898u, 0x07052574u, 0x07ce5853u, 0x056ec6d7u,
                                           0x071a97a2u, 0x0e4935c0u, 0x0ec3fa80u, 0x00015f65u};
    static constexpr uint32_t C_LOAD[14] = {0x080e6299u, 0x03500034u, 0x0eb12856u, 0x0deb2699u, 0x0c988670u,
                                            0x04ef6697u, 0x070983e8u, 0x0a4e6fe9u, 0x03e8a053u, 0x0ecf271eu,
                                            0x0c20d323u, 0x06eb6385u, 0x047f1286u, 0x000156dau};  // 2^400 mod p
    static constexpr uint32_t C_IN[12] = {0x0347fcb8u, 0x19d80000u, 0x6d2002b1u, 0x12e00cdeu, 0xa2090c72u, 0x37669f83u,
                                          0xda0f73e0u, 0x09b09b42u, 0x8f1297bbu, 0xa7c515d9u, 0xfcfa012cu, 0x0577a659u};
    static constexpr uint32_t KP[8][14] = {
        {0x1fffaaabu, 0x1feffffeu, 0x13ffffb8u, 0x1fffeb14u, 0x16241eaau, 0x1a0f6b0eu, 0x1f6730d1u, 0x1f38512au, 0x14774b83u, 0x14bacd75u, 0x1ba7b642u, 0x1e69a4b0u, 0x11ea397eu, 0x0001a010u},
        {0x1fff5556u, 0x1fdffffeu, 0x17ffff72u, 0x1fffd629u, 0x1c483d56u, 0x141ed61du, 0x1ece61a4u, 0x1e70a256u, 0x18ee9708u, 0x19759aebu, 0x174f6c85u, 0x1cd34962u, 0x13d472feu, 0x00034021u},
        {0x1fff0001u, 0x1fcffffeu, 0x1bffff2cu, 0x1fffc13eu, 0x126c5c02u, 0x1e2e412du, 0x1e359276u, 0x1da8f382u, 0x1d65e28du, 0x1e306861u, 0x12f722c8u, 0x1b3cee14u, 0x15beac7eu, 0x0004e032u},
        {0x1ffeaaacu, 0x1fbffffeu, 0x1ffffee6u, 0x1fffac53u, 0x18907aaeu, 0x183dac3cu, 0x1d9cc349u, 0x1ce144aeu, 0x11dd2e12u, 0x12eb35d8u, 0x1e9ed90cu, 0x19a692c5u, 0x17a8e5feu, 0x00068043u},
        {0x1ffe5557u, 0x1faffffeu, 0x13fffea0u, 0x1fff9769u, 0x1eb4995au, 0x124d174bu, 0x1d03f41cu, 0x1c1995dau, 0x16547997u, 0x17a6034eu, 0x1a468f4fu, 0x18103777u, 0x19931f7eu, 0x00082054u},
        {0x1ffe0002u, 0x1f9ffffeu, 0x17fffe5au, 0x1fff827eu, 0x14d8b806u, 0x1c5c825bu, 0x1c6b24eeu, 0x1b51e706u, 0x1acbc51cu, 0x1c60d0c4u, 0x15ee4592u, 0x1679dc29u, 0x1b7d58feu, 0x0009c065u},
        {0x1ffdaaadu, 0x1f8ffffeu, 0x1bfffe14u, 0x1fff6d93u, 0x1afcd6b2u, 0x166bed6au, 0x1bd255c1u, 0x1a8a3832u, 0x1f4310a1u, 0x111b9e3au, 0x1195fbd6u, 0x14e380dbu, 0x1d67927eu, 0x000b6076u},
        {0x1ffd5558u, 0x1f7ffffeu, 0x1ffffdceu, 0x1fff58a8u, 0x1120f55eu, 0x107b587au, 0x1b398694u, 0x19c2895eu, 0x13ba5c26u, 0x15d66bb1u, 0x1d3db219u, 0x134d258cu, 0x1f51cbfeu, 0x000d0087u}};
    // 5 p with limbs 0..12 in [2^30 - 4, 2^30 + 2^28) (see Fp29Cfg::KPW5)
    static constexpr uint32_t KPW5[14] = {0x4ffe5557u, 0x4faffffbu, 0x43fffe9du, 0x4fff9766u, 0x4eb49957u,
                                          0x424d1748u, 0x4d03f419u, 0x4c1995d7u, 0x46547994u, 0x47a6034bu,
                                          0x4a468f4cu, 0x48103774u, 0x49931f7bu, 0x00082051u};
};

template <class C>
struct Fl {
    uint32_t l[C::N];
};
using Fp29 = Fl<Fp29Cfg>;
using FpBls28 = Fl<FpBls28Cfg>;

// Montgomery product a b / 2^(B N) by operand-interleaved product scanning.
// Output limbs 0..N-2 < 2^B (normalised); value < a b / M + p.
template <class C>
__device__ __forceinline__ Fl<C> mul(const Fl<C>& a, const Fl<C>& b) {
    constexpr int N = C::N, B = C::B;
    uint32_t m[N];
    Fl<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * N - 1; k++) {
        GG_COL_BEGIN
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++)
            GG_COL_ACC += (uint64_t)a.l[i] * b.l[k - i];
        GG_COL_END
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k - 1 : N - 1); i++)
            acc += (uint64_t)m[i] * C::P[k - i];
        if (k < N) {
            m[k] = ((uint32_t)acc * C::INV) & C::MASK;
            acc += (uint64_t)m[k] * C::P[0];
        } else {
            r.l[k - N] = (uint32_t)acc & C::MASK;
        }
        acc >>= B;
    }
    r.l[N - 1] = (uint32_t)acc;
    return r;
}

// a^2: the off-diagonal products once, doubled with one shift-add per column
template <class C>
__device__ __forceinline__ Fl<C> sqr(const Fl<C>& a) {
    constexpr int N = C::N, B = C::B;
    uint32_t m[N];
    Fl<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * N - 1; k++) {
        uint64_t s = 0;
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); 2 * i < k; i++) s += (uint64_t)a.l[i] * a.l[k - i];
        if ((k & 1) == 0) s = (s << 1) + (uint64_t)a.l[k / 2] * a.l[k / 2];
        else s <<= 1;
        acc += s;
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k - 1 : N - 1); i++)
            acc += (uint64_t)m[i] * C::P[k - i];
        if (k < N) {
            m[k] = ((uint32_t)acc * C::INV) & C::MASK;
            acc += (uint64_t)m[k] * C::P[0];
        } else {
            r.l[k - N] = (uint32_t)acc & C::MASK;
        }
        acc >>= B;
    }
    r.l[N - 1] = (uint32_t)acc;
    return r;
}

// a b + c d with one reduction: (a b + c d) / M, value < (a b + c d) / M + p.
// A column holds 18 products and 9 reduction products of < 2^58: < 2^63.
template <class C>
__device__ __forceinline__ Fl<C> mul2(const Fl<C>& a, const Fl<C>& b, const Fl<C>& c, const Fl<C>& d) {
    constexpr int N = C::N, B = C::B;
    uint32_t m[N];
    Fl<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * N - 1; k++) {
        GG_COL_BEGIN
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) {
            GG_COL_ACC += (uint64_t)a.l[i] * b.l[k - i];
            GG_COL_ACC += (uint64_t)c.l[i] * d.l[k - i];
        }
        GG_COL_END
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k - 1 : N - 1); i++)
            acc += (uint64_t)m[i] * C::P[k - i];
        if (k < N) {
            m[k] = ((uint32_t)acc * C::INV) & C::MASK;
            acc += (uint64_t)m[k] * C::P[0];
        } else {
            r.l[k - N] = (uint32_t)acc & C::MASK;
        }
        acc >>= B;
    }
    r.l[N - 1] = (uint32_t)acc;
    return r;
}

// a^2 / M + 5 p - s, s an UNNORMALISED sum of three normalised values (limbs
// < 3 * 2^B, value < 5 p): the subtraction is folded into the output columns
// against KPW5, whose limbs dominate s's, so every column term is >= 0; the
// reduction's carry chain normalises the result
template <class C>
__device__ __forceinline__ Fl<C> sqr_subw5(const Fl<C>& a, const Fl<C>& s) {
    constexpr int N = C::N, B = C::B;
    uint32_t m[N];
    Fl<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * N - 1; k++) {
        uint64_t t = 0;
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); 2 * i < k; i++) t += (uint64_t)a.l[i] * a.l[k - i];
        if ((k & 1) == 0) t = (t << 1) + (uint64_t)a.l[k / 2] * a.l[k / 2];
        else t <<= 1;
        acc += t;
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k - 1 : N - 1); i++)
            acc += (uint64_t)m[i] * C::P[k - i];
        if (k < N) {
            m[k] = ((uint32_t)acc * C::INV) & C::MASK;
            acc += (uint64_t)m[k] * C::P[0];
        } else {
            acc += C::KPW5[k - N] - s.l[k - N];
            r.l[k - N] = (uint32_t)acc & C::MASK;
        }
        acc >>= B;
    }
    r.l[N - 1] = (uint32_t)acc + (C::KPW5[N - 1] - s.l[N - 1]);
    return r;
}

// a b / M + K p - s with the subtraction folded into the output columns (the
// reduction's carry chain normalises it): same bound rule on s as sub<K>
template <int K, class C>
__device__ __forceinline__ Fl<C> mul_sub(const Fl<C>& a, const Fl<C>& b, const Fl<C>& s) {
    static_assert(K >= 1 && K <= 8, "multiple of p");
    constexpr int N = C::N, B = C::B;
    uint32_t m[N];
    Fl<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * N - 1; k++) {
        GG_COL_BEGIN
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++)
            GG_COL_ACC += (uint64_t)a.l[i] * b.l[k - i];
        GG_COL_END
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k - 1 : N - 1); i++)
            acc += (uint64_t)m[i] * C::P[k - i];
        if (k < N) {
            m[k] = ((uint32_t)acc * C::INV) & C::MASK;
            acc += (uint64_t)m[k] * C::P[0];
        } else {
            acc += C::KP[K - 1][k - N] - s.l[k - N];
            r.l[k - N] = (uint32_t)acc & C::MASK;
        }
        acc >>= B;
    }
    r.l[N - 1] = (uint32_t)acc + (C::KP[K - 1][N - 1] - s.l[N - 1]);
    return r;
}

// (a b + c d) / M + K p - s: mul2 with the subtraction folded into the output
// columns (bound rule on s as sub<K>)
template <int K, class C>
__device__ __forceinline__ Fl<C> mul2_sub(const Fl<C>& a, const Fl<C>& b, const Fl<C>& c, const Fl<C>& d,
                                          const Fl<C>& s) {
    static_assert(K >= 1 && K <= 8, "multiple of p");
    constexpr int N = C::N, B = C::B;
    uint32_t m[N];
    Fl<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * N - 1; k++) {
        GG_COL_BEGIN
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) {
            GG_COL_ACC += (uint64_t)a.l[i] * b.l[k - i];
            GG_COL_ACC += (uint64_t)c.l[i] * d.l[k - i];
        }
        GG_COL_END
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k - 1 : N - 1); i++)
            acc += (uint64_t)m[i] * C::P[k - i];
        if (k < N) {
            m[k] = ((uint32_t)acc * C::INV) & C::MASK;
            acc += (uint64_t)m[k] * C::P[0];
        } else {
            acc += C::KP[K - 1][k - N] - s.l[k - N];
            r.l[k - N] = (uint32_t)acc & C::MASK;
        }
        acc >>= B;
    }
    r.l[N - 1] = (uint32_t)acc + (C::KP[K - 1][N - 1] - s.l[N - 1]);
    return r;
}

// (a b + c d + e f + g h) / M with one reduction: a column holds 36 products
// and 9 reduction products of < 2^58 (< 2^63.5)
template <class C>
__device__ __forceinline__ Fl<C> mul4(const Fl<C>& a, const Fl<C>& b, const Fl<C>& c, const Fl<C>& d,
                                      const Fl<C>& e, const Fl<C>& f, const Fl<C>& g, const Fl<C>& h) {
    constexpr int N = C::N, B = C::B;
    uint32_t m[N];
    Fl<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * N - 1; k++) {
        GG_COL_BEGIN
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) {
            GG_COL_ACC += (uint64_t)a.l[i] * b.l[k - i];
            GG_COL_ACC += (uint64_t)c.l[i] * d.l[k - i];
            GG_COL_ACC += (uint64_t)e.l[i] * f.l[k - i];
            GG_COL_ACC += (uint64_t)g.l[i] * h.l[k - i];
        }
        GG_COL_END
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k - 1 : N - 1); i++)
            acc += (uint64_t)m[i] * C::P[k - i];
        if (k < N) {
            m[k] = ((uint32_t)acc * C::INV) & C::MASK;
            acc += (uint64_t)m[k] * C::P[0];
        } else {
            r.l[k - N] = (uint32_t)acc & C::MASK;
        }
        acc >>= B;
    }
    r.l[N - 1] = (uint32_t)acc;
    return r;
}

// v - q p with q = floor(v_top / (p_top + 1)) <= floor(v / p): a normalised
// v < 8 p comes out < 2 p (nine products, no comparison)
template <class C>
__device__ __forceinline__ Fl<C> reduce_small(const Fl<C>& v) {
    const uint32_t q = v.l[C::N - 1] / (C::P[C::N - 1] + 1);
    Fl<C> r;
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < C::N - 1; i++) {
        acc += (int64_t)v.l[i] - (int64_t)((uint64_t)q * C::P[i]);
        r.l[i] = (uint32_t)acc & C::MASK;
        acc >>= C::B;  // arithmetic: the borrow
    }
    r.l[C::N - 1] = (uint32_t)((int64_t)v.l[C::N - 1] - (int64_t)((uint64_t)q * C::P[C::N - 1]) + acc);
    return r;
}

// a + b, normalised
template <class C>
__device__ __forceinline__ Fl<C> add(const Fl<C>& a, const Fl<C>& b) {
    Fl<C> r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < C::N - 1; i++) {
        const uint32_t t = a.l[i] + b.l[i] + c;
        r.l[i] = t & C::MASK;
        c = t >> C::B;
    }
    r.l[C::N - 1] = a.l[C::N - 1] + b.l[C::N - 1] + c;
    return r;
}

// a + k p - b, normalised (b < (k - 1) p + 2^232, see KP)
template <int K, class C>
__device__ __forceinline__ Fl<C> sub(const Fl<C>& a, const Fl<C>& b) {
    static_assert(K >= 1 && K <= 8, "multiple of p");
    Fl<C> r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < C::N - 1; i++) {
        const uint32_t t = a.l[i] + (C::KP[K - 1][i] - b.l[i]) + c;
        r.l[i] = t & C::MASK;
        c = t >> C::B;
    }
    r.l[C::N - 1] = a.l[C::N - 1] + (C::KP[K - 1][C::N - 1] - b.l[C::N - 1]) + c;
    return r;
}

// a + b limb by limb, unnormalised (limbs < 2^(B+1) for normalised a, b)
template <class C>
__device__ __forceinline__ Fl<C> add_nn(const Fl<C>& a, const Fl<C>& b) {
    Fl<C> r;
#pragma unroll
    for (int i = 0; i < C::N; i++) r.l[i] = a.l[i] + b.l[i];
    return r;
}

// a + K p - b limb by limb, unnormalised: b normalised (its limbs never exceed
// KP's, as in sub<K>), result limbs < 2^B + 2^(B+1).  Only as a product operand
// whose column bound allows it (one such operand per product, see the callers).
template <int K, class C>
__device__ __forceinline__ Fl<C> sub_nn(const Fl<C>& a, const Fl<C>& b) {
    static_assert(K >= 1 && K <= 8, "multiple of p");
    Fl<C> r;
#pragma unroll
    for (int i = 0; i < C::N; i++) r.l[i] = a.l[i] + (C::KP[K - 1][i] - b.l[i]);
    return r;
}

// a + 5 p - s, normalised, for s an unnormalised sum of three normalised
// values (limbs < 3 * 2^B, value < 5 p), against the wide-limb KPW5
template <class C>
__device__ __forceinline__ Fl<C> subw5(const Fl<C>& a, const Fl<C>& s) {
    Fl<C> r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < C::N - 1; i++) {
        const uint32_t t = a.l[i] + (C::KPW5[i] - s.l[i]) + c;
        r.l[i] = t & C::MASK;
        c = t >> C::B;
    }
    r.l[C::N - 1] = a.l[C::N - 1] + (C::KPW5[C::N - 1] - s.l[C::N - 1]) + c;
    return r;
}

// carry-propagate limbs < 2^31 (value unchanged)
template <class C>
__device__ __forceinline__ Fl<C> norm(const Fl<C>& a) {
    Fl<C> r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < C::N - 1; i++) {
        const uint32_t t = a.l[i] + c;
        r.l[i] = t & C::MASK;
        c = t >> C::B;
    }
    r.l[C::N - 1] = a.l[C::N - 1] + c;
    return r;
}

// v == 0 mod p for a normalised v < kmax p: v = j p with j = v_0 p^-1 mod 2^B
template <class C>
__device__ __forceinline__ bool is_zero_mod(const Fl<C>& v, uint32_t kmax) {
    const uint32_t j = (v.l[0] * C::PINV) & C::MASK;
    if (j > kmax) return false;
    uint64_t acc = 0;
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < C::N - 1; i++) {
        acc += (uint64_t)j * C::P[i];
        diff |= ((uint32_t)acc & C::MASK) ^ v.l[i];
        acc >>= C::B;
    }
    acc += (uint64_t)j * C::P[C::N - 1];
    diff |= (uint32_t)acc ^ v.l[C::N - 1];
    return diff == 0;
}

template <class C>
__device__ __forceinline__ Fl<C> fl_const(const uint32_t (&v)[C::N]) {
    Fl<C> r;
#pragma unroll
    for (int i = 0; i < C::N; i++) r.l[i] = v[i];
    return r;
}

// gnark-layout words of x * R' mod p (canonical) -> N normalised B-bit limbs
template <class C>
__device__ __forceinline__ Fl<C> unpack_l(const Fe<typename C::Std>& w) {
    constexpr int NW = C::Std::N;
    Fl<C> r;
#pragma unroll
    for (int i = 0; i < C::N; i++) {
        const int bit = C::B * i, wi = bit >> 5, off = bit & 31;
        uint32_t x = w.v[wi] >> off;
        if (off > 32 - C::B && wi + 1 < NW) x |= w.v[wi + 1] << (32 - off);
        r.l[i] = i == C::N - 1 ? x : (x & C::MASK);
    }
    return r;
}
// normalised limbs of a value < 2^(32 NW) -> gnark-layout words
template <class C>
__device__ __forceinline__ Fe<typename C::Std> pack_l(const Fl<C>& a) {
    constexpr int NW = C::Std::N, B = C::B;
    Fe<typename C::Std> r;
#pragma unroll
    for (int wi = 0; wi < NW; wi++) {
        const int bit = 32 * wi, i = bit / B, off = bit % B;
        uint32_t x = a.l[i] >> off;
        if (i + 1 < C::N) x |= a.l[i + 1] << (B - off);
        if (off > 2 * B - 32 && i + 2 < C::N) x |= a.l[i + 2] << (2 * B - off);
        r.v[wi] = x;
    }
    return r;
}
// a (R' form, any normalised value < 8 p) -> canonical gnark Montgomery form
template <class C>
__device__ __forceinline__ Fe<typename C::Std> to_std(const Fl<C>& a) {
    using S = typename C::Std;
    constexpr int NW = S::N;
    Fe<S> t = pack_l(mul(a, fl_const<C>(C::C_OUT)));  // < 8p * p / M + p < 1.05 p
    Fe<S> d;
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) d.v[i] = __builtin_subc(t.v[i], S::P[i], br, &br);
#pragma unroll
    for (int i = 0; i < NW; i++) t.v[i] = br ? t.v[i] : d.v[i];
    return t;
}
__device__ __forceinline__ Fp29 unpack29(const Fp& w) { return unpack_l<Fp29Cfg>(w); }

// gnark Montgomery x R -> x R' mod p (canonical, gnark words): the stored form
// of precomputed base points
template <class C>
GG_HD Fe<typename C::Std> to_rl(const Fe<typename C::Std>& x) {
    Fe<typename C::Std> c;
#pragma unroll
    for (int i = 0; i < C::Std::N; i++) c.v[i] = C::C_IN[i];
    return x * c;
}
GG_HD Fp to_r261(const Fp& x) { return to_rl<Fp29Cfg>(x); }

// ---------------------------------------------------------------------------
// XYZZ bucket accumulator over a reduced-radix form (BN254 G1: 9 x 29, and
// BLS12-381 G1: 14 x 28 bits).  Coordinates stay below 7 p between additions
// (bounds in the comments for BN254's M = 169.28 p; BLS12-381's M = 2520 p
// only makes every product term smaller); infinity is ZZ = 0 (all limbs).
template <class C>
struct XyzzL {
    Fl<C> x, y, zz, zzz;
};
using Xyzz29 = XyzzL<Fp29Cfg>;

template <class C>
__device__ __forceinline__ bool is_inf_l(const XyzzL<C>& p) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < C::N; i++) o |= p.zz.l[i];
    return o == 0;
}
template <class C>
__device__ __forceinline__ XyzzL<C> inf_l() {
    XyzzL<C> r;
#pragma unroll
    for (int i = 0; i < C::N; i++) r.x.l[i] = r.y.l[i] = r.zz.l[i] = r.zzz.l[i] = 0;
    return r;
}
__device__ __forceinline__ Xyzz29 inf29() { return inf_l<Fp29Cfg>(); }

// mdbl-2008-s-1 of an affine point (x < p, y < 2p); result coordinates < 6 p
template <class C>
__device__ __forceinline__ XyzzL<C> xyzzl_dbl_affine(const Fl<C>& x, const Fl<C>& y) {
    const Fl<C> U = add(y, y);                    // < 4p
    const Fl<C> V = mul(U, U);                    // < 1.1p
    const Fl<C> W = mul(U, V);                    // < 1.03p
    const Fl<C> S = mul(x, V);                    // < 1.01p
    const Fl<C> xx = mul(x, x);                   // < 1.01p
    const Fl<C> M = add(xx, add(xx, xx));         // < 3.03p
    const Fl<C> X3 = sub<4>(mul(M, M), add(S, S));  // 2S < 3p: < 5.07p
    const Fl<C> D = sub<7>(S, X3);                // X3 < 6p: < 8.01p
    const Fl<C> Y3 = sub<3>(mul(M, D), mul(W, y));  // W y < 2p: < 4.15p
    return XyzzL<C>{X3, Y3, V, W};
}

// acc += (x, y): madd-2008-s (the same formula, hence the same projective
// representative, as xyzz_madd_inplace); x < p normalised, y < 2p with limbs
// < 2^(B+1) (a negated point arrives unnormalised, sub_nn), acc coordinates < 7 p
// and normalised.
template <class C>
__device__ __forceinline__ void xyzzl_madd(XyzzL<C>& p, const Fl<C>& x, const Fl<C>& y) {
    if (is_inf_l(p)) {
        p = XyzzL<C>{x, norm(y), fl_const<C>(C::ONE), fl_const<C>(C::ONE)};
        return;
    }
    const Fl<C> P = mul_sub<8>(x, p.zz, p.x);    // x ZZ < 1.05p, X < 7p: < 9.05p
    const Fl<C> R = mul_sub<8>(y, p.zzz, p.y);   // y ZZZ < 1.09p: < 9.09p
    if (is_zero_mod(P, 9)) {
        p = is_zero_mod(R, 9) ? xyzzl_dbl_affine(x, y) : inf_l<C>();
        return;
    }
    const Fl<C> PP = sqr(P);                     // < 1.49p
    p.zz = mul(p.zz, PP);                        // < 1.07p
    const Fl<C> PPP = mul(P, PP);                // < 1.08p
    p.zzz = mul(p.zzz, PPP);                     // < 1.05p
    const Fl<C> Q = mul(p.x, PP);                // < 1.07p
    // X3 = R^2 - (PPP + 2Q), the unnormalised sum folded into R^2's output
    // columns (PPP + 2Q < 3.22p; limbs < 3 * 2^B): < 1.5p + 5p = 6.5p, normalised
    const Fl<C> X3 = sqr_subw5(R, add_nn(PPP, add_nn(Q, Q)));
    // Y3 = R (Q - X3) - Y PPP in one reduction: R (Q - X3) + Y (3p - PPP)
    // (Q - X3 < 9.06p, 3p - PPP < 3p, Y < 7p): < (82.4 + 21) p / 169.28 + p < 1.62p.
    // Q + 8p - X3 and 3p - PPP stay unnormalised (limbs < 1.5 * 2^(B+1) and
    // < 2^(B+1)): per column 9 products < 2^62.8 + 9 < 2^62.2 + the reduction
    // < 2^61.2 = 1.45e19 < 2^64 (BLS12-381, 14 x 28 bits: < 2^62.8)
    p.y = mul2(R, sub_nn<8>(Q, X3), p.y, sub_nn<3>(Fl<C>{}, PPP));
    p.x = X3;
}
__device__ __forceinline__ void xyzz29_madd(Xyzz29& p, const Fp29& x, const Fp29& y) { xyzzl_madd(p, x, y); }

template <class C>
__device__ __forceinline__ Xyzz<Fe<typename C::Std>> to_std(const XyzzL<C>& p) {
    return Xyzz<Fe<typename C::Std>>{to_std(p.x), to_std(p.y), to_std(p.zz), to_std(p.zzz)};
}

// gnark form (x R mod p, canonical) -> x R' mod p (< 1.01 p, normalised): one
// product by C_LOAD = R'^2 / R mod p.  Zero stays exactly zero (infinity's ZZ).
template <class C>
__device__ __forceinline__ Fl<C> from_std(const Fe<typename C::Std>& v) {
    return mul(unpack_l<C>(v), fl_const<C>(C::C_LOAD));
}
template <class C>
__device__ __forceinline__ XyzzL<C> from_std(const Xyzz<Fe<typename C::Std>>& p) {
    return XyzzL<C>{from_std<C>(p.x), from_std<C>(p.y), from_std<C>(p.zz), from_std<C>(p.zzz)};
}

// dbl-2008-s-1 (a = 0) of an XYZZ point, coordinates < 7 p normalised in and
// out (bounds for BN254's M = 169.28 p; BLS12-381's M = 2520 p only helps)
template <class C>
__device__ __forceinline__ XyzzL<C> xyzzl_dbl(const XyzzL<C>& p) {
    const Fl<C> U = add(p.y, p.y);                     // < 14p
    const Fl<C> V = sqr(U);                            // < 196/169.28 p + p < 2.16p
    const Fl<C> W = mul(U, V);                         // < 1.18p
    const Fl<C> S = mul(p.x, V);                       // < 1.09p
    const Fl<C> xx = sqr(p.x);                         // < 1.29p
    const Fl<C> M = add(xx, add(xx, xx));              // < 3.87p
    const Fl<C> X3 = sub<4>(sqr(M), add(S, S));        // sqr < 1.09p, 2S < 2.18p: < 5.09p
    const Fl<C> D = sub<7>(S, X3);                     // < 8.09p
    const Fl<C> Y3 = sub<3>(mul(M, D), mul(W, p.y));   // M D < 1.19p, W y < 1.05p: < 4.19p
    return XyzzL<C>{X3, Y3, mul(V, p.zz), mul(W, p.zzz)};
}

// p + q, add-2008-s (XYZZ); coordinates < 7 p normalised in, out X3 < 6.11p,
// Y3 < 1.25p, ZZ3, ZZZ3 < 1.01p.  Used where bucket sums meet (level 2 and the
// weighted bucket reduction), not in the mixed-add hot loop.
template <class C>
__device__ __forceinline__ XyzzL<C> xyzzl_add(const XyzzL<C>& p, const XyzzL<C>& q) {
    if (is_inf_l(q)) return p;
    if (is_inf_l(p)) return q;
    const Fl<C> U1 = mul(p.x, q.zz), U2 = mul(q.x, p.zz);      // < 49/169.28 p + p < 1.29p
    const Fl<C> S1 = mul(p.y, q.zzz), S2 = mul(q.y, p.zzz);    // < 1.29p
    const Fl<C> P = sub<3>(U2, U1), R = sub<3>(S2, S1);        // < 4.29p
    if (is_zero_mod(P, 5)) return is_zero_mod(R, 5) ? xyzzl_dbl(p) : inf_l<C>();
    const Fl<C> PP = sqr(P);                                   // < 18.4/169.28 p + p < 1.11p
    const Fl<C> PPP = mul(P, PP);                              // < 1.03p
    const Fl<C> Q = mul(U1, PP);                               // < 1.01p
    const Fl<C> X3 = sub<5>(sqr(R), add(PPP, add(Q, Q)));      // PPP + 2Q < 3.05p: < 6.11p
    // Y3 = R (Q - X3) - S1 PPP as R (Q + 8p - X3) + S1 (3p - PPP), one reduction
    // (the operands' column bound as in xyzzl_madd: R < 4.29p < 9.09p, S1 < 7p)
    const Fl<C> Y3 = mul2(R, sub_nn<8>(Q, X3), S1, sub_nn<3>(Fl<C>{}, PPP));  // < 1.25p
    return XyzzL<C>{X3, Y3, mul(mul(p.zz, q.zz), PP), mul(mul(p.zzz, q.zzz), PPP)};
}

// ---------------------------------------------------------------------------
// BN254 G2 accumulator over Fp2 = Fp[u]/(u^2 + 1) in the radix-2^29 form.
// Products as sums of limb products with one reduction per component:
//   (a b)_0 = a0 b0 + a1 (k p - b1),  (a b)_1 = a0 b1 + a1 b0.
// Coordinates between additions: X < 2p (reduce_small), Y < 1.3p,
// ZZ, ZZZ < 1.04p (each component; bounds at the call sites, M = 169.28 p).
struct Fp2_29 {
    Fp29 c0, c1;
};
struct Xyzz2_29 {
    Fp2_29 x, y, zz, zzz;
};

__device__ __forceinline__ Xyzz2_29 inf2_29() {
    Xyzz2_29 r;
#pragma unroll
    for (int i = 0; i < 9; i++)
        r.x.c0.l[i] = r.x.c1.l[i] = r.y.c0.l[i] = r.y.c1.l[i] = r.zz.c0.l[i] = r.zz.c1.l[i] = r.zzz.c0.l[i] =
            r.zzz.c1.l[i] = 0;
    return r;
}
__device__ __forceinline__ bool is_inf2_29(const Xyzz2_29& p) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) o |= p.zz.c0.l[i] | p.zz.c1.l[i];
    return o == 0;
}
// a b for b1 < (K - 1) p (a, b normalised).  Kp - b1 stays unnormalised
// (limbs < 2^30): a column holds 9 products < 2^59, 9 < 2^58 and 9 reduction
// products < 2^58: < 2^63.2
template <int K>
__device__ __forceinline__ Fp2_29 mul_fp2(const Fp2_29& a, const Fp2_29& b) {
    const Fp29 nb1 = sub_nn<K>(Fp29{}, b.c1);
    return Fp2_29{mul2(a.c0, b.c0, a.c1, nb1), mul2(a.c0, b.c1, a.c1, b.c0)};
}
// a^2 = ((a0 + a1)(a0 - a1), 2 a0 a1) for a1 < (K - 1) p (a normalised); the
// sums stay unnormalised (limbs < 2^30) against a normalised factor
template <int K>
__device__ __forceinline__ Fp2_29 sqr_fp2(const Fp2_29& a) {
    return Fp2_29{mul(add_nn(a.c0, a.c1), sub<K>(a.c0, a.c1)), mul(a.c0, add_nn(a.c1, a.c1))};
}
__device__ __forceinline__ Fp2 to_std2(const Fp2_29& a) { return Fp2{to_std(a.c0), to_std(a.c1)}; }

// mdbl-2008-s-1 of an affine point over Fp2 (x < p, y < 2p per component):
// X3 < 2p, Y3 < 1.3p, ZZ = V < 1.5p, ZZZ = W < 1.2p
__device__ __forceinline__ Xyzz2_29 xyzz2_29_dbl_affine(const Fp2_29& x, const Fp2_29& y) {
    const Fp2_29 U{add(y.c0, y.c0), add(y.c1, y.c1)};  // < 4p
    const Fp2_29 V = sqr_fp2<6>(U);                      // (1.47p, 1.19p)
    const Fp2_29 W = mul_fp2<3>(U, V);                   // (1.11p, 1.06p)
    const Fp2_29 S = mul_fp2<3>(x, V);                   // < 1.03p
    const Fp2_29 xx = sqr_fp2<3>(x);                     // < 1.05p
    const Fp2_29 M{add(xx.c0, add(xx.c0, xx.c0)), add(xx.c1, add(xx.c1, xx.c1))};  // < 3.15p
    const Fp2_29 MM = sqr_fp2<5>(M);                     // (1.30p, 1.12p)
    const Fp2_29 X3{reduce_small(sub<4>(MM.c0, add(S.c0, S.c0))), reduce_small(sub<4>(MM.c1, add(S.c1, S.c1)))};
    const Fp2_29 D{sub<3>(S.c0, X3.c0), sub<3>(S.c1, X3.c1)};  // < 4.03p
    // Y3 = M D - W y: c0 = M0 D0 + M1 (6p - D1) + y0 (3p - W0) + y1 W1,
    //                 c1 = M0 D1 + M1 D0 + y0 (3p - W1) + y1 (3p - W0)   (< 1.25p)
    const Fp29 nD1 = sub<6>(Fp29{}, D.c1), nW0 = sub<3>(Fp29{}, W.c0), nW1 = sub<3>(Fp29{}, W.c1);
    const Fp2_29 Y3{mul4(M.c0, D.c0, M.c1, nD1, y.c0, nW0, y.c1, W.c1),
                    mul4(M.c0, D.c1, M.c1, D.c0, y.c0, nW1, y.c1, nW0)};
    return Xyzz2_29{X3, Y3, V, W};
}

// acc += (x, y), madd-2008-s over Fp2 (the formula of xyzz_madd_inplace, so
// the same projective representative); x < p, y < 2p per component
__device__ __forceinline__ void xyzz2_29_madd(Xyzz2_29& p, const Fp2_29& x, const Fp2_29& y) {
    if (is_inf2_29(p)) {
        const Fp29 one = fl_const<Fp29Cfg>(Fp29Cfg::ONE);
        p = Xyzz2_29{x, y, Fp2_29{one, Fp29{}}, Fp2_29{one, Fp29{}}};
        return;
    }
    // P = x ZZ - X, R = y ZZZ - Y (ZZ1, ZZZ1 < 2p; X < 2p; Y < 2p): < 4.05p
    // (x and y die here on the common path: fewer live registers)
    // (3p - ZZ1 / ZZZ1 unnormalised, limbs < 2^30: 9 products < 2^59 per column
    // next to 9 < 2^58, the reduction and the folded subtraction: < 2^63.2)
    auto r_of = [&]() {
        const Fp29 nzzz1 = sub_nn<3>(Fp29{}, p.zzz.c1);
        return Fp2_29{mul2_sub<3>(y.c0, p.zzz.c0, y.c1, nzzz1, p.y.c0),
                      mul2_sub<3>(y.c0, p.zzz.c1, y.c1, p.zzz.c0, p.y.c1)};
    };
    const Fp29 nzz1 = sub_nn<3>(Fp29{}, p.zz.c1);
    const Fp2_29 P{mul2_sub<3>(x.c0, p.zz.c0, x.c1, nzz1, p.x.c0), mul2_sub<3>(x.c0, p.zz.c1, x.c1, p.zz.c0, p.x.c1)};
    if (is_zero_mod(P.c0, 5) && is_zero_mod(P.c1, 5)) {
        const Fp2_29 R0 = r_of();
        p = (is_zero_mod(R0.c0, 5) && is_zero_mod(R0.c1, 5)) ? xyzz2_29_dbl_affine(x, y) : inf2_29();
        return;
    }
    const Fp2_29 R = r_of();
    const Fp2_29 PP = sqr_fp2<6>(P);            // (1.48p, 1.19p)
    p.zz = mul_fp2<3>(p.zz, PP);                // < 1.03p
    const Fp2_29 PPP = mul_fp2<3>(P, PP);       // (1.11p, 1.06p)
    p.zzz = mul_fp2<3>(p.zzz, PPP);             // < 1.03p
    const Fp2_29 Q = mul_fp2<3>(p.x, PP);       // (1.05p, 1.03p)
    const Fp2_29 RR = sqr_fp2<6>(R);            // (1.48p, 1.19p)
    // X3 = RR - (PPP + 2Q): < 1.48p + 5p (the sum unnormalised, subtracted
    // against the wide-limb 5p), then reduced below 2p
    const Fp2_29 X3{reduce_small(subw5(RR.c0, add_nn(PPP.c0, add_nn(Q.c0, Q.c0)))),
                    reduce_small(subw5(RR.c1, add_nn(PPP.c1, add_nn(Q.c1, Q.c1))))};
    // Y3 = R (Q - X3) - Y PPP, one reduction per component:
    //   c0 = R0 U0 + R1 (6p - U1) + Y0 (3p - PPP0) + Y1 PPP1
    //   c1 = R0 U1 + R1 U0 + Y0 (3p - PPP1) + Y1 (3p - PPP0)      (< 1.3p)
    const Fp2_29 U{sub<3>(Q.c0, X3.c0), sub<3>(Q.c1, X3.c1)};  // < 4.05p
    const Fp29 nU1 = sub<6>(Fp29{}, U.c1), nP0 = sub<3>(Fp29{}, PPP.c0), nP1 = sub<3>(Fp29{}, PPP.c1);
    p.y = Fp2_29{mul4(R.c0, U.c0, R.c1, nU1, p.y.c0, nP0, p.y.c1, PPP.c1),
                 mul4(R.c0, U.c1, R.c1, U.c0, p.y.c0, nP1, p.y.c1, nP0)};
    p.x = X3;
}

__device__ __forceinline__ Xyzz<Fp2> to_std(const Xyzz2_29& p) {
    return Xyzz<Fp2>{to_std2(p.x), to_std2(p.y), to_std2(p.zz), to_std2(p.zzz)};
}

// Where bucket sums meet (level 2 and the weighted bucket reduction of the G2
// groups): dbl-2008-s-1 and add-2008-s over Fp2, coordinates < 2p per
// component and normalised in and out (the accumulator's partials satisfy it:
// X < 2p, Y < 1.3p, ZZ, ZZZ < 1.5p; M = 169.28 p).
__device__ __forceinline__ Xyzz2_29 xyzz2_29_dbl(const Xyzz2_29& p) {
    const Fp2_29 U{add(p.y.c0, p.y.c0), add(p.y.c1, p.y.c1)};  // < 4p
    const Fp2_29 V = sqr_fp2<5>(U);                          // (8p 9p / M + p, 4p 8p / M + p) < (1.43p, 1.19p)
    const Fp2_29 W = mul_fp2<3>(U, V);                       // (4p 1.43p + 4p 3p) / M + p < 1.11p
    const Fp2_29 S = mul_fp2<3>(p.x, V);                     // < 1.06p
    const Fp2_29 xx = sqr_fp2<3>(p.x);                       // (4p 5p, 2p 4p) / M + p < 1.12p
    const Fp2_29 M{add(xx.c0, add(xx.c0, xx.c0)), add(xx.c1, add(xx.c1, xx.c1))};  // < 3.36p
    const Fp2_29 MM = sqr_fp2<5>(M);                         // (6.72p 8.36p / M + p) < 1.34p
    const Fp2_29 X3{reduce_small(sub<4>(MM.c0, add(S.c0, S.c0))), reduce_small(sub<4>(MM.c1, add(S.c1, S.c1)))};
    const Fp2_29 D{sub<3>(S.c0, X3.c0), sub<3>(S.c1, X3.c1)};  // < 4.06p
    // Y3 = M D - W Y (components as in xyzz2_29_dbl_affine; Y < 2p):
    // < (3.36 4.06 + 3.36 6 + 2 3 + 2 1.11) p^2 / M + p < 1.25p; 36 products
    // of normalised limbs per column + the reduction < 2^63.3
    const Fp29 nD1 = sub<6>(Fp29{}, D.c1), nW0 = sub<3>(Fp29{}, W.c0), nW1 = sub<3>(Fp29{}, W.c1);
    const Fp2_29 Y3{mul4(M.c0, D.c0, M.c1, nD1, p.y.c0, nW0, p.y.c1, W.c1),
                    mul4(M.c0, D.c1, M.c1, D.c0, p.y.c0, nW1, p.y.c1, nW0)};
    return Xyzz2_29{X3, Y3, mul_fp2<3>(V, p.zz), mul_fp2<3>(W, p.zzz)};  // < 1.05p
}

// p + q (add-2008-s): out X3 < 2p, Y3 < 1.28p, ZZ3, ZZZ3 < 1.06p
__device__ __forceinline__ Xyzz2_29 xyzz2_29_add(const Xyzz2_29& p, const Xyzz2_29& q) {
    if (is_inf2_29(q)) return p;
    if (is_inf2_29(p)) return q;
    const Fp2_29 U1 = mul_fp2<3>(p.x, q.zz), U2 = mul_fp2<3>(q.x, p.zz);     // (2p 2p + 2p 3p) / M + p < 1.06p
    const Fp2_29 S1 = mul_fp2<3>(p.y, q.zzz), S2 = mul_fp2<3>(q.y, p.zzz);  // < 1.06p
    const Fp2_29 P{sub<3>(U2.c0, U1.c0), sub<3>(U2.c1, U1.c1)};             // < 4.06p
    const Fp2_29 R{sub<3>(S2.c0, S1.c0), sub<3>(S2.c1, S1.c1)};             // < 4.06p
    if (is_zero_mod(P.c0, 5) && is_zero_mod(P.c1, 5))
        return (is_zero_mod(R.c0, 5) && is_zero_mod(R.c1, 5)) ? xyzz2_29_dbl(p) : inf2_29();
    const Fp2_29 PP = sqr_fp2<6>(P);            // (1.48p, 1.19p)
    const Fp2_29 PPP = mul_fp2<3>(P, PP);       // < 1.11p
    const Fp2_29 Q = mul_fp2<3>(U1, PP);        // < 1.04p
    const Fp2_29 RR = sqr_fp2<6>(R);            // (1.48p, 1.19p)
    const Fp2_29 X3{reduce_small(subw5(RR.c0, add_nn(PPP.c0, add_nn(Q.c0, Q.c0)))),
                    reduce_small(subw5(RR.c1, add_nn(PPP.c1, add_nn(Q.c1, Q.c1))))};  // PPP + 2Q < 3.2p
    // Y3 = R (Q - X3) - S1 PPP as in xyzz2_29_madd (S1 in Y's place):
    // < (4.06 4.03 + 4.06 6 + 1.06 3 + 1.06 1.11) p^2 / M + p < 1.28p
    const Fp2_29 U{sub<3>(Q.c0, X3.c0), sub<3>(Q.c1, X3.c1)};  // < 4.04p
    const Fp29 nU1 = sub<6>(Fp29{}, U.c1), nP0 = sub<3>(Fp29{}, PPP.c0), nP1 = sub<3>(Fp29{}, PPP.c1);
    const Fp2_29 Y3{mul4(R.c0, U.c0, R.c1, nU1, S1.c0, nP0, S1.c1, PPP.c1),
                    mul4(R.c0, U.c1, R.c1, U.c0, S1.c0, nP1, S1.c1, nP0)};
    return Xyzz2_29{X3, Y3, mul_fp2<3>(mul_fp2<3>(p.zz, q.zz), PP), mul_fp2<3>(mul_fp2<3>(p.zzz, q.zzz), PPP)};
}

// -p: Y -> 3p - Y reduced below 2p (Y < 2p)
__device__ __forceinline__ Xyzz2_29 xyzz2_29_neg(const Xyzz2_29& p) {
    if (is_inf2_29(p)) return p;
    Xyzz2_29 r = p;
    r.y = Fp2_29{reduce_small(sub<3>(Fp29{}, p.y.c0)), reduce_small(sub<3>(Fp29{}, p.y.c1))};
    return r;
}

}  // namespace gg
