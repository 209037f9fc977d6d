// Radix-2 NTT over BN254 Fr for gfx950 with gnark-crypto's FFT conventions
// (backend/groth16/bn254/prove.go:369-393 call sites; gnark-crypto fft [ext]):
//   DIF: natural order in -> bit-reversed out;  DIT: bit-reversed in -> natural out.
//
// Layout / schedule (DESIGN.md "NTT"):
//   * the 2^L vector lives in HBM as gnark fr.Element (32 B, Montgomery);
//   * a transform is split into passes; each pass owns k consecutive bit
//     positions (butterfly spans) of a 2048-element tile (2^k rows x 2^tl
//     adjacent columns; the first DIT / last DIF pass is contiguous, k = 11);
//   * inside a pass the k stages run as radix-8 register rounds (3 stages per
//     LDS exchange): the first round reads HBM, the last writes HBM, middle
//     rounds go through a padded limb-major LDS tile (conflict-free);
//   * twiddles: per-stage contiguous tables tw[2^b - 1 + i] = w^(i 2^(L-1-b))
//     (n-1 entries, 512 MiB at 2^24), so every stage streams its own table;
//   * coset / 1/n / den scalings are fused into the first or last pass as
//     multiplication by hi[e >> S] * lo[e & (2^S-1)], e = i or bitrev(i),
//     from two 2^(L/2)-entry tables (no n-sized coset tables);
//   * computeH fuses PolyOps (a*b - c) into c's last coset-NTT pass and folds
//     den = 1/(g^n - 1) into the final inverse-transform scaling.
#include "common.h"
#include "field.cuh"
#include "prof.h"
#include <vector>
#include <mutex>
#include <memory>
#include <algorithm>
#include <cstring>
#include <type_traits>

namespace gg {

enum ScaleKind {
    SK_G_NAT = 0,       // g^i
    SK_G_BR = 1,        // g^bitrev(i)
    SK_GINV_NAT_N = 2,  // g^-i / n
    SK_GINV_BR_N = 3,   // g^-bitrev(i) / n
    SK_NINV = 4,        // 1/n
    SK_H_FWD = 5,       // g^bitrev(i) / n          (computeH: iFFT -> coset FFT)
    SK_H_INV = 6,       // den * g^-bitrev(i) / n   (computeH: final coset iFFT)
    SK_DEN_N = 7,       // den / n                  (computeH: iFFT of C)
    SK_COUNT = 8
};

template <class F>
struct ScaleSpec {
    const F* hi;  // 2^(L-S) entries (constant folded in)
    const F* lo;  // 2^S entries
    int shift;     // S
    int bitrev;    // index by bitrev(i) instead of i
};

template <class F>
struct PassParams {
    const F* in;
    F* out;
    const F* tw;
    int log_n;
    int b_lo;
    int k;
    int tl;
    int dit;
    int has_pre;
    ScaleSpec<F> pre;
    int has_post;
    ScaleSpec<F> post;
    int epi_mul_sub;  // out = ea*eb - x
    int epi_mul;      // out = ea*x
    int epi_sub;      // out = x - ea
    const F* ea;
    const F* eb;
    int canon_out;    // last pass of the transform: write canonical values (lazy fields)
};

// Lazily reduced butterflies for BN254 fr (4r < 2^256): values stay below 2r
// inside a transform (also between passes, in HBM), the twiddle product skips
// its final subtraction (mul_nored: a < 4r, w < r -> < 2r), the DIF difference
// a - b + 2r is multiplied unreduced, and the last pass writes canonical values.
// BLS12-381 fr (2r < 2^256 < 4r) keeps the canonical butterflies.
template <class F>
struct NttLazy {
    static constexpr bool on = false;
};
template <>
struct NttLazy<Fr> {
    static constexpr bool on = true;
};
template <class C>
GG_HD constexpr uint32_t twop_limb(int i) {
    uint64_t c = 0;
    uint32_t v = 0;
    for (int j = 0; j <= i; j++) {
        const uint64_t t = (uint64_t)C::P[j] * 2 + c;
        v = (uint32_t)t;
        c = t >> 32;
    }
    return v;
}
// x < 4p -> representative < 2p
template <class C>
__device__ __forceinline__ Fe<C> red2p(const Fe<C>& x) {
    Fe<C> s, r;
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = __builtin_subc(x.v[i], twop_limb<C>(i), br, &br);
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = br ? x.v[i] : s.v[i];
    return r;
}
// a, b < 2p: a + b reduced below 2p
template <class C>
__device__ __forceinline__ Fe<C> add2p(const Fe<C>& a, const Fe<C>& b) {
    Fe<C> r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
    return red2p(r);
}
// a, b < 2p: a - b + 2p in (0, 4p), unreduced
template <class C>
__device__ __forceinline__ Fe<C> subnr2p(const Fe<C>& a, const Fe<C>& b) {
    Fe<C> r;
    uint32_t br = 0, c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = __builtin_addc(r.v[i], twop_limb<C>(i), c, &c);
    return r;
}
// a, b < 2p: (a - b) mod 2p, below 2p
template <class C>
__device__ __forceinline__ Fe<C> sub2p(const Fe<C>& a, const Fe<C>& b) {
    Fe<C> r, s;
    uint32_t br = 0, c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = __builtin_addc(r.v[i], twop_limb<C>(i), c, &c);
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = br ? s.v[i] : r.v[i];
    return r;
}
// x < 2p -> canonical
template <class C>
__device__ __forceinline__ Fe<C> canon(const Fe<C>& x) {
    Fe<C> s, r;
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = __builtin_subc(x.v[i], C::P[i], br, &br);
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = br ? x.v[i] : s.v[i];
    return r;
}

__device__ __forceinline__ uint32_t brev_bits(uint32_t i, int L) {
    return L ? (__brev(i) >> (32 - L)) : 0u;
}

template <class F>
__device__ __forceinline__ F load_fr(const F* p) {
    static_assert(sizeof(F) == 32, "8-limb scalar field");
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    F r;
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    return r;
}

template <class F>
__device__ __forceinline__ void store_fr(F* p, const F& r) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(r.v[0], r.v[1], r.v[2], r.v[3]);
    q[1] = make_uint4(r.v[4], r.v[5], r.v[6], r.v[7]);
}

template <class F>
__device__ __forceinline__ F apply_scale(const ScaleSpec<F>& s, uint32_t g, int L, const F& x) {
    uint32_t e = s.bitrev ? brev_bits(g, L) : g;
    F f = load_fr(s.hi + (e >> s.shift));
    if (s.lo) f = f * load_fr(s.lo + (e & ((1u << s.shift) - 1)));
    return x * f;
}

// ---- radix-8 register-round pass ------------------------------------------
__device__ __forceinline__ int lidx(int e) { return e + (e >> 5); }  // padded LDS index

template <class F, int NB, bool DIT>
__device__ __forceinline__ void ntt_round(const PassParams<F>& P, uint32_t* lds, int TP, int T, int qlo,
                                          bool first, bool last, uint32_t base_hi, uint32_t lo0) {
    constexpr int R = 1 << NB;
    const int tl = P.tl;
    const uint32_t tl_mask = (1u << tl) - 1;
    const int pos = qlo + tl;
    const uint32_t lowmask = (1u << pos) - 1;
    const int groups = T >> NB;
    for (int gi = threadIdx.x; gi < groups; gi += blockDim.x) {
        uint32_t e[R], g[R];
        F x[R];
        const uint32_t low = (uint32_t)gi & lowmask, high = ((uint32_t)gi >> pos) << (pos + NB);
#pragma unroll
        for (int m = 0; m < R; m++) {
            e[m] = high | ((uint32_t)m << pos) | low;
            g[m] = base_hi | ((e[m] >> tl) << P.b_lo) | (lo0 + (e[m] & tl_mask));
        }
        if (first) {
#pragma unroll
            for (int m = 0; m < R; m++) {
                x[m] = load_fr(P.in + g[m]);
                if (P.has_pre) x[m] = apply_scale(P.pre, g[m], P.log_n, x[m]);
            }
        } else {
#pragma unroll
            for (int m = 0; m < R; m++) {
#pragma unroll
                for (int l = 0; l < 8; l++) x[m].v[l] = lds[l * TP + lidx((int)e[m])];
            }
        }
#pragma unroll
        for (int s2 = 0; s2 < NB; s2++) {
            const int r = DIT ? s2 : (NB - 1 - s2);
            const int b = P.b_lo + qlo + r;
            const uint32_t bmask = (1u << b) - 1;
            const F* twb = P.tw + bmask;  // stage-b table starts at 2^b - 1
#pragma unroll
            for (int m = 0; m < R; m++) {
                if (m & (1 << r)) continue;
                const int m2 = m | (1 << r);
                const uint32_t i = g[m] & bmask;
                if constexpr (NttLazy<F>::on) {
                    if (DIT) {
                        F t = i ? mul_nored(x[m2], load_fr(twb + i)) : x[m2];
                        x[m2] = sub2p(x[m], t);
                        x[m] = add2p(x[m], t);
                    } else {
                        F d = subnr2p(x[m], x[m2]);
                        x[m] = add2p(x[m], x[m2]);
                        x[m2] = i ? mul_nored(d, load_fr(twb + i)) : red2p(d);
                    }
                    continue;
                }
                if (DIT) {
                    F t = i ? x[m2] * load_fr(twb + i) : x[m2];
                    x[m2] = x[m] - t;
                    x[m] = x[m] + t;
                } else {
                    F d = x[m] - x[m2];
                    x[m] = x[m] + x[m2];
                    x[m2] = i ? d * load_fr(twb + i) : d;
                }
            }
        }
        if (last) {
#pragma unroll
            for (int m = 0; m < R; m++) {
                F y = x[m];
                // lazy fields: the post-scale's full product also brings y < 2r below r
                if (NttLazy<F>::on && P.canon_out && !P.has_post) y = canon(y);
                if (P.has_post) y = apply_scale(P.post, g[m], P.log_n, y);
                if (P.epi_mul_sub) y = load_fr(P.ea + g[m]) * load_fr(P.eb + g[m]) - y;
                if (P.epi_mul) y = load_fr(P.ea + g[m]) * y;
                if (P.epi_sub) y = y - load_fr(P.ea + g[m]);
                store_fr(P.out + g[m], y);
            }
        } else {
#pragma unroll
            for (int m = 0; m < R; m++) {
#pragma unroll
                for (int l = 0; l < 8; l++) lds[l * TP + lidx((int)e[m])] = x[m].v[l];
            }
        }
    }
}

// MAXNB = stages per register round: 3 (radix-8, 256 threads per 2048-element
// tile, ~190 VGPRs: 2 waves per SIMD) or 2 (radix-4, 512 threads, <= 128 VGPRs:
// 4 waves per SIMD -- more LDS exchanges, better latency hiding)
template <int MAXNB>
constexpr int kNttThreads = MAXNB == 3 ? 256 : (MAXNB == 2 ? 512 : 1024);
template <int MAXNB>
constexpr int kNttWaves = MAXNB == 3 ? 1 : (MAXNB == 2 ? 4 : 8);
template <class F, bool DIT, int MAXNB>
__global__ void __launch_bounds__(kNttThreads<MAXNB>, kNttWaves<MAXNB>) k_ntt_pass(PassParams<F> P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int k = P.k, tl = P.tl;
    const int T = 1 << (k + tl);
    const int TP = T + (T >> 5);
    const int nlo_log = P.b_lo - tl;
    const uint32_t tile = blockIdx.x;
    const uint32_t lob = tile & ((1u << nlo_log) - 1);
    const uint32_t hi = tile >> nlo_log;
    const uint32_t base_hi = hi << (P.b_lo + k);
    const uint32_t lo0 = lob << tl;
    if (k == 0) {  // n = 1: scaling only
        for (int e = threadIdx.x; e < T; e += blockDim.x) {
            uint32_t g = base_hi | (lo0 + (uint32_t)e);
            F x = load_fr(P.in + g);
            if (P.has_pre) x = apply_scale(P.pre, g, P.log_n, x);
            if (P.has_post) x = apply_scale(P.post, g, P.log_n, x);
            if (P.epi_mul_sub) x = load_fr(P.ea + g) * load_fr(P.eb + g) - x;
            if (P.epi_mul) x = load_fr(P.ea + g) * x;
            if (P.epi_sub) x = x - load_fr(P.ea + g);
            store_fr(P.out + g, x);
        }
        return;
    }
    // rounds of <= 3 stages in processing order (DIF: high bits first)
    int done = 0;
    bool first = true;
    while (done < k) {
        const int nb = min(MAXNB, k - done);
        const int qlo = DIT ? done : (k - done - nb);
        const bool last = (done + nb == k);
        if (!first) __syncthreads();
        if constexpr (MAXNB >= 3) {
            if (nb == 3) {
                ntt_round<F, 3, DIT>(P, lds, TP, T, qlo, first, last, base_hi, lo0);
                first = false;
                done += nb;
                continue;
            }
        }
        if constexpr (MAXNB >= 2) {
            if (nb == 2) {
                ntt_round<F, 2, DIT>(P, lds, TP, T, qlo, first, last, base_hi, lo0);
                first = false;
                done += nb;
                continue;
            }
        }
        ntt_round<F, 1, DIT>(P, lds, TP, T, qlo, first, last, base_hi, lo0);
        first = false;
        done += nb;
    }
}

// per-stage twiddle table: tw[(2^b - 1) + i] = w^(i << (L-1-b)), i < 2^b
template <class F>
__global__ void k_stage_twiddles(F* out, size_t count, int L, const F* hi, const F* lo, int S) {
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    uint32_t v = (uint32_t)t + 1;
    int b = 31 - __clz((int)v);
    uint32_t i = v - (1u << b);
    uint32_t ex = i << (L - 1 - b);
    F x = load_fr(hi + (ex >> S)) * load_fr(lo + (ex & ((1u << S) - 1)));
    store_fr(out + t, x);
}


// ---------------------------------------------------------------------------
struct Pass {
    int b_lo, k, tl;
};

static std::vector<Pass> plan_passes(int L, bool dit) {
    // every tile holds 2048 elements: the contiguous pass takes k = 11 bits,
    // strided passes k <= 9 bits with 2^(11-k) adjacent columns (>= 128-B runs)
    std::vector<Pass> up;
    if (L <= 11) {
        up.push_back({0, L, 0});
    } else {
        up.push_back({0, 11, 0});
        int rem = L - 11, P = (rem + 8) / 9, b = 11;
        for (int i = 0; i < P; i++) {
            int k = rem / (P - i);
            up.push_back({b, k, 11 - k});
            b += k;
            rem -= k;
        }
    }
    if (dit) return up;  // DIT: low bits first
    std::vector<Pass> v(up.rbegin(), up.rend());  // DIF: high bits first
    return v;
}

}  // namespace gg

using namespace gg;

namespace gg {
// Domain of one scalar field: gnark-crypto fft.Domain (Generator, FrMultiplicativeGen,
// CardinalityInv) plus the device tables.
template <class C>
struct DomainT {
    using F = Fe<C>;
    int log_n = 0;
    size_t n = 1;
    F omega, omega_inv, g, g_inv, n_inv, den;
    DevBuf tw, twinv;
    int S = 0;
    DevBuf scale_hi[SK_COUNT], scale_lo[SK_COUNT];
    ScaleSpec<F> spec[SK_COUNT];
};
}  // namespace gg

// curve: GG_CURVE_BN254 (Groth16 domain) or GG_CURVE_BLS12_381 (PlonK domains)
struct gg_domain {
    int curve = GG_CURVE_BN254;
    int log_n = 0;
    size_t n = 1;
    std::unique_ptr<DomainT<FrCfg>> bn;
    std::unique_ptr<DomainT<FrBlsCfg>> bls;
    DevBuf scratch;  // computeH b/c buffers
    std::mutex mu;
};

namespace gg {

template <class F>
static void build_pow_tables(int L, int S, const F& x, const F& c, std::vector<F>& hi,
                             std::vector<F>& lo) {
    size_t nlo = (size_t)1 << S, nhi = (size_t)1 << (L - S);
    lo.resize(nlo);
    hi.resize(nhi);
    F acc = F::one();
    for (size_t i = 0; i < nlo; i++) { lo[i] = acc; acc = acc * x; }
    F step = acc;  // x^(2^S)
    acc = c;
    for (size_t i = 0; i < nhi; i++) { hi[i] = acc; acc = acc * step; }
}

template <class F>
static void upload(DevBuf& b, const std::vector<F>& v) {
    b.alloc(v.size() * sizeof(F));
    GG_HIP(hipMemcpy(b.p, v.data(), v.size() * sizeof(F), hipMemcpyHostToDevice));
}

// NTT pass flavour (k_ntt_pass MAXNB); GG_NTT_RADIX=4 or 8 overrides the default.
// Radix-4 rounds at 4 waves per SIMD measured faster on MI355X than radix-8 at 2
// (2^24 BN254: DIF 2.63 -> 2.44 ms, computeH 18.5 -> 16.7 ms; BLS12-381 2^22
// 0.72 -> 0.67 ms): the extra LDS exchanges cost less than the latency they hide.
static int ntt_radix() {
    const char* e = getenv("GG_NTT_RADIX");
    const int r = e ? atoi(e) : 4;
    return (r == 2 || r == 8) ? r : 4;
}

static hipStream_t pick_stream(void* s) { return s ? (hipStream_t)s : hipStreamPerThread; }

// epilogue of the last pass: EPI_MUL_SUB out = ea*eb - x, EPI_MUL out = ea*x,
// EPI_SUB out = x - ea (none when ea is null)
enum { EPI_MUL_SUB = 0, EPI_MUL = 1, EPI_SUB = 2 };
// passes: nullptr = the whole transform (plan_passes); else only these (e.g. the
// last stages of a DIT whose first stages ran elsewhere, ntt_tail_inverse_coset)
template <class C>
void run_transform(DomainT<C>* d, const Fe<C>* in, Fe<C>* out, bool dit, bool inverse_tw, int pre_kind,
                   int post_kind, const Fe<C>* ea, const Fe<C>* eb, hipStream_t st, int epi = EPI_MUL_SUB,
                   const std::vector<Pass>* only = nullptr) {
    using F = Fe<C>;
    const int L = d->log_n;
    auto passes = only ? *only : plan_passes(L, dit);
    const F* src = in;
    for (size_t pi = 0; pi < passes.size(); pi++) {
        const Pass& ps = passes[pi];
        PassParams<F> P{};
        P.in = src;
        P.out = out;
        P.tw = (const F*)(inverse_tw ? d->twinv.p : d->tw.p);
        P.log_n = L;
        P.b_lo = ps.b_lo;
        P.k = ps.k;
        P.tl = ps.tl;
        P.dit = dit ? 1 : 0;
        if (pi == 0 && pre_kind >= 0) { P.has_pre = 1; P.pre = d->spec[pre_kind]; }
        bool last = (pi + 1 == passes.size());
        if (last && post_kind >= 0) { P.has_post = 1; P.post = d->spec[post_kind]; }
        if (last && ea) {
            P.epi_mul_sub = epi == EPI_MUL_SUB;
            P.epi_mul = epi == EPI_MUL;
            P.epi_sub = epi == EPI_SUB;
            P.ea = ea;
            P.eb = eb;
        }
        P.canon_out = last ? 1 : 0;
        int T = 1 << (ps.k + ps.tl);
        unsigned tiles = (unsigned)(d->n / (size_t)T);
        size_t lds = (ps.k > 3) ? (size_t)(T + (T >> 5)) * 32 : 0;  // single-round passes skip LDS
        ProfScope prof("ntt_pass", st, (double)d->n);
        static const int radix = ntt_radix();
        if (radix == 4) {
            lds = (ps.k > 2) ? (size_t)(T + (T >> 5)) * 32 : 0;
            if (dit) hipLaunchKernelGGL((k_ntt_pass<F, true, 2>), dim3(tiles), dim3(512), lds, st, P);
            else hipLaunchKernelGGL((k_ntt_pass<F, false, 2>), dim3(tiles), dim3(512), lds, st, P);
        } else if (radix == 2) {
            lds = (ps.k > 1) ? (size_t)(T + (T >> 5)) * 32 : 0;
            if (dit) hipLaunchKernelGGL((k_ntt_pass<F, true, 1>), dim3(tiles), dim3(1024), lds, st, P);
            else hipLaunchKernelGGL((k_ntt_pass<F, false, 1>), dim3(tiles), dim3(1024), lds, st, P);
        } else {
            if (dit) hipLaunchKernelGGL((k_ntt_pass<F, true, 3>), dim3(tiles), dim3(256), lds, st, P);
            else hipLaunchKernelGGL((k_ntt_pass<F, false, 3>), dim3(tiles), dim3(256), lds, st, P);
        }
        GG_HIP(hipGetLastError());
        prof.stop(st);
        src = out;
    }
}

}  // namespace gg

namespace gg {
template <class C>
static DomainT<C>* domain_build(int log_n, const void* omega_mont, const void* coset_gen_mont) {
    using F = Fe<C>;
    std::unique_ptr<DomainT<C>> d(new DomainT<C>());
    d->log_n = log_n;
    d->n = (size_t)1 << log_n;
    memcpy(d->omega.v, omega_mont, 32);
    memcpy(d->g.v, coset_gen_mont, 32);
    // omega must have order exactly n
    F x = d->omega;
    for (int i = 0; i < log_n; i++) {
        if (i == log_n - 1) GG_CHECK(!(x == F::one()), GG_ERR_INVALID_ARG, "omega order < n");
        x = sqr(x);
    }
    GG_CHECK(x == F::one(), GG_ERR_INVALID_ARG, "omega^n != 1");
    GG_CHECK(!d->g.is_zero(), GG_ERR_INVALID_ARG, "coset generator is zero");
    d->omega_inv = inverse(d->omega);
    d->g_inv = inverse(d->g);
    F nn = F::zero();
    nn.v[0] = (uint32_t)d->n;
    nn.v[1] = (uint32_t)((uint64_t)d->n >> 32);
    nn = to_mont(nn);
    d->n_inv = inverse(nn);
    F gn = pow_u64(d->g, d->n);
    F t = gn - F::one();
    GG_CHECK(!t.is_zero(), GG_ERR_INVALID_ARG, "g^n == 1: coset generator in the domain");
    d->den = inverse(t);

    const int L = log_n;
    d->S = (L + 1) / 2;
    const int S = d->S;
    std::vector<F> hi, lo;
    struct KindDef { F x, c; int br; };
    KindDef defs[SK_COUNT] = {
        {d->g, F::one(), 0},
        {d->g, F::one(), 1},
        {d->g_inv, d->n_inv, 0},
        {d->g_inv, d->n_inv, 1},
        {F::one(), d->n_inv, 0},
        {d->g, d->n_inv, 1},
        {d->g_inv, d->den * d->n_inv, 1},
        {F::one(), d->den * d->n_inv, 0},
    };
    for (int kd = 0; kd < SK_COUNT; kd++) {
        build_pow_tables(L, S, defs[kd].x, defs[kd].c, hi, lo);
        upload(d->scale_hi[kd], hi);
        upload(d->scale_lo[kd], lo);
        d->spec[kd] = ScaleSpec<F>{(const F*)d->scale_hi[kd].p, (const F*)d->scale_lo[kd].p, S,
                                   defs[kd].br};
    }
    // per-stage twiddles (n - 1 entries each for w and w^-1), generated on device
    size_t cnt = d->n - 1;
    d->tw.alloc((cnt + 1) * 32);
    d->twinv.alloc((cnt + 1) * 32);
    if (cnt) {
        for (int inv = 0; inv < 2; inv++) {
            DevBuf h1, l1;
            build_pow_tables(L, S, inv ? d->omega_inv : d->omega, F::one(), hi, lo);
            upload(h1, hi);
            upload(l1, lo);
            hipLaunchKernelGGL(k_stage_twiddles<F>, dim3(grid_for(cnt, 256)), dim3(256), 0, 0,
                               (inv ? d->twinv : d->tw).template as<F>(), cnt, L, h1.as<F>(), l1.as<F>(), S);
            GG_HIP(hipGetLastError());
            GG_HIP(hipDeviceSynchronize());
        }
    }
    return d.release();
}

template <class C>
static void ntt_apply(DomainT<C>* d, void* data_dev, int inverse, bool dit, int coset, hipStream_t st) {
    Fe<C>* a = (Fe<C>*)data_dev;
    int pre = -1, post = -1;
    if (!inverse) {
        if (coset) pre = dit ? SK_G_BR : SK_G_NAT;
    } else {
        if (!coset) post = SK_NINV;
        else post = dit ? SK_GINV_NAT_N : SK_GINV_BR_N;
    }
    run_transform(d, a, a, dit, inverse != 0, pre, post, (const Fe<C>*)nullptr, (const Fe<C>*)nullptr, st);
}
}  // namespace gg

extern "C" int gg_domain_create_ex(int curve, int log_n, const void* omega_mont,
                                   const void* coset_gen_mont, gg_domain_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out && omega_mont && coset_gen_mont, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "bad curve");
    // 2-adicity: BN254 fr 28, BLS12-381 fr 32 (table indices are u32 here)
    GG_CHECK(log_n >= 0 && log_n <= (curve == GG_CURVE_BN254 ? 28 : 30), GG_ERR_INVALID_ARG,
             "log_n out of range");
    std::unique_ptr<gg_domain> d(new gg_domain());
    d->curve = curve;
    d->log_n = log_n;
    d->n = (size_t)1 << log_n;
    if (curve == GG_CURVE_BN254) d->bn.reset(domain_build<FrCfg>(log_n, omega_mont, coset_gen_mont));
    else d->bls.reset(domain_build<FrBlsCfg>(log_n, omega_mont, coset_gen_mont));
    *out = d.release();
    GG_CAPI_END
}

extern "C" int gg_domain_create(int log_n, const void* omega_mont, const void* coset_gen_mont,
                                gg_domain_t* out) {
    return gg_domain_create_ex(GG_CURVE_BN254, log_n, omega_mont, coset_gen_mont, out);
}

extern "C" int gg_domain_release(gg_domain_t d) {
    GG_CAPI_BEGIN
    delete d;
    GG_CAPI_END
}

extern "C" int gg_domain_log_n(gg_domain_t d, int* log_n) {
    GG_CAPI_BEGIN
    GG_CHECK(d && log_n, GG_ERR_INVALID_ARG, "null argument");
    *log_n = d->log_n;
    GG_CAPI_END
}

extern "C" int gg_ntt(gg_domain_t d, void* data_dev, int inverse, int decimation, int coset,
                      void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(d && data_dev, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(decimation == GG_DIF || decimation == GG_DIT, GG_ERR_INVALID_ARG, "bad decimation");
    hipStream_t st = pick_stream(hip_stream);
    bool dit = decimation == GG_DIT;
    if (d->curve == GG_CURVE_BN254) ntt_apply(d->bn.get(), data_dev, inverse, dit, coset, st);
    else ntt_apply(d->bls.get(), data_dev, inverse, dit, coset, st);
    GG_CAPI_END
}

namespace gg {
// computeH (prove.go:353-396) on device buffers A (becomes h), B, C, each 2^L fr
// (already padded), for the domain's scalar field
// Six transforms instead of prove.go's seven: the coset iFFT is linear and
// undoes the coset FFT, so coset_iFFT((a b - c) den) = coset_iFFT(a b) den -
// c_coeffs den, where c_coeffs = iFFT(c) -- c's coset FFT is never needed.  The
// field arithmetic is exact, so h is the reference's, bit for bit (h for any
// a, b, c, satisfied or not: only linearity is used).
template <class C>
static void compute_h_t(DomainT<C>* d, Fe<C>* A, Fe<C>* B, Fe<C>* Cv, Fe<C>* H, hipStream_t st) {
    const Fe<C>* nul = nullptr;
    // a, b: iFFT(DIF) with g^br(i)/n folded in, then DIT FFT -> coset evaluations;
    // the last pass of b's emits a*b in place
    run_transform(d, A, A, false, true, -1, SK_H_FWD, nul, nul, st);
    run_transform(d, A, A, true, false, -1, -1, nul, nul, st);
    run_transform(d, B, B, false, true, -1, SK_H_FWD, nul, nul, st);
    run_transform(d, B, B, true, false, -1, -1, (const Fe<C>*)A, nul, st, EPI_MUL);
    // c: plain iFFT (DIF, natural -> bit-reversed coefficients) with den / n
    run_transform(d, Cv, Cv, false, true, -1, SK_DEN_N, nul, nul, st);
    // coset iFFT (DIF) of a*b with den * g^-br(i) / n folded in, minus den c:
    // h bit-reversed.  H may alias A or B (C is read by the last pass).
    GG_CHECK(H != Cv, GG_ERR_INTERNAL, "computeH: h must not alias c");
    run_transform(d, B, H, false, true, -1, SK_H_INV, (const Fe<C>*)Cv, nul, st, EPI_SUB);
}
// any curve's domain (BN254 or BLS12-381 Groth16); fr buffers as opaque 32-B elements
void compute_h_device(gg_domain* dom, Fr* A, Fr* B, Fr* C, Fr* H, hipStream_t st) {
    if (dom->curve == GG_CURVE_BN254) compute_h_t(dom->bn.get(), A, B, C, H, st);
    else compute_h_t(dom->bls.get(), (FrBls*)A, (FrBls*)B, (FrBls*)C, (FrBls*)H, st);
}
}  // namespace gg

extern "C" int gg_groth16_compute_h(gg_domain_t d, const void* a, const void* b, const void* c,
                                    size_t len, int inputs_on_device, void* h_dev,
                                    void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(d && a && b && c && h_dev, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(len <= d->n, GG_ERR_INVALID_ARG, "len > domain cardinality");
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t st = pick_stream(hip_stream);
    size_t nb = d->n * 32;
    d->scratch.reserve(3 * nb);
    char* base = (char*)d->scratch.p;
    Fr* A = (Fr*)base;
    Fr* B = (Fr*)(base + nb);
    Fr* C = (Fr*)(base + 2 * nb);
    hipMemcpyKind kind = inputs_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    const void* src[3] = {a, b, c};
    Fr* dst[3] = {A, B, C};
    for (int i = 0; i < 3; i++) {
        if (len) GG_HIP(hipMemcpyAsync(dst[i], src[i], len * 32, kind, st));
        if (len < d->n) GG_HIP(hipMemsetAsync((char*)dst[i] + len * 32, 0, nb - len * 32, st));
    }
    compute_h_device(d, A, B, C, (Fr*)h_dev, st);
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}

namespace gg {
// helpers for the PlonK kernels (plonk.hip)
size_t domain_size(gg_domain* d, int* curve) {
    if (curve) *curve = d->curve;
    return d->n;
}
void any_ntt_inplace(gg_domain* d, void* data, int inverse, int dit, int coset, hipStream_t st) {
    if (d->curve == GG_CURVE_BN254) ntt_apply(d->bn.get(), data, inverse, dit != 0, coset, st);
    else ntt_apply(d->bls.get(), data, inverse, dit != 0, coset, st);
}
// The distributed big-domain inverse of the PlonK quotient (plonk_prover.hip):
// a DIT with bit-reversed input runs its first L - u stages inside contiguous
// blocks of 2^(L - u) elements -- each block's size-2^(L - u) inverse DFT (root
// w^(2^u), the same stage twiddles), computed by the block's owner without any
// scaling (ntt_inverse_dit_noscale) -- and its last u stages across the blocks,
// with the coset inverse's g^-i / n on the natural-order output
// (ntt_tail_inverse_coset).  Together: FFTInverse(DIT, OnCoset).
void ntt_inverse_dit_noscale(gg_domain* d, void* data, hipStream_t st) {
    if (d->curve == GG_CURVE_BN254)
        run_transform(d->bn.get(), (const Fr*)data, (Fr*)data, true, true, -1, -1, (const Fr*)nullptr,
                      (const Fr*)nullptr, st);
    else
        run_transform(d->bls.get(), (const FrBls*)data, (FrBls*)data, true, true, -1, -1, (const FrBls*)nullptr,
                      (const FrBls*)nullptr, st);
}
void ntt_tail_inverse_coset(gg_domain* d, void* data, int u, hipStream_t st) {
    const int L = d->log_n;
    GG_CHECK(u >= 1 && u <= 4 && L >= 12, GG_ERR_INTERNAL, "tail transform: 1..4 stages of a >= 2^12 domain");
    const std::vector<Pass> tail = {{L - u, u, 11 - u}};
    if (d->curve == GG_CURVE_BN254)
        run_transform(d->bn.get(), (const Fr*)data, (Fr*)data, true, true, -1, SK_GINV_NAT_N, (const Fr*)nullptr,
                      (const Fr*)nullptr, st, EPI_MUL_SUB, &tail);
    else
        run_transform(d->bls.get(), (const FrBls*)data, (FrBls*)data, true, true, -1, SK_GINV_NAT_N,
                      (const FrBls*)nullptr, (const FrBls*)nullptr, st, EPI_MUL_SUB, &tail);
}
// evaluateXnMinusOneDomainBigCoset (backend/plonk/<curve>/prove.go:1253-1276):
// res[0] = g^n, res[i] = res[i-1] * w_big^n, res[i] -= 1, then fr.BatchInvert
template <class C>
static void xn_minus_one_inv_t(const DomainT<C>* d, size_t n_small, void* out) {
    using F = Fe<C>;
    const size_t rho = d->n / n_small;
    std::vector<F> res(rho);
    res[0] = pow_u64(d->g, n_small);
    const F t = pow_u64(d->omega, n_small);
    for (size_t i = 1; i < rho; i++) res[i] = res[i - 1] * t;
    for (size_t i = 0; i < rho; i++) {
        res[i] = res[i] - F::one();
        GG_CHECK(!res[i].is_zero(), GG_ERR_INVALID_ARG, "x^n - 1 vanishes on the big coset");
        res[i] = inverse(res[i]);
    }
    memcpy(out, res.data(), rho * sizeof(F));
}
void xn_minus_one_inv(gg_domain* big, size_t n_small, void* out) {
    if (big->curve == GG_CURVE_BN254) xn_minus_one_inv_t(big->bn.get(), n_small, out);
    else xn_minus_one_inv_t(big->bls.get(), n_small, out);
}
}  // namespace gg




// ===========================================================================
// Distributed computeH over N GPUs (DESIGN.md "Multi-GPU"), for the
// scalar field of either Groth16 curve (backend/groth16/bn254/prove.go:353-396
// and backend/groth16/bls12-381/prove.go:353-396, the same generated code).
// n = m * N.  Rank k holds the cyclic slice y_k[j] = x[k + N j] of every input
// vector.  A transform of size n is a local size-m transform (root w^N),
// a twist by w^(+-k c1), one all-to-all, and m/N size-N transforms per rank:
//   iFFT:  x_coef[c1 + m c2] = (1/N) sum_k wN^(-k c2) w^(-k c1) iDFT_m(y_k)[c1]
//   FFT:   E[k + N j] = DFT_m( c1 -> w^(c1 k) sum_c2 wN^(c2 k) x'[c1 + m c2] )[j]
// Rank r owns the coefficients c1 = bitrev_m(p), p in [r m/N, (r+1) m/N), all
// c2 < N, so each exchange moves contiguous chunks.  The last step writes h in
// bit-reversed order: coefficient c1 + m c2 lands at r m + N q + bitrev_N(c2),
// i.e. rank r holds h_bitrev[r m, (r+1) m) -- the Z slice [r m, (r+1) m) of
// pk.G1.Z (setup.go:265) -- so the Z-MSM needs no further exchange.
// Three all-to-alls per proof: a, b, c (3 chunks per rank pair); a, b on the
// coset (2 chunks: c stops at its coefficients, h = den coset_iFFT(a b) - den c
// by linearity); then a b (1 chunk).
// ===========================================================================
namespace gg {
template <class C>
struct HShardT {
    using F = Fe<C>;
    std::unique_ptr<DomainT<C>> loc;  // size-m domain, root w^N
    F invN, invN_den;
    DevBuf w_hi, w_lo, wi_hi, wi_lo, g_hi, g_lo, gi_hi, gi_lo;  // split power tables over [0, n)
    int S = 0;
    F wN[16], wNi[16];
    F gm[16], gmi[16];  // g^(m i), g^(-m i): the coset factors of the size-N steps
    DevBuf y, full;     // 3 x m local vectors; staging of host inputs
    DevBuf hblk;        // m elements: h_bitrev[rank m, (rank+1) m)
    DevBuf ccoef;       // m elements: den * c's coefficients of this rank's (q, c2), [c2 chunk + q]
};
}  // namespace gg

struct gg_hshard {
    int curve = GG_CURVE_BN254;
    int log_n = 0, rank = 0, world = 1, log_w = 0, M = 0;
    size_t n = 0, m = 0, chunk = 0;  // chunk = m / N elements per (rank, poly)
    std::unique_ptr<gg::HShardT<gg::FrCfg>> bn;
    std::unique_ptr<gg::HShardT<gg::FrBlsCfg>> bls;
    // the phases of one proof run in order 1, 2, 3, 4 on a handle (phase 4
    // subtracts the c coefficients phase 2 left in ccoef): the last phase run,
    // 0 = none / completed.  Phase 1 may start over at any point (a proof
    // abandoned after a failed exchange); any other phase out of order is refused.
    int last_phase = 0;
    hipStream_t st = nullptr;
    std::mutex mu;
    ~gg_hshard() {
        if (st) (void)hipStreamDestroy(st);
    }
};

namespace gg {
template <class F>
struct PowTab {
    const F *hi, *lo;
    int S;
    __device__ __forceinline__ F at(uint32_t e) const {
        return load_fr(hi + (e >> S)) * load_fr(lo + (e & ((1u << S) - 1)));
    }
};

// the size-N steps' constants: powers of the primitive N-th root and its
// inverse, and the per-output scale cs[i] (folding 1/N and g^(+-m i))
template <class F, int N>
struct SmallRoots {
    F fwd[N], inv[N], cs[N];
};

// X[j] = sum_k x[k] r^(j k) in place, r[i] = r^i: radix-2 DIT in registers
// (N/2 log N butterflies, the r^0 ones without a product -- 5 products for
// N = 8 where the direct sum takes 49)
template <class F, int N>
__device__ __forceinline__ void dft_small(F (&x)[N], const F (&r)[N]) {
    constexpr int LG = N <= 1 ? 0 : (N == 2 ? 1 : (N == 4 ? 2 : (N == 8 ? 3 : 4)));
#pragma unroll
    for (int i = 0; i < N; i++) {
        int j = 0;
#pragma unroll
        for (int b = 0; b < LG; b++) j |= ((i >> b) & 1) << (LG - 1 - b);
        if (i < j) {
            F t = x[i];
            x[i] = x[j];
            x[j] = t;
        }
    }
#pragma unroll
    for (int len = 2; len <= N; len <<= 1)
#pragma unroll
        for (int i = 0; i < N; i += len)
#pragma unroll
            for (int j = 0; j < len / 2; j++) {
                const F u = x[i + j];
                F v = x[i + j + len / 2];
                if (j) v = v * r[(N / len) * j];
                x[i + j] = u + v;
                x[i + j + len / 2] = u - v;
            }
}

// y[j] = x[rank + N j] (zero past len)
template <class F>
__global__ void k_gather_cyclic(F* y, const F* x, size_t len, size_t m, int rank, int N) {
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    size_t i = (size_t)rank + (size_t)N * j;
    F v = i < len ? load_fr(x + i) : F::zero();
    store_fr(y + j, v);
}

// send[(r * npoly + poly) * chunk + q] = y[p] * w^(sign * rank * bitrev_M(p)), p = r chunk + q
template <class F>
__global__ void k_twist_scatter(F* send, const F* y, size_t m, size_t chunk, int M, int npoly, int poly,
                                uint32_t rank, PowTab<F> tw) {
    size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= m) return;
    uint32_t c1 = brev_bits((uint32_t)p, M);
    F v = load_fr(y + p);
    if (rank) v = v * tw.at(rank * c1);
    size_t r = p / chunk, q = p - r * chunk;
    store_fr(send + (r * npoly + poly) * chunk + q, v);
}

// phase 2: finish the inverse transform (size-N iDFT, 1/N), scale by g^c, start
// the forward coset transform (size-N DFT, twist w^(c1 k')) -- per (poly, q).
// recv holds a, b, c (3 chunks per source rank); send gets a, b (2 chunks per
// destination).  c (poly 2) stops after the inverse half: by linearity
// h = den coset_iFFT(a b) - den c_coef, so c needs no coset evaluation -- its
// coefficients times den go to ccoef for phase 4.
template <class F, int N>
__global__ void __launch_bounds__(256) k_cross_fwd(F* send, const F* recv, size_t chunk, int M, uint32_t rank,
                                                   SmallRoots<F, N> R, PowTab<F> gpow, PowTab<F> wpow, F* ccoef,
                                                   F cden) {
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= chunk * 3) return;
    const int poly = (int)(t / chunk);
    const size_t q = t - (size_t)poly * chunk;
    const uint32_t c1 = brev_bits((uint32_t)(rank * chunk + q), M);
    // co[c2] = iDFT_N(in)[c2] / N * g^(c1 + m c2) = g^c1 * (iDFT_N(in)[c2] * cs[c2]);
    // out[k2] = DFT_N(co)[k2] * w^(c1 k2) = g^c1 w^(c1 k2) * DFT_N(iDFT_N(in) * cs)[k2]
    F x[N];
#pragma unroll
    for (int k = 0; k < N; k++) x[k] = load_fr(recv + ((size_t)k * 3 + poly) * chunk + q);
    dft_small<F, N>(x, R.inv);
    if (poly == 2) {
#pragma unroll
        for (int c2 = 0; c2 < N; c2++) store_fr(ccoef + (size_t)c2 * chunk + q, x[c2] * cden);
        return;
    }
#pragma unroll
    for (int c2 = 0; c2 < N; c2++) x[c2] = x[c2] * R.cs[c2];
    dft_small<F, N>(x, R.fwd);
    const F wc = wpow.at(c1);
    F f = gpow.at(c1);
#pragma unroll
    for (int k2 = 0; k2 < N; k2++) {
        if (k2) f = f * wc;
        store_fr(send + ((size_t)k2 * 2 + poly) * chunk + q, x[k2] * f);
    }
}

// y[p] = recv[(r * npoly + poly) * chunk + q], p = r chunk + q
template <class F>
__global__ void k_unpack(F* y, const F* recv, size_t m, size_t chunk, int npoly, int poly) {
    size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= m) return;
    size_t r = p / chunk, q = p - r * chunk;
    store_fr(y + p, load_fr(recv + (r * npoly + poly) * chunk + q));
}

// phase 4: size-N iDFT * den / N * g^-c, written at N q + bitrev_N(c2)
template <class F, int N>
__global__ void __launch_bounds__(256) k_cross_inv_out(F* h, const F* recv, size_t chunk, int M, int logN,
                                                       uint32_t rank, SmallRoots<F, N> R, PowTab<F> gipow,
                                                       const F* ccoef) {
    size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= chunk) return;
    const uint32_t c1 = brev_bits((uint32_t)(rank * chunk + q), M);
    // iDFT_N(in)[c2] * scale * g^-(c1 + m c2) = g^-c1 * (iDFT_N(in)[c2] * cs[c2])
    F x[N];
#pragma unroll
    for (int k = 0; k < N; k++) x[k] = load_fr(recv + (size_t)k * chunk + q);
    dft_small<F, N>(x, R.inv);
    const F gi = gipow.at(c1);
#pragma unroll
    for (int c2 = 0; c2 < N; c2++)
        store_fr(h + (size_t)N * q + brev_bits((uint32_t)c2, logN),
                 x[c2] * R.cs[c2] * gi - load_fr(ccoef + (size_t)c2 * chunk + q));
}

template <class F>
static void pow_tab_upload(int L, int S, const F& x, DevBuf& hi, DevBuf& lo) {
    std::vector<F> h, l;
    build_pow_tables(L, S, x, F::one(), h, l);
    upload(hi, h);
    upload(lo, l);
}

template <class C>
static HShardT<C>* hs_impl(gg_hshard* hs) {
    if constexpr (std::is_same<C, FrCfg>::value) return hs->bn.get();
    else return hs->bls.get();
}

template <class C, int N>
static void launch_cross_fwd(gg_hshard* hs, Fe<C>* send, const Fe<C>* recv, hipStream_t st) {
    using F = Fe<C>;
    HShardT<C>* t = hs_impl<C>(hs);
    SmallRoots<F, N> R;
    for (int i = 0; i < N; i++) {
        R.fwd[i] = t->wN[i];
        R.inv[i] = t->wNi[i];
        R.cs[i] = t->invN * t->gm[i];
    }
    PowTab<F> gp{t->g_hi.template as<F>(), t->g_lo.template as<F>(), t->S};
    PowTab<F> wp{t->w_hi.template as<F>(), t->w_lo.template as<F>(), t->S};
    hipLaunchKernelGGL((k_cross_fwd<F, N>), dim3(grid_for(hs->chunk * 3, 256)), dim3(256), 0, st, send, recv,
                       hs->chunk, hs->M, (uint32_t)hs->rank, R, gp, wp, t->ccoef.template as<F>(), t->invN_den);
    GG_HIP(hipGetLastError());
}

template <class C, int N>
static void launch_cross_inv(gg_hshard* hs, Fe<C>* h, const Fe<C>* recv, hipStream_t st) {
    using F = Fe<C>;
    HShardT<C>* t = hs_impl<C>(hs);
    SmallRoots<F, N> R;
    for (int i = 0; i < N; i++) {
        R.fwd[i] = t->wN[i];
        R.inv[i] = t->wNi[i];
        R.cs[i] = t->invN_den * t->gmi[i];
    }
    PowTab<F> gi{t->gi_hi.template as<F>(), t->gi_lo.template as<F>(), t->S};
    hipLaunchKernelGGL((k_cross_inv_out<F, N>), dim3(grid_for(hs->chunk, 256)), dim3(256), 0, st, h, recv,
                       hs->chunk, hs->M, hs->log_w, (uint32_t)hs->rank, R, gi,
                       (const F*)t->ccoef.template as<F>());
    GG_HIP(hipGetLastError());
}

// ---- the four local phases (exchanges between them are the caller's) ----
// compact: a, b, c already hold this rank's cyclic slices x[rank + N j] (len of
// them), e.g. gathered on the host by the stager, instead of full vectors
template <class C>
static void phase1_t(gg_hshard* hs, const Fe<C>* a, const Fe<C>* b, const Fe<C>* c, size_t len, Fe<C>* send,
                     hipStream_t st, bool compact) {
    using F = Fe<C>;
    HShardT<C>* t = hs_impl<C>(hs);
    const size_t m = hs->m;
    F* y = t->y.template as<F>();
    PowTab<F> twi{t->wi_hi.template as<F>(), t->wi_lo.template as<F>(), t->S};
    const F* src[3] = {a, b, c};
    for (int p = 0; p < 3; p++) {
        F* yp = y + (size_t)p * m;
        hipLaunchKernelGGL(k_gather_cyclic<F>, dim3(grid_for(m, 256)), dim3(256), 0, st, yp, src[p], len, m,
                           compact ? 0 : hs->rank, compact ? 1 : hs->world);
        GG_HIP(hipGetLastError());
        // iDFT_m (DIF: natural -> bit-reversed), 1/m folded in
        run_transform(t->loc.get(), yp, yp, false, true, -1, SK_NINV, (const F*)nullptr, (const F*)nullptr, st);
        hipLaunchKernelGGL(k_twist_scatter<F>, dim3(grid_for(m, 256)), dim3(256), 0, st, send, yp, m, hs->chunk,
                           hs->M, 3, p, (uint32_t)hs->rank, twi);
        GG_HIP(hipGetLastError());
    }
}

template <class C>
static void phase2_t(gg_hshard* hs, const Fe<C>* recv, Fe<C>* send, hipStream_t st) {
    switch (hs->world) {
        case 1: launch_cross_fwd<C, 1>(hs, send, recv, st); break;
        case 2: launch_cross_fwd<C, 2>(hs, send, recv, st); break;
        case 4: launch_cross_fwd<C, 4>(hs, send, recv, st); break;
        case 8: launch_cross_fwd<C, 8>(hs, send, recv, st); break;
        case 16: launch_cross_fwd<C, 16>(hs, send, recv, st); break;
        default: throw Error(GG_ERR_UNSUPPORTED, "distributed computeH: world must be 1, 2, 4, 8 or 16");
    }
}

template <class C>
static void phase3_t(gg_hshard* hs, const Fe<C>* recv, Fe<C>* send, hipStream_t st) {
    using F = Fe<C>;
    HShardT<C>* t = hs_impl<C>(hs);
    const size_t m = hs->m;
    F* y = t->y.template as<F>();
    const F* nul = nullptr;
    for (int p = 0; p < 2; p++) {  // a, b: phase 2 sent 2 polys per rank pair
        hipLaunchKernelGGL(k_unpack<F>, dim3(grid_for(m, 256)), dim3(256), 0, st, y + (size_t)p * m, recv, m,
                           hs->chunk, 2, p);
        GG_HIP(hipGetLastError());
    }
    // coset evaluations on this rank's points g w^(rank + N j) (DIT: bit-reversed -> natural);
    // the last pass of b's transform emits a*b
    run_transform(t->loc.get(), y, y, true, false, -1, -1, nul, nul, st);
    run_transform(t->loc.get(), y + m, y + m, true, false, -1, -1, y, nul, st, EPI_MUL);
    // inverse of the product's evaluations: iDFT_m, then twist w^(-rank c1)
    run_transform(t->loc.get(), y + m, y + m, false, true, -1, SK_NINV, nul, nul, st);
    PowTab<F> twi{t->wi_hi.template as<F>(), t->wi_lo.template as<F>(), t->S};
    hipLaunchKernelGGL(k_twist_scatter<F>, dim3(grid_for(m, 256)), dim3(256), 0, st, send, y + m, m, hs->chunk,
                       hs->M, 1, 0, (uint32_t)hs->rank, twi);
    GG_HIP(hipGetLastError());
}

template <class C>
static void phase4_t(gg_hshard* hs, const Fe<C>* recv, Fe<C>* h, hipStream_t st) {
    switch (hs->world) {
        case 1: launch_cross_inv<C, 1>(hs, h, recv, st); break;
        case 2: launch_cross_inv<C, 2>(hs, h, recv, st); break;
        case 4: launch_cross_inv<C, 4>(hs, h, recv, st); break;
        case 8: launch_cross_inv<C, 8>(hs, h, recv, st); break;
        case 16: launch_cross_inv<C, 16>(hs, h, recv, st); break;
        default: throw Error(GG_ERR_UNSUPPORTED, "distributed computeH: world must be 1, 2, 4, 8 or 16");
    }
}

// curve dispatch over opaque 32-B elements (Fr* for both fields)
static void phase_order(gg_hshard* hs, int phase) {
    GG_CHECK(phase == 1 || hs->last_phase == phase - 1, GG_ERR_INVALID_ARG,
             "distributed computeH: phase " + std::to_string(phase) + " after phase " +
                 std::to_string(hs->last_phase) +
                 " on this handle (phases run 1, 2, 3, 4 in order, one proof at a time per handle)");
}
// records a phase as done only once its body has been enqueued; a phase that
// throws leaves the handle expecting phase 1 again (its y / ccoef state is stale)
struct PhaseStep {
    gg_hshard* hs;
    int phase;
    bool ok = false;
    PhaseStep(gg_hshard* h, int p) : hs(h), phase(p) { phase_order(h, p); }
    ~PhaseStep() { hs->last_phase = ok && phase != 4 ? phase : 0; }
};
void hshard_phase1(gg_hshard* hs, const Fr* a, const Fr* b, const Fr* c, size_t len, Fr* send, hipStream_t st,
                   bool compact = false) {
    PhaseStep step(hs, 1);
    if (hs->curve == GG_CURVE_BN254) phase1_t<FrCfg>(hs, a, b, c, len, send, st, compact);
    else phase1_t<FrBlsCfg>(hs, (const FrBls*)a, (const FrBls*)b, (const FrBls*)c, len, (FrBls*)send, st, compact);
    step.ok = true;
}
void hshard_phase2(gg_hshard* hs, const Fr* recv, Fr* send, hipStream_t st) {
    PhaseStep step(hs, 2);
    if (hs->curve == GG_CURVE_BN254) phase2_t<FrCfg>(hs, recv, send, st);
    else phase2_t<FrBlsCfg>(hs, (const FrBls*)recv, (FrBls*)send, st);
    step.ok = true;
}
void hshard_phase3(gg_hshard* hs, const Fr* recv, Fr* send, hipStream_t st) {
    PhaseStep step(hs, 3);
    if (hs->curve == GG_CURVE_BN254) phase3_t<FrCfg>(hs, recv, send, st);
    else phase3_t<FrBlsCfg>(hs, (const FrBls*)recv, (FrBls*)send, st);
    step.ok = true;
}
void hshard_phase4(gg_hshard* hs, const Fr* recv, Fr* h, hipStream_t st) {
    PhaseStep step(hs, 4);
    if (hs->curve == GG_CURVE_BN254) phase4_t<FrCfg>(hs, recv, h, st);
    else phase4_t<FrBlsCfg>(hs, (const FrBls*)recv, (FrBls*)h, st);
    step.ok = true;
}

size_t hshard_m(const gg_hshard* hs, int* rank, int* world, int* log_n) {
    *rank = hs->rank;
    *world = hs->world;
    *log_n = hs->log_n;
    return hs->m;
}
int hshard_curve(const gg_hshard* hs) { return hs->curve; }
Fr* hshard_h(gg_hshard* hs) {
    return hs->curve == GG_CURVE_BN254 ? hs->bn->hblk.as<Fr>() : hs->bls->hblk.as<Fr>();
}

// bytes per rank pair of the all-to-all that follows phase `phase` (1..3):
// 3 polys after phase 1, 2 after phase 2, 1 after phase 3
size_t hshard_exchange_bytes(const gg_hshard* hs, int phase) {
    return hs->chunk * 32 * (size_t)(phase == 1 ? 3 : phase == 2 ? 2 : 1);
}

template <class C>
static void hshard_build(gg_hshard* hs, HShardT<C>* t, const void* omega_mont, const void* coset_gen_mont) {
    using F = Fe<C>;
    F w, g;
    memcpy(w.v, omega_mont, 32);
    memcpy(g.v, coset_gen_mont, 32);
    F wm = pow_u64(w, (uint64_t)hs->world);
    t->loc.reset(domain_build<C>(hs->M, wm.v, g.v));  // checks the order of w^N = m
    // w must have order exactly n: w^(n/2) != 1 (w^N already has order m)
    GG_CHECK(!(pow_u64(w, hs->n / 2) == F::one()), GG_ERR_INVALID_ARG, "omega order < n");
    GG_CHECK(pow_u64(w, hs->n) == F::one(), GG_ERR_INVALID_ARG, "omega^n != 1");
    F wNroot = pow_u64(w, hs->m);  // primitive N-th root
    F wNinv = inverse(wNroot);
    F a = F::one(), b = F::one();
    for (int i = 0; i < 16; i++) {
        t->wN[i] = a;
        t->wNi[i] = b;
        a = a * wNroot;
        b = b * wNinv;
    }
    F nn = F::zero();
    nn.v[0] = (uint32_t)hs->world;
    t->invN = inverse(to_mont(nn));
    F gn = pow_u64(g, hs->n) - F::one();
    GG_CHECK(!gn.is_zero(), GG_ERR_INVALID_ARG, "g^n == 1: coset generator in the domain");
    t->invN_den = t->invN * inverse(gn);
    {
        const F gmr = pow_u64(g, hs->m), gmr_i = inverse(gmr);
        F x = F::one(), y = F::one();
        for (int i = 0; i < 16; i++) {
            t->gm[i] = x;
            t->gmi[i] = y;
            x = x * gmr;
            y = y * gmr_i;
        }
    }
    t->S = (hs->log_n + 1) / 2;
    pow_tab_upload(hs->log_n, t->S, w, t->w_hi, t->w_lo);
    pow_tab_upload(hs->log_n, t->S, inverse(w), t->wi_hi, t->wi_lo);
    pow_tab_upload(hs->log_n, t->S, g, t->g_hi, t->g_lo);
    pow_tab_upload(hs->log_n, t->S, inverse(g), t->gi_hi, t->gi_lo);
    t->y.alloc(3 * hs->m * 32);
    t->hblk.alloc(hs->m * 32);
    t->ccoef.alloc(hs->m * 32);
}

gg_hshard* hshard_create(int curve, int log_n, const void* omega_mont, const void* coset_gen_mont, int rank,
                         int world) {
    GG_CHECK(omega_mont && coset_gen_mont, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "bad curve");
    GG_CHECK(world >= 1 && world <= 16 && (world & (world - 1)) == 0, GG_ERR_UNSUPPORTED,
             "distributed computeH: world must be a power of two <= 16");
    GG_CHECK(rank >= 0 && rank < world, GG_ERR_INVALID_ARG, "rank out of range");
    int lw = 0;
    while ((1 << lw) < world) lw++;
    GG_CHECK(log_n >= 1 && log_n <= 28 && log_n >= 2 * lw, GG_ERR_INVALID_ARG,
             "distributed computeH needs 2^log_n >= world^2");
    std::unique_ptr<gg_hshard> hs(new gg_hshard());
    hs->curve = curve;
    hs->log_n = log_n;
    hs->rank = rank;
    hs->world = world;
    hs->log_w = lw;
    hs->n = (size_t)1 << log_n;
    hs->M = log_n - lw;
    hs->m = hs->n >> lw;
    hs->chunk = hs->m >> lw;
    if (curve == GG_CURVE_BN254) {
        hs->bn.reset(new HShardT<FrCfg>());
        hshard_build(hs.get(), hs->bn.get(), omega_mont, coset_gen_mont);
    } else {
        hs->bls.reset(new HShardT<FrBlsCfg>());
        hshard_build(hs.get(), hs->bls.get(), omega_mont, coset_gen_mont);
    }
    return hs.release();
}

// Whole distributed computeH on this rank; xchg(ctx, send, recv, bytes_per_rank)
// performs the all-to-all (blocking).  a/b/c: full vectors on the device.
void hshard_run(gg_hshard* hs, const Fr* a, const Fr* b, const Fr* c, size_t len, bool compact, Fr* send,
                Fr* recv, gg_exchange_fn xchg, void* ctx, hipStream_t st) {
    std::lock_guard<std::mutex> lk(hs->mu);  // y / hblk / ccoef are per-handle scratch
    auto exchange = [&](int phase) {
        GG_WAIT_STREAM(st);
        set_last_error("");
        int rc = xchg(ctx, send, recv, hshard_exchange_bytes(hs, phase));
        if (rc == GG_ERR_TIMEOUT) throw Error(rc, gg_last_error());  // the one-process barrier's deadline
        const std::string why = gg_last_error();
        GG_CHECK(rc == 0, GG_ERR_INTERNAL,
                 "exchange callback failed after phase " + std::to_string(phase) + (why.empty() ? "" : ": " + why));
    };
    hshard_phase1(hs, a, b, c, len, send, st, compact);
    exchange(1);
    hshard_phase2(hs, recv, send, st);
    exchange(2);
    hshard_phase3(hs, recv, send, st);
    exchange(3);
    hshard_phase4(hs, recv, hshard_h(hs), st);
}
}  // namespace gg

extern "C" int gg_hshard_create_ex(int curve, int log_n, const void* omega_mont, const void* coset_gen_mont,
                                   int rank, int world, gg_hshard_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out, GG_ERR_INVALID_ARG, "null argument");
    *out = hshard_create(curve, log_n, omega_mont, coset_gen_mont, rank, world);
    GG_CAPI_END
}

extern "C" int gg_hshard_create(int log_n, const void* omega_mont, const void* coset_gen_mont, int rank,
                                int world, gg_hshard_t* out) {
    return gg_hshard_create_ex(GG_CURVE_BN254, log_n, omega_mont, coset_gen_mont, rank, world, out);
}

extern "C" int gg_hshard_release(gg_hshard_t hs) {
    GG_CAPI_BEGIN
    delete hs;
    GG_CAPI_END
}

extern "C" int gg_hshard_info(gg_hshard_t hs, size_t* m, size_t* exchange_bytes) {
    GG_CAPI_BEGIN
    GG_CHECK(hs, GG_ERR_INVALID_ARG, "null argument");
    if (m) *m = hs->m;
    if (exchange_bytes) *exchange_bytes = hs->world * hshard_exchange_bytes(hs, 1);
    GG_CAPI_END
}

extern "C" int gg_hshard_exchange_bytes(gg_hshard_t hs, int phase, size_t* bytes_per_rank) {
    GG_CAPI_BEGIN
    GG_CHECK(hs && bytes_per_rank, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(phase >= 1 && phase <= 3, GG_ERR_INVALID_ARG, "phase must be 1..3");
    *bytes_per_rank = hshard_exchange_bytes(hs, phase);
    GG_CAPI_END
}

extern "C" int gg_hshard_phase(gg_hshard_t hs, int phase, const void* a, const void* b, const void* c,
                               size_t len, int inputs_on_device, const void* recv, void* send_or_h,
                               void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(hs && send_or_h, GG_ERR_INVALID_ARG, "null argument");
    std::lock_guard<std::mutex> lk(hs->mu);
    hipStream_t st = pick_stream(hip_stream);
    if (phase == 1) {
        GG_CHECK(a && b && c, GG_ERR_INVALID_ARG, "null input");
        GG_CHECK(len <= hs->n, GG_ERR_INVALID_ARG, "len > domain cardinality");
        const Fr* src[3] = {(const Fr*)a, (const Fr*)b, (const Fr*)c};
        if (!inputs_on_device) {
            DevBuf& full = hs->curve == GG_CURVE_BN254 ? hs->bn->full : hs->bls->full;
            full.reserve(3 * std::max<size_t>(len, 1) * 32);
            for (int i = 0; i < 3; i++) {
                Fr* d = full.as<Fr>() + i * len;
                if (len) GG_HIP(hipMemcpyAsync(d, src[i], len * 32, hipMemcpyHostToDevice, st));
                src[i] = d;
            }
        }
        hshard_phase1(hs, src[0], src[1], src[2], len, (Fr*)send_or_h, st);
    } else {
        GG_CHECK(recv, GG_ERR_INVALID_ARG, "null recv");
        if (phase == 2) hshard_phase2(hs, (const Fr*)recv, (Fr*)send_or_h, st);
        else if (phase == 3) hshard_phase3(hs, (const Fr*)recv, (Fr*)send_or_h, st);
        else if (phase == 4) hshard_phase4(hs, (const Fr*)recv, (Fr*)send_or_h, st);
        else throw Error(GG_ERR_INVALID_ARG, "phase must be 1..4");
    }
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}
