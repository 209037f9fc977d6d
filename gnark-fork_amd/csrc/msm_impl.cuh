#pragma once
// (shared by msm_g1.hip / msm_g2.hip)
// Pippenger bucket MSM over BN254 G1 / G2 for gfx950.
//
// Replaces G1Jac/G2Jac.MultiExp (prove.go:201-290) and iciclegnark
// MsmOnDevice / MsmG2OnDevice (icicle.go:302-382).
//
// Design (DESIGN.md "MSM"):
//  * Fixed-base precomputation, sized for 288 GB HBM: at base creation every
//    point P_i is stored with its window shifts 2^(c*w) * P_i (affine,
//    w < W = ceil(255/c)).  All W windows then share ONE set of 2^(c-1)
//    buckets: no per-window bucket reduction, no Horner doubling chain.
//  * Signed c-bit digits (|d| <= 2^(c-1)); entry (w, i, sign) goes to bucket |d|-1.
//  * Counting sort by bucket: histogram (atomics) -> exclusive scan -> scatter.
//  * Bucket accumulation as a segmented reduction that is immune to skewed
//    scalars (real witnesses are mostly 0/1): every bucket is cut into work
//    items of <= K entries, one thread per item, mixed XYZZ additions; then
//    the per-bucket partials are summed the same way until one remains.
//  * Bucket reduction sum_b (b+1) S_b: one thread per segment of buckets with
//    a running sum, plus a double-and-add shift, then a tree sum.
#include "common.h"
#include "curve.cuh"
#include "field29.cuh"
#include "prof.h"
#include <mutex>
#include <vector>
#include <algorithm>
#include <memory>
#include <cmath>
#include <cstdlib>
#include <cstring>

struct gg_msm_base;

namespace gg {

// ------------------------------------------------------------------ loads
template <class T>
__device__ __forceinline__ T ld(const T* p) {
    static_assert(sizeof(T) % 16 == 0, "16B multiple");
    T r;
    const uint4* s = reinterpret_cast<const uint4*>(p);
    uint4* d = reinterpret_cast<uint4*>(&r);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 16); i++) d[i] = s[i];
    return r;
}
template <class T>
__device__ __forceinline__ void st(T* p, const T& v) {
    uint4* d = reinterpret_cast<uint4*>(p);
    const uint4* s = reinterpret_cast<const uint4*>(&v);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 16); i++) d[i] = s[i];
}

// ---- non-template kernels (msm_common.hip)
__global__ void k_scan_block(const uint32_t* in, uint32_t* out, uint32_t* sums, size_t n);
__global__ void k_scan_add(uint32_t* out, const uint32_t* sums, size_t n);
__global__ void k_set_total(uint32_t* out, const uint32_t* in, size_t n);
__global__ void k_bucket_max(const uint32_t* offsets, size_t nb, uint32_t* maxcnt);
void exclusive_scan(const uint32_t* in, uint32_t* out, size_t n, hipStream_t st,
                    std::vector<DevBuf>& tmp, int depth = 0);
int choose_c(size_t n, size_t point_bytes, int total_bits = 255);
// precompute groups for a table of `bytes` (all W windows stored) plus `extra`
// bytes of other allocations: GG_MSM_GROUPS if set, else the smallest power of
// two G <= W whose table (bytes / G, rounded up to whole copies) and extra fit
// the free HBM less a reserve, capped by gg_set_hbm_budget
int choose_groups(double bytes, double extra, int W);
// the same for several tables that must share one G (bytes[i] with all W[i] windows stored)
int choose_groups_multi(const double* bytes, const int* W, int k, double extra);
// scalar field of a base: 0 = BN254 fr (254-bit), 1 = BLS12-381 fr (255-bit)
inline int scalar_total_bits(int scurve) { return scurve ? 256 : 255; }
// Window layout: W windows of bits[w] (<= c) bits at bit offset off[w], summing
// to scalar bits + 1 (the signed-digit carry): 255 for BN254 fr (254-bit),
// 256 for BLS12-381 fr (255-bit).  Widths are balanced (they differ
// by at most one bit), so no window is much narrower than c: a narrow top
// window would pile all n of its entries into a few buckets.
struct WinSpec {
    uint8_t bits[64];
    uint8_t off[64];
};
inline WinSpec make_windows(int c, int W, int total) {
    WinSpec ws{};
    const int q = total / W, r = total % W;
    int o = 0;
    for (int w = 0; w < W; w++) {
        ws.bits[w] = (uint8_t)(q + (w < r ? 1 : 0));
        ws.off[w] = (uint8_t)o;
        o += ws.bits[w];
    }
    (void)c;
    return ws;
}
struct MsmSort;
// up to kMaxBatch scalar vectors sorted together over one base (msm_prepare_batch)
constexpr int kMaxBatch = 4;
struct VecPtrs {
    const void* p[kMaxBatch];
};
void sort_entries(const gg_msm_base* b, MsmSort* s, const VecPtrs& vp, hipStream_t st);
// slog > 0: the sort keeps the bucket stripe sres of 2^slog (buckets b with
// b mod 2^slog = sres, see MsmSort)
void msm_prepare(const gg_msm_base* b, MsmSort* s, const Fr* scalars_dev, hipStream_t st, int slog = 0,
                 uint32_t sres = 0);
// does a batch of nvec vectors over a base of this shape fit the sort's 32-bit words (msm.hip)
bool msm_batch_fits(size_t n, int W, int c, int G, int nvec);
void msm_prepare_batch(const gg_msm_base* b, MsmSort* s, const VecPtrs& vp, int nvec, hipStream_t st, int slog = 0,
                       uint32_t sres = 0);
// b's sort from a's (same window layout, a indexes its scalars directly, bmap:
// a's scalar index -> b's point or ~0); waits for sa->ready_ev on st
void msm_prepare_derived(const gg_msm_base* a, const MsmSort* sa, const gg_msm_base* b, MsmSort* sb,
                         const uint32_t* bmap, hipStream_t st);

constexpr uint32_t LIGHT = 16;
// Bucket ids: B = j 2^(c-1) + b for precompute group j (< G) and bucket b of the
// group.  The sort orders the low c-1 bits bit-reversed (pi(b) = bitrev_{c-1}(b),
// see sort_entries); pi is an involution, so the same map takes a sort position
// q back to its bucket B.
__device__ __forceinline__ uint32_t bucket_perm(uint32_t B, int c) {
    const uint32_t m = (1u << (c - 1)) - 1;
    return (B & ~m) | (__brev(B & m) >> (33 - c));
}
// which groups accumulate in a reduced-radix form, and which one
template <class F>
struct RadixOf {
    static constexpr bool on = false;
    using C = Fp29Cfg;
};
template <>
struct RadixOf<Fp> {
    static constexpr bool on = true;
    using C = Fp29Cfg;
};
template <>
struct RadixOf<Fp2> {
    static constexpr bool on = true;
    using C = Fp29Cfg;
};
template <>
struct RadixOf<FpBls> {
    static constexpr bool on = true;
    using C = FpBls28Cfg;
};
// base coordinates (field elements, gnark form) -> x R' mod p in place
template <class C>
__global__ void __launch_bounds__(256) k_to_radix(Fe<typename C::Std>* v, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fe<typename C::Std> x = v[i];
    v[i] = to_rl<C>(x);
}
 // buckets spanning <= LIGHT ranges are combined serially

// Level 1, balanced: thread t adds the sorted entries [t K, min((t+1) K, E)) --
// every lane does exactly K mixed XYZZ adds, whatever the bucket sizes (the
// per-bucket items this replaces were K(m-1)/m..K long, and a wave waited for
// its longest).  Where the range crosses a bucket boundary the running sum is
// flushed: the range's first segment goes to head[t], its last to tail[t], and
// a segment that starts and ends inside the range is a whole bucket, written
// straight to S[brev(q)] (natural bucket order, see sort_entries).
// tbucket[t] = bucket (sort order) of the range's first entry.
// Partials are stored in the accumulator's own form (radix limbs for the
// groups that accumulate in one): a flush is then a few stores instead of a
// conversion (4 or 8 products), which matters because a wave executes the
// flush whenever ANY of its lanes crosses a bucket boundary -- about every
// other step at 2^24.  The consumers convert once, a lane per partial.
template <class F>
struct PartialOf {
    using T = Xyzz<F>;
};
template <>
struct PartialOf<Fp> {
    using T = XyzzL<Fp29Cfg>;
};
template <>
struct PartialOf<FpBls> {
    using T = XyzzL<FpBls28Cfg>;
};
template <>
struct PartialOf<Fp2> {
    using T = Xyzz2_29;
};

// the group law on the partial form, for the lane-per-bucket level 2 and
// weighted sums (k_range_tree_r, k_bucket_sum_r, k_bucket_runsum)
template <class F>
struct PartialOps {  // G1 groups: XyzzL, coordinates < 7p
    using T = typename PartialOf<F>::T;
    using C = typename RadixOf<F>::C;
    static __device__ __forceinline__ T inf() { return inf_l<C>(); }
    static __device__ __forceinline__ T add(const T& p, const T& q) { return xyzzl_add(p, q); }
    static __device__ __forceinline__ T neg(const T& p) {
        T r = p;
        if (!is_inf_l(r)) r.y = sub<8>(Fl<C>{}, r.y);  // y < 7p
        return r;
    }
};
template <>
struct PartialOps<Fp2> {  // BN254 G2: Xyzz2_29, coordinates < 2p
    using T = Xyzz2_29;
    static __device__ __forceinline__ T inf() { return inf2_29(); }
    static __device__ __forceinline__ T add(const T& p, const T& q) { return xyzz2_29_add(p, q); }
    static __device__ __forceinline__ T neg(const T& p) { return xyzz2_29_neg(p); }
};

template <class P>
__device__ __forceinline__ void range_store(const P& acc, bool first, bool last, uint32_t q, int c, size_t t,
                                            P* head, P* tail, P* S) {
    if (first) st(head + t, acc);
    else if (last) st(tail + t, acc);
    else st(S + bucket_perm(q, c), acc);
}

// waves per SIMD the accumulation is compiled for: 2 (<= 256 VGPRs) for the G1
// groups; 1 (512 VGPRs, no scratch spills) for the Fp2 groups (BN254 G2 in the
// radix-2^29 form needs ~300, BLS12-381 G2 more)
#ifndef GG_G2_WAVES1
#define GG_G2_WAVES1 0
#endif
#ifndef GG_G1_WAVES
#define GG_G1_WAVES 2
#endif
#ifndef GG_BLS_WAVES
#define GG_BLS_WAVES 2
#endif
template <class F>
constexpr int kAccumWaves = (GG_G2_WAVES1 && std::is_same<F, Fp2>::value) || std::is_same<F, Fp2Bls>::value
                                ? 1
                                : (std::is_same<F, Fp>::value ? GG_G1_WAVES
                                                              : (std::is_same<F, FpBls>::value ? GG_BLS_WAVES : 2));

// entry k (0..3) of a 16-B chunk of sorted entries held in registers
__device__ __forceinline__ uint32_t chunk_at(const uint4& c, uint32_t k) {
    return k == 0 ? c.x : (k == 1 ? c.y : (k == 2 ? c.z : c.w));
}
__device__ __forceinline__ uint4 chunk_ld(const uint32_t* sorted, uint32_t base4) {
    return *reinterpret_cast<const uint4*>(sorted + base4);
}

// dynamic LDS of k_accum_range<F>: the BN254 G2 gather slots (two 8-KB slots
// per wave, four waves per block)
#ifndef GG_ACCUM_R4LOOP
#define GG_ACCUM_R4LOOP 0  // A/B builds: round 4's G2 loop (no LDS gather)
#endif
#ifndef GG_G1_PIPE
#define GG_G1_PIPE 0  // A/B builds: the G1 loop with every load unconditional
#endif
// The register-path gathers (BN254 G1 in GG_G1_LDS=0 builds) carry the nontemporal hint: a point is
// read once per launch, and the hint keeps the gathers from displacing the
// entry chunks in L2 / MALL.  A/B on one box (profiles/r05_d_accum_ab.txt):
// 13.90 vs 14.07-14.14 ms per 2^24 launch.  The LDS-DMA gathers (BN254 G2,
// BLS12-381 G1) keep the default policy: with the hint G2 took 26.89 vs 26.2 ms.
// The hint pays on big tables only: the 8-way shard's 1.7-GB tables (2^21 wires)
// proved in 17.33 / 17.65 vs 17.71-18.13 ms without it (r05_m, r05_n), so a
// launch takes it from a table of GG_ACCUM_NT_GB (default 4) GB up.
// GG_PT_NT=0 builds the default policy everywhere, 2 the hint everywhere.
#ifndef GG_PT_NT
#define GG_PT_NT 1
#endif
// one accumulation point (a gather with no reuse), NT: with the nontemporal hint
template <bool NT, class T>
__device__ __forceinline__ T ld_pt(const T* p) {
    if constexpr (NT) {
        typedef unsigned int u4v __attribute__((ext_vector_type(4)));
        static_assert(sizeof(T) % 16 == 0, "16B multiple");
        T r;
        const u4v* s = reinterpret_cast<const u4v*>(p);
        u4v* d = reinterpret_cast<u4v*>(&r);
#pragma unroll
        for (int i = 0; i < (int)(sizeof(T) / 16); i++) d[i] = __builtin_nontemporal_load(s + i);
        return r;
    } else {
        return ld(p);
    }
}
// Points gathered straight into LDS (global_load_lds_dwordx4: no VGPRs), for
// the accumulations whose adds use all the registers of two waves per SIMD
// (BN254 G2, BLS12-381 G1): per wave two slots of NCH 16-B chunks x 64 lanes,
// laid out [slot][chunk][lane] (one DMA instruction fills one [chunk] row, the
// read-back is conflict-free).  The caller reads point e out of its slot, then
// issues the gather of point e + 1 into the other one: the compiler's wait for
// the slot being read then covers only the older gather.
template <int NCH>
struct LdsRing {
    uint4* wb;
    uint32_t lane;
    __device__ __forceinline__ explicit LdsRing(uint4* lds)
        : wb(lds + (threadIdx.x >> 6) * (2u * NCH * 64u)), lane(threadIdx.x & 63u) {}
    __device__ __forceinline__ void gather(const void* src, uint32_t slot) const {
#pragma unroll
        for (int k = 0; k < NCH; k++)
            __builtin_amdgcn_global_load_lds((const void*)((const char*)src + 16 * k),
                                             (__attribute__((address_space(3))) void*)(wb + (slot * NCH + k) * 64u),
                                             16, 0, GG_PT_NT == 2 ? 2 : 0);
    }
    template <class T>
    __device__ __forceinline__ T read(uint32_t slot) const {
        static_assert(sizeof(T) == 16 * NCH, "point size");
        T r;
        uint4* d = reinterpret_cast<uint4*>(&r);
#pragma unroll
        for (int k = 0; k < NCH; k++) d[k] = wb[(slot * NCH + k) * 64u + lane];
        return r;
    }
};
// The sorted entries of an LDS-ring accumulation, read in 16-B chunks (round 6).
// The ring loops of round 5 loaded one 4-B entry and one bucket boundary per
// step: each lane's next entry sits K entries away from its neighbour's, so every
// such load touches a line of its own, and the point gathers streaming through
// L2 evict it between a lane's steps -- 2.3 GB of re-fetches per 2^24 G1 launch
// above the register loop's (r05_z2 vs r05_z3 PMC: 14.89 -> 17.23 GB FETCH).
// Here a lane holds two chunks: c0 with the entry the next gather needs, c1 the
// four after it, loaded four steps before use.  Step i is the same on every lane
// of a wave (all start at their e0 together), so the reload is a uniform branch;
// K is a multiple of 4 (msm_finish_multi), so e0 and every chunk are 16-B aligned.
// GG_RING_CHUNKS=0 builds round 5's per-step loads (A/B).
// BN254 G2 (256 VGPRs at two waves per SIMD) keeps its per-step entry loads:
// the chunks' 8 VGPRs spill 196 instead of 16 B there (GG_RING_CHUNKS_G2=1).
#ifndef GG_RING_CHUNKS
#define GG_RING_CHUNKS 1
#endif
#ifndef GG_RING_CHUNKS_G2
#define GG_RING_CHUNKS_G2 0
#endif
struct EntryChunks {
    uint4 c0, c1;
    // entries e0 .. e0 + 7 (the sorted list has 64 B of slack past its end)
    __device__ __forceinline__ EntryChunks(const uint32_t* sorted, uint32_t e0)
        : c0(chunk_ld(sorted, e0)), c1(chunk_ld(sorted, e0 + 4)) {}
    // step i (uniform): the chunk holding entry e0 + i + 2 moves into c0 when that
    // entry starts a chunk, and the chunk after it is requested; issue this before
    // the step's gather, so the wait for that gather covers the load
    __device__ __forceinline__ void advance(const uint32_t* sorted, uint32_t e0, uint32_t i) {
        if (((i + 2) & 3u) == 0) {
            c0 = c1;
            c1 = chunk_ld(sorted, e0 + i + 6);
        }
    }
    // entry e0 + i + 2 (after advance(i))
    __device__ __forceinline__ uint32_t next2(uint32_t i) const { return chunk_at(c0, (i + 2) & 3u); }
};
// BN254 G2 (128-B points), BLS12-381 G1 (96-B) and BN254 G1 (64-B) take the LDS
// ring.  BN254 G1 too since r05w: 149 instead of 164 VGPRs, three waves per
// SIMD either way, the one-GPU 2^24 prove 106.8 / 106.8 vs 108.8 / 108.7 ms,
// the 8-way shard 17.48 vs 17.66 ms (profiles/r05_w_g1_lds_ab.md); GG_G1_LDS=0
// builds the register loop (with the nontemporal policy below) for A/B.
#ifndef GG_G1_LDS
#define GG_G1_LDS 1
#endif
template <class F>
constexpr bool kLdsGather = !GG_ACCUM_R4LOOP && (std::is_same<F, Fp2>::value || std::is_same<F, FpBls>::value ||
                                                 (GG_G1_LDS && std::is_same<F, Fp>::value));
// dynamic LDS of k_accum_range<F>: two slots per wave, four waves per block
template <class F>
constexpr size_t kAccumLds = kLdsGather<F> ? 4 * 2 * sizeof(Affine<F>) * 64 : 0;

template <class F, bool NT>
__global__ void __launch_bounds__(256, kAccumWaves<F>) k_accum_range(const Affine<F>* pts, const uint32_t* sorted,
                                                     const uint32_t* offsets, uint32_t nb, int c,
                                                     uint32_t K, int skip_inf, typename PartialOf<F>::T* head,
                                                     typename PartialOf<F>::T* tail, typename PartialOf<F>::T* S,
                                                     uint32_t* tbucket, uint32_t pmask) {
    const uint32_t E = offsets[nb];
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t e0w = (uint64_t)t * K;
    if (e0w >= E) return;
    const uint32_t e0 = (uint32_t)e0w;
    const uint32_t e1 = (uint32_t)min<uint64_t>(e0w + K, E);
    // bucket of e0: the largest q with offsets[q] <= e0 (empty buckets share
    // their successor's offset, so this is the non-empty one holding e0)
    uint32_t lo = 0, hi = nb;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (offsets[mid] <= e0) lo = mid;
        else hi = mid;
    }
    uint32_t q = lo;
    tbucket[t] = q;
    // the next boundary is loaded one flush ahead: a flush (taken by the whole
    // wave when any lane crosses a boundary) then never waits on a load
    uint32_t bnd = offsets[q + 1], bnd2 = offsets[min(q + 2, nb)];
    uint32_t seg0 = e0;
    if constexpr (std::is_same<F, Fp>::value || std::is_same<F, FpBls>::value) {
        // G1: reduced-radix accumulator (field29.cuh; BN254 9 x 29, BLS12-381
        // 14 x 28 bits); the base holds x R' mod p, partials leave in radix form
        using C = typename RadixOf<F>::C;
        XyzzL<C> acc = inf_l<C>();
        if constexpr (kLdsGather<F>) {  // 64-B (BN254) / 96-B (BLS12-381) points through the LDS ring
            extern __shared__ uint4 acc_lds[];
            const LdsRing<sizeof(Affine<F>) / 16> ring(acc_lds);
#if GG_RING_CHUNKS
            EntryChunks ec(sorted, e0);
            uint32_t v = ec.c0.x, vn = ec.c0.y;
            ring.gather(pts + (v & pmask), 0);
            for (uint32_t i = 0;; i++) {
                const uint32_t e = e0 + i;
                if (e >= e1) break;
                const uint32_t sl = i & 1u;
                const Affine<F> qp = ring.template read<Affine<F>>(sl);
                const uint32_t cv = v;
                if (e == bnd) {  // before the gather (see the Fp2 branch)
                    range_store(acc, seg0 == e0, false, q, c, t, head, tail, S);
                    acc = inf_l<C>();
                    seg0 = e;
                    q++;
                    bnd = bnd2;
                    if (bnd == e) {
                        uint32_t b2;
                        do {
                            q++;
                            b2 = offsets[min(q + 1, nb)];
                        } while (b2 == e);
                        bnd = b2;
                    }
                }
                ec.advance(sorted, e0, i);
                const uint32_t nidx = (e + 1 < e1) ? vn : v;
                ring.gather(pts + (nidx & pmask), sl ^ 1u);
                v = nidx;
                vn = ec.next2(i);
                // every step, after the gather: loaded at the flush instead, its
                // value is copied into the loop-carried register at once, which
                // waits for it (ISA); a wave's lanes share 2-3 lines of offsets
                bnd2 = offsets[min(q + 2, nb)];
#else
            const uint32_t elast = e1 - 1;
            uint32_t v = sorted[e0], vn = sorted[min(e0 + 1, elast)];
            ring.gather(pts + (v & pmask), 0);
            for (uint32_t e = e0; e < e1; e++) {
                const uint32_t sl = (e - e0) & 1u;
                const Affine<F> qp = ring.template read<Affine<F>>(sl);
                const uint32_t cv = v;
                if (e == bnd) {  // before the gather (see the Fp2 branch)
                    range_store(acc, seg0 == e0, false, q, c, t, head, tail, S);
                    acc = inf_l<C>();
                    seg0 = e;
                    q++;
                    bnd = bnd2;
                    if (bnd == e) {
                        uint32_t b2;
                        do {
                            q++;
                            b2 = offsets[min(q + 1, nb)];
                        } while (b2 == e);
                        bnd = b2;
                    }
                }
                const uint32_t nidx = (e + 1 < e1) ? vn : v;
                ring.gather(pts + (nidx & pmask), sl ^ 1u);
                v = nidx;
                vn = sorted[min(e + 2, elast)];
                bnd2 = offsets[min(q + 2, nb)];
#endif
                if (skip_inf && qp.is_inf()) continue;
                const Fl<C> x = unpack_l<C>(qp.x);
                Fl<C> y = unpack_l<C>(qp.y);
                if (cv >> 31) y = sub_nn<2>(Fl<C>{}, y);
                xyzzl_madd(acc, x, y);
            }
            range_store(acc, seg0 == e0, true, q, c, t, head, tail, S);
            return;
        }
#if !GG_G1_PIPE  // default: 16-B entry chunks loaded every fourth step
        // A/B (round 5, profiles/r05_c_*): a loop with every load unconditional
        // and no wait on the fresh gather inside the step (GG_G1_PIPE=1) ran
        // 14.11-14.19 vs 13.98 ms per 2^24 launch: it loads an entry and a
        // bucket boundary every step, and the extra traffic costs more clock
        // (2.00 vs 2.03 GHz effective) than the overlap gains -- three waves
        // per SIMD (164 VGPRs) already hide the gather behind the other waves
        uint4 ch = chunk_ld(sorted, (e0 + 1) & ~3u);
        uint32_t v = sorted[e0], vn = (e0 + 1 < e1) ? chunk_at(ch, (e0 + 1) & 3u) : 0u;
        Affine<F> p = ld_pt<NT>(pts + (v & pmask));
        for (uint32_t e = e0; e < e1; e++) {
            Affine<F> qp = p;
            const uint32_t cv = v;
            if (e + 1 < e1) {
                p = ld_pt<NT>(pts + (vn & pmask));
                v = vn;
                if (e + 2 < e1) {
                    const uint32_t j = e + 2;
                    if ((j & 3u) == 0) ch = chunk_ld(sorted, j);
                    vn = chunk_at(ch, j & 3u);
                }
            }
            if (e == bnd) {
                range_store(acc, seg0 == e0, false, q, c, t, head, tail, S);
                acc = inf_l<C>();
                seg0 = e;
                do { q++; bnd = bnd2; bnd2 = offsets[min(q + 2, nb)]; } while (bnd == e);
            }
#else
        // A/B variant (GG_G1_PIPE=1): a software pipeline of distance one in
        // which the gather of point e + 1 is waited for only at the next step.
        // The VM counter is in order, so nothing the step needs may come from
        // a load issued after that gather, and every load is unconditional (a
        // load under a branch leaves its value in a register the loop copies:
        // a wait at the copy).  The default loop above waits for the fresh
        // gather inside the step (its chunk select) and is still as fast: the
        // other waves of the SIMD cover the wait.
        const uint32_t elast = e1 - 1;
        uint32_t v = sorted[e0], vn = sorted[min(e0 + 1, elast)];
        Affine<F> p = ld_pt<NT>(pts + (v & pmask));
        for (uint32_t e = e0; e < e1; e++) {
            Affine<F> qp = p;
            const uint32_t cv = v;
            // the last step re-gathers its own point (a valid index, unused)
            const uint32_t nidx = (e + 1 < e1) ? vn : v;
            p = ld_pt<NT>(pts + (nidx & pmask));
            v = nidx;
            vn = sorted[min(e + 2, elast)];
            if (e == bnd) {
                range_store(acc, seg0 == e0, false, q, c, t, head, tail, S);
                acc = inf_l<C>();
                seg0 = e;
                q++;
                bnd = bnd2;  // offsets[q + 1], loaded in an earlier step
                if (bnd == e) {  // a run of empty buckets: walk to the next boundary (rare)
                    uint32_t b2;
                    do {
                        q++;
                        b2 = offsets[min(q + 1, nb)];
                    } while (b2 == e);
                    bnd = b2;
                }
            }
            bnd2 = offsets[min(q + 2, nb)];
#endif
            if (skip_inf && qp.is_inf()) continue;
            const Fl<C> x = unpack_l<C>(qp.x);
            Fl<C> y = unpack_l<C>(qp.y);
            if (cv >> 31) y = sub_nn<2>(Fl<C>{}, y);  // 2p - y, limbs < 2^(B+1) (xyzzl_madd takes it)
            xyzzl_madd(acc, x, y);
        }
        range_store(acc, seg0 == e0, true, q, c, t, head, tail, S);
        return;
    }
    if constexpr (std::is_same<F, Fp2>::value) {
        // BN254 G2: radix-2^29 Fp2 accumulator (field29.cuh), base in x * 2^261 form.
        // The 128-B points do not fit a register prefetch at two waves per SIMD
        // (the adds use all 256 VGPRs), so the next point is gathered straight
        // into LDS (global_load_lds_dwordx4, no VGPRs): two 8-KB slots per wave,
        // [slot][16-B chunk][lane], the gather of point e + 1 issued after point
        // e has been read out of its slot.  The flush (which reads a boundary
        // loaded in an earlier step) comes before that gather: a use of an
        // ordinary load's value while an LDS DMA is in flight waits for the DMA.
#if GG_ACCUM_R4LOOP  // A/B build only: round 4's loop (no prefetch)
        Xyzz2_29 acc = inf2_29();
        uint2 ch = *reinterpret_cast<const uint2*>(sorted + (e0 & ~1u));
        for (uint32_t e = e0; e < e1; e++) {
            if (e == bnd) {
                range_store(acc, seg0 == e0, false, q, c, t, head, tail, S);
                acc = inf2_29();
                seg0 = e;
                do { q++; bnd = bnd2; bnd2 = offsets[min(q + 2, nb)]; } while (bnd == e);
            }
            if ((e & 1u) == 0 && e != e0) ch = *reinterpret_cast<const uint2*>(sorted + e);
            const uint32_t cv = (e & 1u) ? ch.y : ch.x;
            const Affine<F> pt = ld(pts + (cv & pmask));
#else
        extern __shared__ uint4 acc_lds[];
        const LdsRing<8> ring(acc_lds);
        Xyzz2_29 acc = inf2_29();
#if GG_RING_CHUNKS_G2
        EntryChunks ec(sorted, e0);
        uint32_t v = ec.c0.x, vn = ec.c0.y;
        ring.gather(pts + (v & pmask), 0);
        for (uint32_t i = 0;; i++) {
            const uint32_t e = e0 + i;
            if (e >= e1) break;
            const uint32_t s = i & 1u;
#else
        const uint32_t elast = e1 - 1;
        uint32_t v = sorted[e0], vn = sorted[min(e0 + 1, elast)];
        ring.gather(pts + (v & pmask), 0);
        for (uint32_t e = e0; e < e1; e++) {
            const uint32_t s = (e - e0) & 1u;
#endif
            const Affine<F> pt = ring.template read<Affine<F>>(s);
            const uint32_t cv = v;
            if (e == bnd) {
                range_store(acc, seg0 == e0, false, q, c, t, head, tail, S);
                acc = inf2_29();
                seg0 = e;
                q++;
                bnd = bnd2;  // offsets[q + 1], loaded in an earlier step
                if (bnd == e) {  // a run of empty buckets (rare)
                    uint32_t b2;
                    do {
                        q++;
                        b2 = offsets[min(q + 1, nb)];
                    } while (b2 == e);
                    bnd = b2;
                }
            }
#if GG_RING_CHUNKS_G2
            ec.advance(sorted, e0, i);
            const uint32_t nidx = (e + 1 < e1) ? vn : v;  // the last step re-gathers its own point
            ring.gather(pts + (nidx & pmask), s ^ 1u);
            v = nidx;
            vn = ec.next2(i);
#else
            const uint32_t nidx = (e + 1 < e1) ? vn : v;  // the last step re-gathers its own point
            ring.gather(pts + (nidx & pmask), s ^ 1u);
            v = nidx;
            vn = sorted[min(e + 2, elast)];
#endif
            bnd2 = offsets[min(q + 2, nb)];
#endif
            if (skip_inf && pt.is_inf()) continue;
            const Fp2_29 x{unpack29(pt.x.a0), unpack29(pt.x.a1)};
            Fp2_29 y{unpack29(pt.y.a0), unpack29(pt.y.a1)};
            if (cv >> 31) y = Fp2_29{sub<2>(Fp29{}, y.c0), sub<2>(Fp29{}, y.c1)};  // 2p - y
            xyzz2_29_madd(acc, x, y);
        }
        range_store(acc, seg0 == e0, true, q, c, t, head, tail, S);
        return;
    }
    if constexpr (std::is_same<typename PartialOf<F>::T, Xyzz<F>>::value) {  // gnark's form (BLS12-381 G2)
        Xyzz<F> acc = Xyzz<F>::inf();
        if constexpr (sizeof(F) <= 32) {
            // G1: software pipeline, the next point is in flight while this one is added
            uint32_t v = sorted[e0], vn = (e0 + 1 < e1) ? sorted[e0 + 1] : 0u;
            Affine<F> p = ld(pts + (v & pmask));
            for (uint32_t e = e0; e < e1; e++) {
                Affine<F> qp = p;
                const uint32_t cv = v;
                if (e + 1 < e1) {
                    p = ld(pts + (vn & pmask));
                    v = vn;
                    if (e + 2 < e1) vn = sorted[e + 2];
                }
                if (e == bnd) {  // bucket boundary: flush [seg0, e) of bucket q
                    range_store(acc, seg0 == e0, false, q, c, t, head, tail, S);
                    acc = Xyzz<F>::inf();
                    seg0 = e;
                    do { q++; bnd = bnd2; bnd2 = offsets[min(q + 2, nb)]; } while (bnd == e);
                }
                if (skip_inf && qp.is_inf()) continue;  // hole of a wire-indexed table
                if (cv >> 31) qp.y = -qp.y;
                xyzz_madd_inplace(acc, qp);
            }
        } else {
            // G2: no room for a second point in registers
            for (uint32_t e = e0; e < e1; e++) {
                if (e == bnd) {
                    range_store(acc, seg0 == e0, false, q, c, t, head, tail, S);
                    acc = Xyzz<F>::inf();
                    seg0 = e;
                    do { q++; bnd = bnd2; bnd2 = offsets[min(q + 2, nb)]; } while (bnd == e);
                }
                const uint32_t v = sorted[e];
                Affine<F> p = ld(pts + (v & pmask));
                if (skip_inf && p.is_inf()) continue;
                if (v >> 31) p.y = -p.y;
                xyzz_madd_inplace(acc, p);
            }
        }
        range_store(acc, seg0 == e0, true, q, c, t, head, tail, S);
    }
}

// ---- quad-cooperative XYZZ add (latency-bound tree levels) -----------------
// The four lanes of a quad (lanes 4j..4j+3 of a wave) hold the same p and q and
// compute p + q (add-2008-s) together: in each of four rounds every lane does
// one of the independent products and the quad swaps them through DPP
// quad_perm broadcasts.  The dependent chain is 4 products instead of the ~15
// one lane issues, which is what the reduction levels pay: there are few sums
// in flight there, so the chip is idle and a level lasts one add's latency.
template <int SRC, class T>
__device__ __forceinline__ T quad_bcast(const T& v) {
    static_assert(sizeof(T) % 4 == 0 && SRC >= 0 && SRC < 4, "word-sized, lane of a quad");
    T r;
    const int* s = reinterpret_cast<const int*>(&v);
    int* d = reinterpret_cast<int*>(&r);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++)
        d[i] = __builtin_amdgcn_mov_dpp(s[i], SRC * 0x55, 0xf, 0xf, false);  // quad_perm(S,S,S,S)
    return r;
}

template <class T>
__device__ __forceinline__ T sel4(uint32_t k, const T& a0, const T& a1, const T& a2, const T& a3) {
    T r;
    const uint32_t* w0 = reinterpret_cast<const uint32_t*>(&a0);
    const uint32_t* w1 = reinterpret_cast<const uint32_t*>(&a1);
    const uint32_t* w2 = reinterpret_cast<const uint32_t*>(&a2);
    const uint32_t* w3 = reinterpret_cast<const uint32_t*>(&a3);
    uint32_t* d = reinterpret_cast<uint32_t*>(&r);
    // masks, not a select of pointers: every word is loaded from all four
    // operands, which keeps them in registers (a pointer select forced them
    // into scratch)
    const uint32_t m0 = 0u - (k == 0), m1 = 0u - (k == 1), m2 = 0u - (k == 2), m3 = 0u - (k == 3);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++)
        d[i] = (w0[i] & m0) | (w1[i] & m1) | (w2[i] & m2) | (w3[i] & m3);
    return r;
}

// p += q on a quad; k = lane & 3.  p and q must be the same on the four lanes
// (then every branch is uniform over the quad and the result is too).
template <class F>
__device__ __forceinline__ void xyzz_add_quad(Xyzz<F>& p, const Xyzz<F>& q, uint32_t k) {
    if (q.is_inf()) return;
    if (p.is_inf()) {
        p = q;
        return;
    }
    F m = sel4(k, p.x, p.y, q.x, q.y) * sel4(k, q.zz, q.zzz, p.zz, p.zzz);
    const F U1 = quad_bcast<0>(m), S1 = quad_bcast<1>(m);
    const F P = quad_bcast<2>(m) - U1, R = quad_bcast<3>(m) - S1;
    if (P.is_zero()) {
        p = R.is_zero() ? xyzz_dbl(p) : Xyzz<F>::inf();
        return;
    }
    m = sel4(k, P, R, p.zz, p.zzz) * sel4(k, P, R, q.zz, q.zzz);
    const F PP = quad_bcast<0>(m), RR = quad_bcast<1>(m), Z2 = quad_bcast<2>(m), Z3 = quad_bcast<3>(m);
    m = sel4(k, P, U1, Z2, P) * PP;
    const F PPP = quad_bcast<0>(m), Q = quad_bcast<1>(m), ZZ3 = quad_bcast<2>(m);
    const F X3 = RR - PPP - dbl(Q);
    const F D = Q - X3;
    m = sel4(k, R, S1, Z3, R) * sel4(k, D, PPP, PPP, D);
    p.y = quad_bcast<0>(m) - quad_bcast<1>(m);
    p.zzz = quad_bcast<2>(m);
    p.x = X3;
    p.zz = ZZ3;
}

template <class T>
__device__ __forceinline__ T shfl_xor_words(const T& v, int mask) {
    static_assert(sizeof(T) % 4 == 0, "word-sized struct");
    T r;
    const int* s = reinterpret_cast<const int*>(&v);
    int* d = reinterpret_cast<int*>(&r);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++) d[i] = __shfl_xor(s[i], mask, 64);
    return r;
}

// Ranges [t0, t1] covering bucket q (sort order) of the balanced accumulation:
// the bucket's sum is X(t0) + head[t0+1] + ... + head[t1], where X(t0) is
// head[t0] if the bucket starts at t0's first entry, else tail[t0].
struct BucketSpan {
    uint32_t t0, t1;
    bool empty, first, direct;  // direct: a whole bucket inside one range, already in S
};
__device__ __forceinline__ BucketSpan bucket_span(const uint32_t* offsets, uint32_t q, uint32_t E, uint32_t K) {
    BucketSpan s{};
    const uint32_t o0 = offsets[q], o1 = offsets[q + 1];
    s.empty = o0 == o1;
    if (s.empty) return s;
    s.t0 = o0 / K;
    s.t1 = (o1 - 1) / K;
    s.first = o0 == s.t0 * K;
    const uint32_t end1 = (uint32_t)min<uint64_t>((uint64_t)(s.t1 + 1) * K, E);
    s.direct = s.t0 == s.t1 && !s.first && o1 != end1;
    return s;
}

// Heavy buckets (> LIGHT ranges, e.g. the digit-1 bucket of a 0/1-heavy
// witness): in-place segmented tree over head[t0+1 .. t1], one quad per slot;
// after the launches with stride 1, fan, fan^2, ... head[t0+1] holds the sum.
template <class F>
__global__ void __launch_bounds__(256) k_range_tree(Xyzz<F>* head, const uint32_t* tbucket,
                                                    const uint32_t* offsets, uint32_t nb, uint32_t K,
                                                    uint32_t stride, uint32_t fan) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = (uint32_t)g & 3;
    const size_t p = g >> 2;
    const uint32_t E = offsets[nb];
    if ((uint64_t)p * K >= E) return;  // every branch below is uniform over the quad
    const uint32_t q = tbucket[p];
    const BucketSpan s = bucket_span(offsets, q, E, K);
    const uint32_t m = s.t1 - s.t0;  // ranges after t0
    if (m <= LIGHT || p <= s.t0) return;
    const uint32_t j = (uint32_t)p - (s.t0 + 1);
    if (j % (fan * stride)) return;
    if (j + stride >= m) return;
    Xyzz<F> acc = ld(head + p);
    for (uint32_t k = 1; k < fan && j + k * stride < m; k++) xyzz_add_quad(acc, ld(head + p + k * stride), lane);
    if (lane == 0) st(head + p, acc);
}

// Level 2: one quad per bucket combines its ranges' partials into S in natural
// bucket order b = brev(q) (the sort order is pi(b) = bitrev_{c-1}(b)).
template <class F>
__global__ void __launch_bounds__(256) k_bucket_combine(const Xyzz<F>* head, const Xyzz<F>* tail,
                                                        const uint32_t* offsets, uint32_t nb, int c,
                                                        uint32_t K, Xyzz<F>* S) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = (uint32_t)g & 3;
    const size_t q = g >> 2;
    if (q >= nb) return;
    const uint32_t E = offsets[nb];
    const BucketSpan s = bucket_span(offsets, (uint32_t)q, E, K);
    Xyzz<F>* out = S + bucket_perm((uint32_t)q, c);
    if (s.empty) {
        if (lane == 0) st(out, Xyzz<F>::inf());
        return;
    }
    if (s.direct) return;
    Xyzz<F> acc = ld((s.first ? head : tail) + s.t0);
    const uint32_t m = s.t1 - s.t0;
    if (m > LIGHT) xyzz_add_quad(acc, ld(head + s.t0 + 1), lane);  // tree result
    else
        for (uint32_t t = s.t0 + 1; t <= s.t1; t++) xyzz_add_quad(acc, ld(head + t), lane);
    if (lane == 0) st(out, acc);
}

// k_bucket_combine over radix-form partials (round 6): each partial converted
// to gnark's form as it is loaded -- a direct bucket from SP, a straddling one
// from its ranges' heads / tail -- instead of three conversion launches over
// every head, tail and S slot before the combine (the small MSMs of the quad
// path: a PlonK part's slices, configs[1]'s 2^20 MSM).  The heavy buckets' tree
// runs before it on the radix heads (k_range_tree_r).
template <class F>
__global__ void __launch_bounds__(256) k_bucket_combine_r(const typename PartialOf<F>::T* headP,
                                                          const typename PartialOf<F>::T* tailP,
                                                          const typename PartialOf<F>::T* SP, const uint32_t* offsets,
                                                          uint32_t nb, int c, uint32_t K, Xyzz<F>* S) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = (uint32_t)g & 3;
    const size_t q = g >> 2;
    if (q >= nb) return;
    const uint32_t E = offsets[nb];
    const BucketSpan s = bucket_span(offsets, (uint32_t)q, E, K);
    const uint32_t pq = bucket_perm((uint32_t)q, c);
    Xyzz<F>* out = S + pq;
    if (s.empty) {
        if (lane == 0) st(out, Xyzz<F>::inf());
        return;
    }
    if (s.direct) {
        if (lane == 0) st(out, to_std(ld(SP + pq)));
        return;
    }
    Xyzz<F> acc = to_std(ld((s.first ? headP : tailP) + s.t0));
    const uint32_t m = s.t1 - s.t0;
    if (m > LIGHT) xyzz_add_quad(acc, to_std(ld(headP + s.t0 + 1)), lane);  // tree result
    else
        for (uint32_t t = s.t0 + 1; t <= s.t1; t++) xyzz_add_quad(acc, to_std(ld(headP + t)), lane);
    if (lane == 0) st(out, acc);
}

// k_range_tree over radix-form partials, a lane per slot (xyzzl_add)
template <class F>
__global__ void __launch_bounds__(256) k_range_tree_r(typename PartialOf<F>::T* head, const uint32_t* tbucket,
                                                      const uint32_t* offsets, uint32_t nb, uint32_t K,
                                                      uint32_t stride, uint32_t fan) {
    using O = PartialOps<F>;
    const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t E = offsets[nb];
    if ((uint64_t)p * K >= E) return;
    const BucketSpan s = bucket_span(offsets, tbucket[p], E, K);
    const uint32_t m = s.t1 - s.t0;
    if (m <= LIGHT || p <= s.t0) return;
    const uint32_t j = (uint32_t)p - (s.t0 + 1);
    if (j % (fan * stride) || j + stride >= m) return;
    typename O::T acc = ld(head + p);
    for (uint32_t k = 1; k < fan && j + k * stride < m; k++) acc = O::add(acc, ld(head + p + k * stride));
    st(head + p, acc);
}

// partials in the accumulator's form -> gnark's (for the quad-cooperative path)
template <class F>
__global__ void __launch_bounds__(256) k_partials_to_std(const typename PartialOf<F>::T* in, size_t n,
                                                         Xyzz<F>* out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) st(out + i, to_std(ld(in + i)));
}

// Level 2 and the weighted bucket sums in the reduced-radix form, for the
// groups that accumulate in it (BN254 / BLS12-381 G1): one lane per bucket or
// per segment (every lane busy) instead of quad-cooperative adds.
// k_bucket_sum_r: lane B (natural bucket id, all groups) forms the bucket's sum
// from its range partials as k_bucket_combine does (a direct bucket from S,
// else the first range's head or tail plus the later heads -- after
// k_range_tree for heavy buckets) and stores it in radix form, laid out
// [i][t] for bucket B = t L + i so that k_bucket_runsum's loads coalesce.
#ifndef GG_G2_SUM_WAVES
#define GG_G2_SUM_WAVES 1  // A/B builds: waves per SIMD of the BN254 G2 level 2 (2 spills)
#endif
template <class F>
constexpr int kSumWaves = std::is_same<F, Fp2>::value ? GG_G2_SUM_WAVES : 1;
template <class F>
__global__ void __launch_bounds__(256, kSumWaves<F>) k_bucket_sum_r(const typename PartialOf<F>::T* head,
                                                       const typename PartialOf<F>::T* tail,
                                                       const typename PartialOf<F>::T* S, const uint32_t* offsets,
                                                       uint32_t nb_total, int c, uint32_t K, int logL,
                                                       typename PartialOf<F>::T* Sr) {
    using O = PartialOps<F>;
    const uint32_t B = blockIdx.x * blockDim.x + threadIdx.x;
    if (B >= nb_total) return;
    const uint32_t nseg = nb_total >> logL;
    const BucketSpan sp = bucket_span(offsets, bucket_perm(B, c), offsets[nb_total], K);
    typename O::T acc = O::inf();
    if (!sp.empty) {
        acc = ld(sp.direct ? S + B : (sp.first ? head : tail) + sp.t0);
        const uint32_t rend = sp.direct ? sp.t0 : (sp.t1 - sp.t0 > LIGHT ? sp.t0 + 1 : sp.t1);  // heavy: tree result
        for (uint32_t r = sp.t0 + 1; r <= rend; r++) acc = O::add(acc, ld(head + r));
    }
    st(Sr + (size_t)(B & ((1u << logL) - 1)) * nseg + (B >> logL), acc);
}

// k_bucket_runsum: lane t walks the L buckets of segment t (group j = t / T)
// from the top, R = running sum, A = sum of the running sums =
// sum_i (i + 1) S_{tL+i}; then D_t = A - L R.  Writes D_t and R_t in gnark's
// form: the group's weighted sum is sum_t D_t + L sum_t (t + 1) R_t.  Every lane
// runs the same step sequence through ONE inlined add (the code of several
// would overflow the instruction cache): R += S_i, A += R (L times), R = 2R
// (log L times, after R is written out), A += -R.
template <class F>
__global__ void __launch_bounds__(256) k_bucket_runsum(const typename PartialOf<F>::T* Sr, uint32_t nseg, int logL,
                                                        Xyzz<F>* Dout, Xyzz<F>* Rout) {
    using O = PartialOps<F>;
    using T = typename O::T;
    // the next bucket's load in flight during the two adds -- not for the Fp2
    // points (288 B each), whose live set would spill
    constexpr bool kPf = !std::is_same<F, Fp2>::value;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg) return;
    const int L = 1 << logL, steps = 2 * L + logL + 1;
    T R = O::inf(), A = O::inf(), cur, nxt;
    if constexpr (kPf) nxt = ld(Sr + (size_t)(L - 1) * nseg + t);
    for (int k = 0; k < steps; k++) {
        T x, y;
        if (k < 2 * L) {
            const int i = L - 1 - (k >> 1);
            if (k & 1) {
                x = A;
                y = R;
            } else {
                if constexpr (kPf) {
                    cur = nxt;
                    if (i > 0) nxt = ld(Sr + (size_t)(i - 1) * nseg + t);
                } else {
                    cur = ld(Sr + (size_t)i * nseg + t);
                }
                x = R;
                y = cur;
            }
        } else {
            // R is final: written out, then doubled in place (X = L R)
            if (k == 2 * L) st(Rout + t, to_std(R));
            x = k < 2 * L + logL ? R : A;
            y = k < 2 * L + logL ? R : O::neg(R);
        }
        const T z = O::add(x, y);
        if (k < 2 * L) {
            if (k & 1) A = z;
            else R = z;
        } else if (k < 2 * L + logL) {
            R = z;
        } else {
            A = z;
        }
    }
    st(Dout + t, to_std(A));
}

// copy a list of small device arrays into one contiguous staging buffer
constexpr int MAX_GATHER = 192;
template <class F>
struct GatherList {
    const Xyzz<F>* src[MAX_GATHER];
    uint32_t off[MAX_GATHER + 1];
    int n;
};
template <class F>
__global__ void k_gather_items(GatherList<F> L, Xyzz<F>* out) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    int q = 0;
    while (q < L.n && t >= L.off[q + 1]) q++;
    if (q >= L.n) return;
    st(out + t, ld(L.src[q] + (t - L.off[q])));
}

// Generic strided group sum: view X[a][c] = in[a*sa + c*sb], a < A, c < Bc;
// out[a'*Bc + c] = sum_{k<G, a'G+k<A} X[a'G+k][c].  Several jobs per launch so
// independent reductions advance in lockstep (their latencies overlap).
template <class F>
struct RedJob {
    const Xyzz<F>* in;
    Xyzz<F>* out;
    uint32_t A, Bc, sa, sb, G, nthreads;
};
constexpr int MAX_RED_JOBS = 16;
template <class F>
struct RedJobs {
    RedJob<F> j[MAX_RED_JOBS];
    int n;
};

// One output per quad (xyzz_add_quad): launch 4 lanes per output.
template <class F>
__global__ void __launch_bounds__(256) k_reduce_jobs(RedJobs<F> J) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = g & 3;
    uint32_t t = g >> 2;
    int q = 0;
    while (q < J.n && t >= J.j[q].nthreads) { t -= J.j[q].nthreads; q++; }
    if (q >= J.n) return;  // uniform over the quad
    const RedJob<F>& jb = J.j[q];
    uint32_t a2 = t / jb.Bc, c = t % jb.Bc;
    uint32_t a0 = a2 * jb.G;
    uint32_t a1 = min(jb.A, a0 + jb.G);
    Xyzz<F> acc = ld(jb.in + (size_t)a0 * jb.sa + (size_t)c * jb.sb);
    for (uint32_t a = a0 + 1; a < a1; a++)
        xyzz_add_quad(acc, ld(jb.in + (size_t)a * jb.sa + (size_t)c * jb.sb), lane);
    if (lane == 0) st(jb.out + (size_t)a2 * jb.Bc + c, acc);
}

// Whole tree sums in one launch: block t of job q writes
// out[t] = sum_{a < A} in[a*sa + t*sb].  The block's NQ = blockDim/4 quads take
// a = quad, quad + NQ, ... with quad adds, then a log2(NQ)-level tree through LDS
// finishes it.  Replaces log2(A) lockstep launches of k_reduce_jobs (each level
// cost a launch plus one add's latency).
template <class F>
__global__ void __launch_bounds__(256) k_reduce_block(RedJobs<F> J) {
    __shared__ Xyzz<F> sh[32];
    uint32_t t = blockIdx.x;
    int q = 0;
    while (q < J.n && t >= J.j[q].nthreads) { t -= J.j[q].nthreads; q++; }
    if (q >= J.n) return;  // uniform over the block
    const RedJob<F>& jb = J.j[q];
    const uint32_t lane = threadIdx.x & 3, quad = threadIdx.x >> 2, NQ = blockDim.x >> 2;
    Xyzz<F> acc = Xyzz<F>::inf();
    for (uint32_t a = quad; a < jb.A; a += NQ)
        xyzz_add_quad(acc, ld(jb.in + (size_t)a * jb.sa + (size_t)t * jb.sb), lane);
    for (uint32_t h = NQ >> 1; h >= 1; h >>= 1) {
        if (quad >= h && quad < 2 * h && lane == 0) sh[quad - h] = acc;
        __syncthreads();
        if (quad < h) xyzz_add_quad(acc, sh[quad], lane);
        __syncthreads();
    }
    if (threadIdx.x == 0) st(jb.out + t, acc);
}

// ------------------------------------------------------------ precompute
template <class F>
__global__ void k_pre_init(const Affine<F>* in, size_t n, Affine<F>* out0, Xyzz<F>* cur) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Affine<F> p = ld(in + i);
    st(out0 + i, p);
    st(cur + i, Xyzz<F>::from_affine(p));  // infinity (0, 0) -> ZZ = ZZZ = 0
}

template <class F>
__global__ void __launch_bounds__(256) k_pre_dbl(Xyzz<F>* cur, size_t n, int c) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Xyzz<F> p = ld(cur + i);
    for (int k = 0; k < c; k++) p = xyzz_dbl(p);
    st(cur + i, p);
}


// batch-normalize XYZZ -> affine: thread t owns elements t, t+T, t+2T, ... (M of them)
template <class F>
__global__ void __launch_bounds__(256) k_pre_normalize(const Xyzz<F>* cur, size_t n, size_t T,
                                                       F* prefix, Affine<F>* out) {
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    // batch inversion of ZZZ along the thread's strided chain; infinity points
    // (ZZZ = 0) enter the product as 1 and come out as (0, 0)
    F acc = F::one();
    for (size_t i = t; i < n; i += T) {
        st(prefix + i, acc);
        F z = ld(cur + i).zzz;
        if (!z.is_zero()) acc = acc * z;
    }
    F inv = inverse(acc);
    size_t last = t + ((n - 1 - t) / T) * T;
    for (size_t i = last;; i -= T) {
        Xyzz<F> p = ld(cur + i);
        if (p.zzz.is_zero()) {
            st(out + i, Affine<F>::inf());
        } else {
            F izzz = inv * ld(prefix + i);  // 1/ZZZ_i
            inv = inv * p.zzz;
            F izz = sqr(izzz) * sqr(p.zz);  // lambda^-6 * lambda^4 = 1/ZZ
            st(out + i, Affine<F>{p.x * izz, p.y * izzz});
        }
        if (i < T) break;
    }
}

}  // namespace gg

using gg::DevBuf;
namespace gg {
// Sorted entries of one scalar vector over a base shape (n, c, W, scalar index
// map).  Bases with identical shapes can share one: the Groth16 prover sorts
// the wires once for A/K and once for B1/G2.
struct MsmSort {
    DevBuf sorted, counts, offsets, maxcnt;
    DevBuf keys, tmp_entry, tmp_key, hist, hoff, bin_start, seg2, chunk_start, chunk_hist, chunk_pos,
        chunk_desc;
    std::vector<DevBuf> scan_tmp;
    // Bucket stripe (multi-GPU split of one MSM by buckets): with
    // slog > 0 only the buckets b = 2^slog j + sres of every group are sorted,
    // renumbered j -- a c - slog bucket space -- and msm_finish returns
    // sum_b (b + 1) S_b over the stripe, so the 2^slog stripes' results add up
    // to the whole MSM.  Every stripe reads all scalars, but sorts, accumulates
    // and reduces only its 2^-slog share of the entries and buckets.
    int slog = 0;
    uint32_t sres = 0;
    // a batch of nvec scalar vectors (msm_prepare_batch): kp = the power of two
    // >= nvec copies of the bucket space, vector v in groups v G .. v G + G - 1
    int nvec = 1, kp = 1;
    uint32_t* pin = nullptr;          // pinned read-back: [0] = entries of the fullest bucket, [1] = entries
    hipEvent_t pin_ev = nullptr;      // after the read-back copy
    hipEvent_t ready_ev = nullptr;    // after the sort
    void ensure_events() {
        if (!pin) GG_HIP(hipHostMalloc((void**)&pin, 16, hipHostMallocDefault));
        if (!pin_ev) GG_HIP(hipEventCreateWithFlags(&pin_ev, hipEventDisableTiming));
        if (!ready_ev) GG_HIP(hipEventCreateWithFlags(&ready_ev, hipEventDisableTiming));
    }
    MsmSort() = default;
    MsmSort(const MsmSort&) = delete;
    MsmSort& operator=(const MsmSort&) = delete;
    ~MsmSort() {
        if (pin) (void)hipHostFree(pin);
        if (pin_ev) (void)hipEventDestroy(pin_ev);
        if (ready_ev) (void)hipEventDestroy(ready_ev);
    }
};
// Accumulation / reduction scratch of one MSM in flight: range partials
// (head, tail), range -> bucket map, dense bucket sums S, reduction arena.
struct MsmScratch {
    DevBuf head, tail, tbucket, S, arena, scal, seg;
    DevBuf headP, tailP, SP;  // partials in the accumulator's form (radix groups)
};
// Everything one MSM needs besides the (read-only) base: several MSMs over one
// base run concurrently on different streams with one MsmWork each.
struct MsmWork {
    MsmSort sort;
    MsmScratch scr;
};
}  // namespace gg

struct gg_msm_base {
    int group = GG_G1;
    size_t n = 0;  // resident points
    int c = 0, W = 0;
    gg::WinSpec win{};  // per-window bit widths / offsets
    // precompute groups (the memory knob, DESIGN.md "MSM"): only every G-th
    // window's shift 2^off(w) P is stored (Ws = ceil(W / G) copies); window
    // w = G w' + j reads copy w' and adds into bucket group j, whose sum is
    // scaled by 2^(j c) at the end.  G = 1: every window stored, one group.
    int G = 1, Ws = 0;
    size_t nb = 0;  // buckets over all groups: G 2^(c-1)
    DevBuf pts;   // Ws * n affine points, copy-major
    DevBuf sidx;  // n u32 or empty
    bool has_sidx = false;
    bool has_inf = false;  // wire-indexed table with infinity holes (skipped)
    int scurve = 0;        // scalar field: 0 = BN254 fr, 1 = BLS12-381 fr
    uint32_t max_sidx = 0;
    std::mutex mu;
    gg::MsmWork own;  // this base's sort + scratch (gg_msm, the Groth16 prover)
};

namespace gg {

template <class F>
inline void precompute(gg_msm_base* b, const Affine<F>* dev_in, hipStream_t st) {
    const size_t n = b->n;
    b->pts.alloc((size_t)b->Ws * n * sizeof(Affine<F>));
    Affine<F>* out = b->pts.as<Affine<F>>();
    DevBuf cur(n * sizeof(Xyzz<F>));
    // ~64 elements per thread amortise one Fermat inversion, >= 16K threads
    const size_t T = std::min<size_t>(n, std::max<size_t>(16384, n / 64));
    DevBuf prefix(n * sizeof(F));
    hipLaunchKernelGGL(k_pre_init<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, dev_in, n, out,
                       cur.as<Xyzz<F>>());
    GG_HIP(hipGetLastError());
    for (int w = 1; w < b->Ws; w++) {
        // copy w holds 2^off(G w) P: G windows of (uniform, when G > 1) width c on
        const int dbl = b->G == 1 ? (int)b->win.bits[w - 1] : b->G * b->c;
        hipLaunchKernelGGL(k_pre_dbl<F>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                           cur.as<Xyzz<F>>(), n, dbl);
        GG_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_pre_normalize<F>, dim3(grid_for(T, 256)), dim3(256), 0, st,
                           (const Xyzz<F>*)cur.p, n, T, prefix.as<F>(), out + (size_t)w * n);
        GG_HIP(hipGetLastError());
    }
    if constexpr (RadixOf<F>::on) {
        // the accumulation reads the points in its reduced-radix Montgomery
        // domain (field29.cuh): x R' mod p, same layout
        using C = typename RadixOf<F>::C;
        using E = Fe<typename C::Std>;
        const size_t total = (size_t)b->Ws * n * 2 * (sizeof(F) / sizeof(E));
        hipLaunchKernelGGL(k_to_radix<C>, dim3(grid_for(total, 256)), dim3(256), 0, st, (E*)out, total);
        GG_HIP(hipGetLastError());
    }
    GG_WAIT_STREAM(st);
}

// One term of a batched reduction: 2^mlog * sum_j (j + off) X_j over n = 2^k
// elements (weighted), or 2^mlog * sum_j X_j (plain).
template <class F>
struct RedItem {
    const Xyzz<F>* X;
    uint32_t n, off;
    int mlog;
    bool plain;
    int mult = 1;  // small signed factor of the whole term (bucket stripes), applied on the host
    int res = 0;   // which result the term adds to (a batch of MSMs: one per scalar vector)
};

// Sum of reduction terms with log-depth, wide tree sums (DESIGN.md "MSM /
// bucket reduction"): a weighted sum WS(X, off) = sum_j (j + off) X_j over
// n = 2^k elements is split as j = q*M + r into M * WS(H, 0) + WS(G, off) with
// row sums H_q and column sums G_r; a plain sum keeps its row sums.  Every
// round's jobs of every term go into the same launches (one add's latency per
// round for all of them), pieces of <= HOST_N elements finish on the host after
// ONE read-back, combined by Horner over their 2^mlog factors.
// Terms carry a result index (RedItem::res < nres): a batch's results come out of
// the same launches and the same read-back.
template <class F>
inline std::vector<Xyzz<F>> reduce_terms_multi(std::vector<RedItem<F>> items, int nres, MsmScratch* scr,
                                               hipStream_t st) {
    static const bool split = getenv("GG_RED_SPLIT") && atoi(getenv("GG_RED_SPLIT"));  // A/B: a read-back per term
    if (split && items.size() > 1) {
        std::vector<Xyzz<F>> acc(nres, Xyzz<F>::inf());
        for (const auto& it : items)
            acc[it.res] = xyzz_add(acc[it.res], reduce_terms_multi<F>({it}, nres, scr, st)[it.res]);
        return acc;
    }
    const size_t XB = sizeof(Xyzz<F>);
    size_t total = 0;
    for (const auto& it : items) total += it.n;
    const size_t arena_elems = 3 * total + 1024 * (items.size() + 1);
    scr->arena.reserve(arena_elems * XB);
    Xyzz<F>* arena = scr->arena.as<Xyzz<F>>();
    size_t used = 0;
    auto alloc = [&](size_t cnt) {
        GG_CHECK(used + cnt <= arena_elems, GG_ERR_INTERNAL, "bucket reduction arena overflow");
        Xyzz<F>* p = arena + used;
        used += cnt;
        return p;
    };
    using Item = RedItem<F>;
    struct Job { const Xyzz<F>* in; uint32_t A, Bc, sa, sb; Item dest; };
    std::vector<Item> host_items;
    uint32_t HOST_N = 8;  // weighted sums of <= HOST_N elements finish on the host (MI355X sweep: 8)
    if (const char* e = getenv("GG_RED_HOST_N")) HOST_N = (uint32_t)std::max(2, atoi(e));  // tuning
    while (!items.empty()) {
        std::vector<Job> jobs;
        for (const Item& it : items) {
            if (it.n <= HOST_N) { host_items.push_back(it); continue; }
            int lg = 31 - __builtin_clz(it.n);
            int mlg = lg / 2;
            uint32_t M = 1u << mlg, rows = it.n >> mlg;
            if (it.plain) {  // row sums only
                jobs.push_back({it.X, M, rows, 1u, M, Item{nullptr, rows, 0u, it.mlog, true, it.mult, it.res}});
                continue;
            }
            jobs.push_back({it.X, M, rows, 1u, M, Item{nullptr, rows, 0u, it.mlog + mlg, false, it.mult, it.res}});
            jobs.push_back({it.X, rows, M, M, 1u, Item{nullptr, M, it.off, it.mlog, false, it.mult, it.res}});
        }
        // one launch per round: every output of every job is a block-wide sum
        static const bool block_mode = !(getenv("GG_RED_BLOCK") && atoi(getenv("GG_RED_BLOCK")) == 0);
        if (block_mode && !jobs.empty()) {
            RedJobs<F> J;
            J.n = 0;
            size_t blocks = 0;
            uint32_t maxA = 1;
            auto flush = [&]() {
                if (!J.n) return;
                uint32_t nq = 1;
                while (nq < maxA && nq < 64) nq <<= 1;
                hipLaunchKernelGGL(k_reduce_block<F>, dim3((unsigned)blocks), dim3(4 * nq), 0, st, J);
                GG_HIP(hipGetLastError());
                J.n = 0;
                blocks = 0;
                maxA = 1;
            };
            for (auto& j : jobs) {
                Xyzz<F>* out = alloc(j.Bc);
                J.j[J.n++] = RedJob<F>{j.in, out, j.A, j.Bc, j.sa, j.sb, j.A, j.Bc};
                blocks += j.Bc;
                maxA = std::max(maxA, j.A);
                j.in = out;
                j.A = 1;
                j.sa = j.Bc;
                j.sb = 1;
                if (J.n == MAX_RED_JOBS) flush();
            }
            flush();
        }
        bool active = false;
        for (auto& j : jobs) if (j.A > 1) active = true;
        while (active) {
            size_t t2 = 0;
            for (auto& j : jobs) if (j.A > 1) t2 += (size_t)((j.A + 1) / 2) * j.Bc;
            uint32_t G = t2 >= (256u << 10) ? 8 : (t2 >= (96u << 10) ? 4 : 2);
            RedJobs<F> J;
            J.n = 0;
            size_t threads = 0;
            auto flush = [&]() {
                if (!J.n) return;
                hipLaunchKernelGGL(k_reduce_jobs<F>, dim3(grid_for(4 * threads, 256)), dim3(256), 0, st, J);
                GG_HIP(hipGetLastError());
                J.n = 0;
                threads = 0;
            };
            active = false;
            for (auto& j : jobs) {
                if (j.A <= 1) continue;
                uint32_t A2 = (j.A + G - 1) / G;
                Xyzz<F>* out = alloc((size_t)A2 * j.Bc);
                J.j[J.n++] = RedJob<F>{j.in, out, j.A, j.Bc, j.sa, j.sb, G, A2 * j.Bc};
                threads += (size_t)A2 * j.Bc;
                j.in = out;
                j.A = A2;
                j.sa = j.Bc;
                j.sb = 1;
                if (A2 > 1) active = true;
                if (J.n == MAX_RED_JOBS) flush();
            }
            flush();
        }
        std::vector<Item> next;
        for (auto& j : jobs) { Item it = j.dest; it.X = j.in; next.push_back(it); }
        items.swap(next);
    }
    // host: tiny weighted / plain sums + Horner over the 2^mlog factors
    GG_CHECK(host_items.size() <= (size_t)MAX_GATHER, GG_ERR_INTERNAL, "too many host reduction items");
    GatherList<F> GL;
    GL.n = (int)host_items.size();
    GL.off[0] = 0;
    for (size_t k = 0; k < host_items.size(); k++) {
        GL.src[k] = host_items[k].X;
        GL.off[k + 1] = GL.off[k] + host_items[k].n;
    }
    std::vector<Xyzz<F>> flat(GL.off[GL.n]);
    if (GL.n) {
        Xyzz<F>* stage = alloc(GL.off[GL.n]);
        hipLaunchKernelGGL(k_gather_items<F>, dim3(grid_for(GL.off[GL.n], 256)), dim3(256), 0, st, GL, stage);
        GG_HIP(hipGetLastError());
        GG_HIP(hipMemcpyAsync(flat.data(), stage, flat.size() * XB, hipMemcpyDeviceToHost, st));
    }
    GG_WAIT_STREAM(st);
    std::vector<std::vector<Xyzz<F>>> hx(host_items.size());
    for (size_t k = 0; k < host_items.size(); k++)
        hx[k].assign(flat.begin() + GL.off[k], flat.begin() + GL.off[k + 1]);
    std::vector<std::vector<std::pair<int, Xyzz<F>>>> vals(nres);
    auto scaled = [](const Xyzz<F>& v, int m) {  // m v by double-and-add (|m| small)
        if (m == 1 || v.is_inf()) return v;
        const uint32_t u = (uint32_t)(m < 0 ? -m : m);
        Xyzz<F> r = Xyzz<F>::inf();
        for (int bit = 31; bit >= 0; bit--) {
            if (!r.is_inf()) r = xyzz_dbl(r);
            if ((u >> bit) & 1u) r = xyzz_add(r, v);
        }
        if (m < 0 && !r.is_inf()) r.y = -r.y;
        return r;
    };
    // result r: its items' sums, then Horner over their 2^mlog factors (r06q: the
    // results of a batch finished side by side on kept workers measured neutral)
    auto finish = [&](int r) {
        auto& vr = vals[r];
        for (size_t k = 0; k < host_items.size(); k++) {
            if (host_items[k].res != r) continue;
            const auto& X = hx[k];
            Xyzz<F> run = Xyzz<F>::inf(), acc = Xyzz<F>::inf();
            if (host_items[k].plain) {
                for (const auto& x : X) acc = xyzz_add(acc, x);
                vr.push_back({host_items[k].mlog, scaled(acc, host_items[k].mult)});
                continue;
            }
            for (size_t j = X.size(); j-- > 1;) {
                run = xyzz_add(run, X[j]);
                acc = xyzz_add(acc, run);
            }
            if (host_items[k].off) {
                run = xyzz_add(run, X[0]);  // run = sum of all
                for (uint32_t o = 0; o < host_items[k].off; o++) acc = xyzz_add(acc, run);
            }
            vr.push_back({host_items[k].mlog, scaled(acc, host_items[k].mult)});
        }
        std::sort(vr.begin(), vr.end(), [](const auto& x, const auto& y) { return x.first > y.first; });
        Xyzz<F> acc = Xyzz<F>::inf();
        int cur = vr.empty() ? 0 : vr[0].first;
        for (auto& v : vr) {
            for (; cur > v.first; cur--) acc = acc.is_inf() ? acc : xyzz_dbl(acc);
            acc = xyzz_add(acc, v.second);
        }
        for (; cur > 0; cur--) acc = acc.is_inf() ? acc : xyzz_dbl(acc);
        return acc;
    };
    std::vector<Xyzz<F>> out(nres, Xyzz<F>::inf());
    for (int r = 0; r < nres; r++) out[r] = finish(r);
    return out;
}
template <class F>
inline Xyzz<F> reduce_terms(std::vector<RedItem<F>> items, MsmScratch* scr, hipStream_t st) {
    return reduce_terms_multi<F>(std::move(items), 1, scr, st)[0];
}

// level 2 + bucket reduction through k_bucket_sum_r / k_bucket_runsum (reduced-radix G1 groups);
// GG_MSM_SEGSUM=0 keeps k_bucket_combine + bucket_reduce_2d
template <class F>
constexpr bool kSegsumGroup = RadixOf<F>::on && (std::is_same<F, Fp>::value || std::is_same<F, FpBls>::value ||
                                                   std::is_same<F, Fp2>::value);
inline bool segsum_enabled() {
    const char* e = getenv("GG_MSM_SEGSUM");  // per MSM: tests switch it
    return !(e && atoi(e) == 0);
}
// GG_MSM_COMBINE_FUSED=0: the quad path converts every partial in three launches
// before k_bucket_combine (A/B; per MSM: tests switch it)
inline bool combine_fused() {
    const char* e = getenv("GG_MSM_COMBINE_FUSED");
    return !(e && atoi(e) == 0);
}


// Entries per accumulation range (one thread each).  Every range costs the same,
// so the grid runs in whole "rounds" of the chip's concurrent threads C (occupancy
// of k_accum_range<F> x CUs x 256): R = entries / (C K_pref) rounds, rounded, and
// K = entries / (R C) -- no half-empty last round.  K_pref: 32 below 4M entries,
// 64, 128 from 2^26 (MI355X sweeps: 2^20 G1 best at 64-80, 2^24 at 128; longer
// ranges mean fewer level-2 partials).  GG_MSM_K1 overrides.
template <class F>
inline uint32_t range_length(size_t E) {
    if (const char* e = getenv("GG_MSM_K1")) return (uint32_t)std::max(1, atoi(e));
    static const double C = [] {
        int blocks = 0, cus = 0, dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_accum_range<F, false>, 256, kAccumLds<F>) != hipSuccess ||
            blocks < 1 || cus < 1) {
            (void)hipGetLastError();
            return 256.0 * 256 * 2;
        }
        return (double)blocks * cus * 256;
    }();
    const double kpref = E < ((size_t)4 << 20) ? 32 : (E >= ((size_t)1 << 26) ? 128 : 64);
    const double rounds = std::max(1.0, std::round((double)E / (C * kpref)));
    return (uint32_t)std::max(1.0, std::ceil((double)E / (rounds * C)));
}

// Accumulation + reduction of base b over a prepared sort s (its own or one
// shared with a base of identical shape), scratch scr.  Waits (device side) for
// s->ready_ev.  A batch sort (s->nvec vectors) gives one result per vector in
// out[0 .. nvec): one accumulation launch, one level 2, one reduction -- the
// vectors' buckets are groups v G .. v G + G - 1 of a kp times larger space.
template <class F>
inline void msm_finish_multi(gg_msm_base* b, MsmSort* s, MsmScratch* scr, hipStream_t st, Xyzz<F>* out) {
    // a bucket stripe (s->slog > 0) works in its c - slog bucket space: nb and ce
    // below; the group scales 2^(j c) keep the base's c
    const int slog = s->slog, nvec = s->nvec, kp = s->kp;
    const size_t n = b->n, nb = (b->nb >> slog) * (size_t)kp;
    const int ce = b->c - slog;
    const int Gb = b->G, Ge = b->G * kp;  // the base's groups, the batch's
    for (int v = 0; v < nvec; v++) out[v] = Xyzz<F>::inf();
    if (n == 0) return;
    GG_HIP(hipStreamWaitEvent(st, s->ready_ev, 0));
    const uint32_t* offs = s->offsets.as<uint32_t>();
    size_t E = (size_t)b->W * n * (size_t)nvec;  // entries (upper bound: digit-0 entries are not sorted)
    if (slog) {
        // a stripe holds ~2^-slog of the entries: wait for the sort's count so
        // the ranges fill the chip for the entries there are
        GG_WAIT_EVENT(s->pin_ev);
        E = std::max<size_t>(s->pin[1], 1);
    }
    uint32_t K = range_length<F>(E);
    // the LDS-ring loops read their entries in aligned 16-B chunks (EntryChunks)
    if constexpr (kLdsGather<F>)
        if ((std::is_same<F, Fp2>::value ? GG_RING_CHUNKS_G2 : GG_RING_CHUNKS) != 0) K = (K + 3u) & ~3u;
    const size_t T = (E + K - 1) / K;  // ranges
    using PT = typename PartialOf<F>::T;
    constexpr bool kRadixP = !std::is_same<PT, Xyzz<F>>::value;  // partials in the accumulator's form
    scr->head.reserve((T + 1) * sizeof(Xyzz<F>));
    scr->tail.reserve((T + 1) * sizeof(Xyzz<F>));
    scr->tbucket.reserve((T + 1) * 4);
    scr->S.reserve(nb * sizeof(Xyzz<F>));
    Xyzz<F>* head = scr->head.as<Xyzz<F>>();
    Xyzz<F>* S = scr->S.as<Xyzz<F>>();
    PT *hP = (PT*)head, *tP = scr->tail.as<PT>(), *SP = (PT*)S;
    if constexpr (kRadixP) {
        scr->headP.reserve((T + 1) * sizeof(PT));
        scr->tailP.reserve((T + 1) * sizeof(PT));
        scr->SP.reserve(nb * sizeof(PT));
        hP = scr->headP.as<PT>();
        tP = scr->tailP.as<PT>();
        SP = scr->SP.as<PT>();
    }
    {
        // per-group names: the Groth16 prove runs G1 and G2 accumulations at once
        const char* acc_name = sizeof(F) == sizeof(Fp) ? "msm_accum" : (sizeof(F) == sizeof(Fp2) ? "msm_accum_g2" : "msm_accum_bls");
        ProfScope ps_acc(acc_name, st, (double)n);
        // A probe BUILD (-DGG_ACCUM_PROBE=1, traffic attribution only, wrong sums;
        // never an environment switch of the product library): every entry reads
        // one of the first <= 1024 points, so HBM sees everything but the point
        // gathers.  Such a library refuses proofs (gg_build_flags, capi.hip).
        uint32_t pmask = 0x7fffffffu;
        if (kAccumProbe) {
            pmask = 1023u;
            while (pmask && pmask >= n) pmask >>= 1;  // stay inside the base
        }
        // the nontemporal hint on the BN254 G1 register path, for big tables (above)
        static const double nt_min = [] {
            const char* e = getenv("GG_ACCUM_NT_GB");
            return 1e9 * (e ? atof(e) : 4.0);
        }();
        const bool nt = !kLdsGather<F> && (GG_PT_NT == 2 || (GG_PT_NT == 1 && std::is_same<F, Fp>::value &&
                                                              (double)b->pts.bytes >= nt_min));
        auto* const accum = nt ? &k_accum_range<F, true> : &k_accum_range<F, false>;
        hipLaunchKernelGGL(accum, dim3(grid_for(T, 256)), dim3(256), kAccumLds<F>, st,
                           (const Affine<F>*)b->pts.p,
                           s->sorted.as<uint32_t>(), offs, (uint32_t)nb, ce, K, (int)b->has_inf, hP, tP, SP,
                           scr->tbucket.as<uint32_t>(), pmask);
        GG_HIP(hipGetLastError());
        ps_acc.stop(st);
    }
    GG_WAIT_EVENT(s->pin_ev);
    const uint32_t maxcnt = s->pin[0];
    // ranges after the first one of the fullest bucket (upper bound)
    const uint32_t max_ranges = maxcnt / K + 1;
    // ---- level 2: heavy buckets' ranges by a segmented tree (skew-robust,
    // log_fan(ranges) launches), then every bucket's partials into S
    ProfScope ps_acc2("msm_accum2", st, (double)n);
    const size_t nbg = nb / (size_t)Ge;
    // segments of L = 2^logL buckets, >= 2^17 of them per group (a lane each:
    // fewer leave the chip idle while each lane walks its chain); below 2^18
    // buckets per group the quad path is faster (MI355X: 2^20 MSM, c = 17)
    // groups of 2^17 buckets take the segment path too, with L = 2 (the B1 / G2
    // MSMs of a 2^21-wire key shard; the 8-way 2^24 shard alone, alternating
    // A/B: 18.62 / 18.26 vs 19.11 / 18.04 ms, profiles/r03_af_*; 2^16 .. 2^18:
    // 18.20 / 18.08 vs 18.57 / 18.63, r03_ae_*); the 2^20 MSM's 2^16 buckets
    // stay on the quad path.  GG_MSM_SEGSUM_MINLOG=k moves the threshold
    static const int seg_minlog = [] {
        const char* e = getenv("GG_MSM_SEGSUM_MINLOG");
        return e ? std::max(8, std::min(18, atoi(e))) : 17;
    }();
    // GG_MSM_SEGS_LOG=s: segments per group >= 2^s (default 17) where L > 2
    static const int segs_log = [] {
        const char* e = getenv("GG_MSM_SEGS_LOG");
        return e ? std::max(12, std::min(20, atoi(e))) : 17;
    }();
    const int lgb = 31 - __builtin_clz((unsigned)std::max<size_t>(nbg, 1));
    const int logL = lgb >= segs_log + 1 ? std::min(4, lgb - segs_log) : (lgb >= seg_minlog ? 1 : 0);
    if constexpr (kSegsumGroup<F>) {
        if (segsum_enabled() && logL >= 1) {
            // level 2 and the weighted sums in radix form, a lane per bucket / segment
            for (uint32_t stride = 1; max_ranges > LIGHT && stride < max_ranges;) {
                const uint32_t fan = (stride == 1) ? 4u : 2u;
                hipLaunchKernelGGL(k_range_tree_r<F>, dim3(grid_for(T, 256)), dim3(256), 0, st, hP,
                                   (const uint32_t*)scr->tbucket.p, offs, (uint32_t)nb, K, stride, fan);
                GG_HIP(hipGetLastError());
                stride *= fan;
            }
            const uint32_t Tg = (uint32_t)(nbg >> logL), G = (uint32_t)Ge;
            scr->seg.reserve(2 * (size_t)G * Tg * sizeof(Xyzz<F>) + nb * sizeof(PT));
            Xyzz<F>* D = scr->seg.as<Xyzz<F>>();
            Xyzz<F>* Rs = D + (size_t)G * Tg;
            PT* Sr = reinterpret_cast<PT*>(Rs + (size_t)G * Tg);
            // (r06r: this level 2 split into a copy pass that lists the buckets
            // straddling a range boundary and an add pass over the list measured
            // slower -- the adds of those buckets are the kernel's time either way)
            hipLaunchKernelGGL(k_bucket_sum_r<F>, dim3(grid_for(nb, 256)), dim3(256), 0, st, (const PT*)hP,
                               (const PT*)tP, (const PT*)SP, offs, (uint32_t)nb, ce, K, logL, Sr);
            GG_HIP(hipGetLastError());
            hipLaunchKernelGGL(k_bucket_runsum<F>, dim3(grid_for((size_t)G * Tg, 256)), dim3(256), 0, st,
                               (const PT*)Sr, (uint32_t)(G * Tg), logL, D, Rs);
            GG_HIP(hipGetLastError());
            ps_acc2.stop(st);
            ProfScope ps_red("msm_reduce", st, (double)nb);
            // sum_j 2^(j c) (sum_s D_s + L sum_s (s + 1) R_s) over the groups j:
            // every group's two lists reduced in the same launches, one read-back
            // A stripe's buckets are b = 2^slog j + sres (j its dense id), so
            // sum_b (b + 1) S_b = 2^slog sum_j (j + 1) T_j - (2^slog - 1 - sres) sum_j T_j,
            // and sum_j T_j = sum_s R_s.
            const int sneg = slog ? -(int)((1u << slog) - 1u - s->sres) : 0;
            std::vector<RedItem<F>> terms;
            for (int jg = 0; jg < nvec * Gb; jg++) {
                const int j = jg % Gb, v = jg / Gb;  // group j of vector v
                terms.push_back({(const Xyzz<F>*)Rs + (size_t)jg * Tg, Tg, 1u, j * b->c + logL + slog, false, 1, v});
                terms.push_back({(const Xyzz<F>*)D + (size_t)jg * Tg, Tg, 0u, j * b->c + slog, true, 1, v});
                if (sneg) terms.push_back({(const Xyzz<F>*)Rs + (size_t)jg * Tg, Tg, 0u, j * b->c, true, sneg, v});
            }
            const std::vector<Xyzz<F>> res = reduce_terms_multi<F>(std::move(terms), nvec, scr, st);
            for (int v = 0; v < nvec; v++) out[v] = res[v];
            ps_red.stop(st);
            return;
        }
    }
    bool combined = false;
    if constexpr (kRadixP) {
        if (combine_fused()) {  // the quad path's conversions inside the combine (k_bucket_combine_r)
            for (uint32_t stride = 1; max_ranges > LIGHT && stride < max_ranges;) {
                const uint32_t fan = (stride == 1) ? 4u : 2u;
                hipLaunchKernelGGL(k_range_tree_r<F>, dim3(grid_for(T, 256)), dim3(256), 0, st, hP,
                                   (const uint32_t*)scr->tbucket.p, offs, (uint32_t)nb, K, stride, fan);
                GG_HIP(hipGetLastError());
                stride *= fan;
            }
            hipLaunchKernelGGL(k_bucket_combine_r<F>, dim3(grid_for(4 * nb, 256)), dim3(256), 0, st, (const PT*)hP,
                               (const PT*)tP, (const PT*)SP, offs, (uint32_t)nb, ce, K, S);
            GG_HIP(hipGetLastError());
            combined = true;
        } else {  // the quad path works on gnark's form
            hipLaunchKernelGGL(k_partials_to_std<F>, dim3(grid_for(T + 1, 256)), dim3(256), 0, st, (const PT*)hP,
                               T + 1, head);
            hipLaunchKernelGGL(k_partials_to_std<F>, dim3(grid_for(T + 1, 256)), dim3(256), 0, st, (const PT*)tP,
                               T + 1, scr->tail.as<Xyzz<F>>());
            hipLaunchKernelGGL(k_partials_to_std<F>, dim3(grid_for(nb, 256)), dim3(256), 0, st, (const PT*)SP, nb, S);
            GG_HIP(hipGetLastError());
        }
    }
    if (!combined) {
        for (uint32_t stride = 1; max_ranges > LIGHT && stride < max_ranges;) {
            const uint32_t fan = (stride == 1) ? 4u : 2u;
            hipLaunchKernelGGL(k_range_tree<F>, dim3(grid_for(4 * T, 256)), dim3(256), 0, st, head,
                               (const uint32_t*)scr->tbucket.p, offs, (uint32_t)nb, K, stride, fan);
            GG_HIP(hipGetLastError());
            stride *= fan;
        }
        hipLaunchKernelGGL(k_bucket_combine<F>, dim3(grid_for(4 * nb, 256)), dim3(256), 0, st, (const Xyzz<F>*)head,
                           (const Xyzz<F>*)scr->tail.p, offs, (uint32_t)nb, ce, K, S);
        GG_HIP(hipGetLastError());
    }
    ps_acc2.stop(st);
    // ---- bucket reduction: sum_b (b+1) S_b
    ProfScope ps_red("msm_reduce", st, (double)nb);
    // one weighted sum per precompute group, sum_j 2^(j c) R_j, in one batched reduction
    const int sneg = slog ? -(int)((1u << slog) - 1u - s->sres) : 0;  // bucket stripe, as above
    std::vector<RedItem<F>> terms;
    for (int jg = 0; jg < nvec * Gb; jg++) {
        const int j = jg % Gb, v = jg / Gb;
        const Xyzz<F>* Sj = (const Xyzz<F>*)S + (size_t)jg * nbg;
        terms.push_back({Sj, (uint32_t)nbg, 1u, j * b->c + slog, false, 1, v});
        if (sneg) terms.push_back({Sj, (uint32_t)nbg, 0u, j * b->c, true, sneg, v});
    }
    const std::vector<Xyzz<F>> res = reduce_terms_multi<F>(std::move(terms), nvec, scr, st);
    for (int v = 0; v < nvec; v++) out[v] = res[v];
    ps_red.stop(st);
}

template <class F>
inline Xyzz<F> msm_finish(gg_msm_base* b, MsmSort* s, MsmScratch* scr, hipStream_t st) {
    GG_CHECK(s->nvec == 1, GG_ERR_INTERNAL, "msm_finish of a batch sort");
    Xyzz<F> r;
    msm_finish_multi<F>(b, s, scr, st, &r);
    return r;
}

template <class F>
inline Xyzz<F> msm_run(gg_msm_base* b, MsmWork* w, const Fr* scalars_dev, hipStream_t st) {
    if (b->n == 0) return Xyzz<F>::inf();
    msm_prepare(b, &w->sort, scalars_dev, st);
    return msm_finish<F>(b, &w->sort, &w->scr, st);
}

// nvec MSMs over one base (same points, different scalars) as one: one sort, one
// accumulation launch, one level 2 and one bucket reduction (msm_prepare_batch)
template <class F>
inline void msm_run_batch(gg_msm_base* b, MsmWork* w, const VecPtrs& vp, int nvec, hipStream_t st, Xyzz<F>* out) {
    if (b->n == 0) {
        for (int v = 0; v < nvec; v++) out[v] = Xyzz<F>::inf();
        return;
    }
    msm_prepare_batch(b, &w->sort, vp, nvec, st);
    msm_finish_multi<F>(b, &w->sort, &w->scr, st, out);
}

// device-resident points: keep[i] = point i is not infinity (or keep_inf)
template <class F>
__global__ void k_base_keep(const Affine<F>* pts, size_t n, int keep_inf, uint32_t* keep, uint32_t* any_inf) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const bool inf = pts[i].is_inf();
    if (inf) *any_inf = 1u;
    keep[i] = (!inf || keep_inf) ? 1u : 0u;
}
template <class F>
__global__ void k_base_compact(const Affine<F>* pts, size_t n, const uint32_t* keep, const uint32_t* pos,
                               Affine<F>* out, uint32_t* idx) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !keep[i]) return;
    out[pos[i]] = pts[i];
    idx[pos[i]] = (uint32_t)i;
}

// groups: precompute groups G (power of two), 0 = choose from free HBM
// (choose_groups: the smallest G whose table fits)
template <class F>
inline void window_layout(gg_msm_base* b, int window_bits, int total, int groups) {
    const size_t pb = sizeof(Affine<F>);
    b->c = window_bits ? window_bits : choose_c(std::max<size_t>(b->n, 1), pb, total);
    GG_CHECK(b->c >= 2 && b->c <= 24, GG_ERR_INVALID_ARG, "window_bits out of range [2, 24]");
    b->W = (total + b->c - 1) / b->c;
    b->c = (total + b->W - 1) / b->W;  // widest balanced window for this W
    GG_CHECK(b->W <= 64, GG_ERR_INVALID_ARG, "too many windows");
    if (groups == 0) groups = choose_groups((double)b->W * (double)b->n * (double)pb, 0.0, b->W);
    GG_CHECK(groups >= 1 && groups <= 16 && (groups & (groups - 1)) == 0, GG_ERR_INVALID_ARG,
             "precompute groups must be 1, 2, 4, 8 or 16");
    b->G = std::min(groups, 1 << (31 - __builtin_clz((unsigned)b->W)));  // at most W groups
    b->Ws = (b->W + b->G - 1) / b->G;
    if (b->G == 1) {
        b->win = make_windows(b->c, b->W, total);
    } else {  // uniform widths: window G w' + j sits j c bits above copy w'
        for (int w = 0; w < b->W; w++) {
            b->win.bits[w] = (uint8_t)b->c;
            b->win.off[w] = (uint8_t)(w * b->c);
        }
    }
    b->nb = (size_t)b->G << (b->c - 1);
    GG_CHECK(b->nb < ((size_t)1 << 30), GG_ERR_UNSUPPORTED, "too many buckets");
    GG_CHECK((double)b->W * (double)b->n < 2147483648.0, GG_ERR_UNSUPPORTED,
             "too many points x windows for 31-bit entry ids");
}

// points already in HBM (no scalar index map): infinity points dropped by a
// flag / scan / scatter on the device, no round trip through host memory
template <class F>
inline void create_base_dev(gg_msm_base* b, const Affine<F>* pts, size_t n, int window_bits, bool keep_inf,
                            int total, int groups) {
    hipStream_t st = hipStreamPerThread;
    DevBuf keep(std::max<size_t>(n, 1) * 4), pos(std::max<size_t>(n, 1) * 4), flag(16);
    GG_HIP(hipMemsetAsync(flag.p, 0, 4, st));
    hipLaunchKernelGGL(k_base_keep<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, pts, n, (int)keep_inf,
                       keep.as<uint32_t>(), flag.as<uint32_t>());
    GG_HIP(hipGetLastError());
    std::vector<DevBuf> tmp;
    exclusive_scan(keep.as<uint32_t>(), pos.as<uint32_t>(), n, st, tmp);
    uint32_t last_pos = 0, last_keep = 0, any_inf = 0;
    GG_HIP(hipMemcpyAsync(&last_pos, pos.as<uint32_t>() + (n - 1), 4, hipMemcpyDeviceToHost, st));
    GG_HIP(hipMemcpyAsync(&last_keep, keep.as<uint32_t>() + (n - 1), 4, hipMemcpyDeviceToHost, st));
    GG_HIP(hipMemcpyAsync(&any_inf, flag.p, 4, hipMemcpyDeviceToHost, st));
    GG_WAIT_STREAM(st);
    const size_t kept = (size_t)last_pos + last_keep;
    b->n = kept;
    b->has_inf = keep_inf && any_inf;
    const bool dropped = kept < n;
    b->has_sidx = dropped;
    window_layout<F>(b, window_bits, total, groups);
    if (!kept) {
        b->max_sidx = 0;
        if (dropped) b->sidx.alloc(4);
        return;
    }
    DevBuf cmp(kept * sizeof(Affine<F>)), idx(kept * 4);
    hipLaunchKernelGGL(k_base_compact<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, pts, n, keep.as<uint32_t>(),
                       pos.as<uint32_t>(), cmp.as<Affine<F>>(), idx.as<uint32_t>());
    GG_HIP(hipGetLastError());
    uint32_t max_idx = 0;  // indices increase: the last kept one is the largest
    GG_HIP(hipMemcpyAsync(&max_idx, idx.as<uint32_t>() + (kept - 1), 4, hipMemcpyDeviceToHost, st));
    GG_WAIT_STREAM(st);
    b->max_sidx = max_idx;
    if (dropped) b->sidx = std::move(idx);
    precompute<F>(b, cmp.as<Affine<F>>(), st);
}

template <class F>
inline void create_base(gg_msm_base* b, const void* points, size_t n, int on_device,
                        const uint32_t* sidx, int window_bits, bool keep_inf = false,
                        int scurve = 0, int groups = 0) {
    b->scurve = scurve;
    const int total = scalar_total_bits(scurve);
    const size_t pb = sizeof(Affine<F>);
    if (on_device && !sidx && n) {
        create_base_dev<F>(b, (const Affine<F>*)points, n, window_bits, keep_inf, total, groups);
        return;
    }
    std::vector<uint8_t> host;
    const uint8_t* src;
    if (on_device) {  // with a caller's scalar index map: compact on the host
        host.resize(n * pb);
        if (n) GG_HIP(hipMemcpy(host.data(), points, n * pb, hipMemcpyDeviceToHost));
        src = host.data();
    } else {
        src = (const uint8_t*)points;
    }
    // drop infinity points, build the scalar index map (keep_inf: a wire-indexed
    // table whose infinity holes stay in place and are skipped when summing)
    std::vector<uint8_t> keep;
    keep.reserve(n * pb);
    std::vector<uint32_t> idx;
    idx.reserve(n);
    bool dropped = false;
    static const uint8_t zero[128] = {0};
    for (size_t i = 0; i < n; i++) {
        const uint8_t* p = src + i * pb;
        if (memcmp(p, zero, pb) == 0) {
            if (keep_inf) b->has_inf = true;
            else { dropped = true; continue; }
        }
        keep.insert(keep.end(), p, p + pb);
        idx.push_back(sidx ? sidx[i] : (uint32_t)i);
    }
    b->n = idx.size();
    b->has_sidx = dropped || sidx != nullptr;
    b->max_sidx = 0;
    for (uint32_t v : idx) b->max_sidx = std::max(b->max_sidx, v);
    window_layout<F>(b, window_bits, total, groups);
    if (b->has_sidx) {
        b->sidx.alloc(std::max<size_t>(b->n, 1) * 4);
        if (b->n) GG_HIP(hipMemcpy(b->sidx.p, idx.data(), b->n * 4, hipMemcpyHostToDevice));
    }
    if (b->n == 0) return;
    DevBuf tmp(b->n * pb);
    GG_HIP(hipMemcpy(tmp.p, keep.data(), b->n * pb, hipMemcpyHostToDevice));
    precompute<F>(b, tmp.as<Affine<F>>(), hipStreamPerThread);
}

}  // namespace gg

