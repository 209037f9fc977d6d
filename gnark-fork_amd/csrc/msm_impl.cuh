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
#include "prof.h"
#include <mutex>
#include <vector>
#include <algorithm>
#include <memory>
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
__global__ void k_set_total_max(uint32_t* out, const uint32_t* in, size_t n, const uint32_t* maxcnt);
__global__ void k_item_counts(const uint32_t* offsets, size_t nb, int K, uint32_t* itemcnt,
                              uint32_t* maxcnt);
__global__ void k_item_buckets(const uint32_t* item_off, size_t nb, const uint32_t* n_items_dev,
                               uint32_t* item_bucket);
void exclusive_scan(const uint32_t* in, uint32_t* out, size_t n, hipStream_t st,
                    std::vector<DevBuf>& tmp, int depth = 0);
int choose_c(size_t n, size_t point_bytes, int total_bits = 255);
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
void sort_entries(const gg_msm_base* b, MsmSort* s, const Fr* scalars_dev, hipStream_t st);
void msm_prepare(const gg_msm_base* b, MsmSort* s, const Fr* scalars_dev, hipStream_t st);

constexpr uint32_t LIGHT = 16;  // buckets with <= LIGHT items: merged inside the accumulation block
// In-block merge of light buckets' partials inside k_accum_affine: measured
// slower on MI355X (the end-of-block tree is latency-bound: 2^20 accumulation
// 1.45 -> 1.70 ms vs 0.11 ms for k_bucket_sum), so it is off for both groups.
template <class F>
constexpr bool kMergeInBlock = false;

// level 1: sum up to K affine points of one bucket into an XYZZ partial, then
// merge the partials of light buckets inside the block (LDS tree, <= 4 steps):
// afterwards a light bucket's sum is part[item_off[b]] (+ part[next 256-item
// block start] if the bucket straddles one).  Heavy buckets keep one partial per
// item for k_seg_tree.  n_items is read from the device (no host sync).
template <class F>
__global__ void __launch_bounds__(256, 2) k_accum_affine(const Affine<F>* pts, const uint32_t* sorted,
                                                      const uint32_t* offsets,
                                                      const uint32_t* item_off,
                                                      const uint32_t* item_bucket,
                                                      const uint32_t* n_items_dev, int K,
                                                      int skip_inf, Xyzz<F>* partial) {
    extern __shared__ __attribute__((aligned(16))) unsigned char acc_lds[];
    [[maybe_unused]] Xyzz<F>* sh = reinterpret_cast<Xyzz<F>*>(acc_lds);
    const size_t n_items = *n_items_dev;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((size_t)blockIdx.x * blockDim.x >= n_items) return;  // whole block past the end
    const bool valid = t < n_items;
    Xyzz<F> acc = Xyzz<F>::inf();
    uint32_t io0 = 0, io1 = 0;
    if (valid) {
    uint32_t b = item_bucket[t];
    io0 = item_off[b];
    io1 = item_off[b + 1];
    uint32_t j = (uint32_t)t - io0;
    // bucket b (cnt entries) is cut into m = ceil(cnt / K) near-equal items
    const uint32_t o = offsets[b], cnt = offsets[b + 1] - o;
    const uint32_t m = (cnt + (uint32_t)K - 1) / (uint32_t)K;
    const uint32_t lo = o + (uint32_t)(((uint64_t)j * cnt) / m);
    const uint32_t hi = o + (uint32_t)(((uint64_t)(j + 1) * cnt) / m);
    if constexpr (sizeof(F) <= 32) {
        // G1: software pipeline, the next point is in flight while this one is added
        uint32_t v = 0, vn = 0;
        Affine<F> p;
        if (lo < hi) {
            v = sorted[lo];
            p = ld(pts + (v & 0x7fffffffu));
        }
        if (lo + 1 < hi) vn = sorted[lo + 1];
        for (uint32_t e = lo; e < hi; e++) {
            Affine<F> q = p;
            const uint32_t cv = v;
            if (e + 1 < hi) {
                p = ld(pts + (vn & 0x7fffffffu));
                v = vn;
                if (e + 2 < hi) vn = sorted[e + 2];
            }
            if (skip_inf && q.is_inf()) continue;  // hole of a wire-indexed table
            if (cv >> 31) q.y = -q.y;
            xyzz_madd_inplace(acc, q);
        }
    } else {
        // G2: no room for a second point in registers (235 VGPRs at occupancy 2)
        for (uint32_t e = lo; e < hi; e++) {
            uint32_t v = sorted[e];
            Affine<F> p = ld(pts + (v & 0x7fffffffu));
            if (skip_inf && p.is_inf()) continue;
            if (v >> 31) p.y = -p.y;
            xyzz_madd_inplace(acc, p);
        }
    }
    }  // valid
    // in-block segmented tree over the light buckets' partials (G1 only: the G2
    // XYZZ add does not fit the 256-VGPR budget of this kernel; G2 light
    // buckets are summed by k_bucket_sum instead)
    if constexpr (!kMergeInBlock<F>) {
        if (valid) st(partial + t, acc);
        return;
    }
    const bool light = valid && (io1 - io0) <= LIGHT;
    const size_t blk0 = (size_t)blockIdx.x * blockDim.x;
    const size_t seg_lo = light ? std::max<size_t>(io0, blk0) : t;
    const size_t seg_hi = light ? std::min<size_t>(std::min<size_t>(io1, blk0 + blockDim.x), n_items) : t;
    const uint32_t rel = (uint32_t)(t - seg_lo);
    sh[threadIdx.x] = acc;
    for (uint32_t s2 = 1; s2 < LIGHT; s2 <<= 1) {
        const bool act = light && (rel % (2 * s2)) == 0 && t + s2 < seg_hi;
        if (!__syncthreads_or(act)) break;
        if (act) {
            Xyzz<F> o2 = sh[threadIdx.x + s2];
            xyzz_add_inplace(acc, o2);
            sh[threadIdx.x] = acc;
        }
    }
    if (valid) st(partial + t, acc);
}

// In-place segmented tree over the level-1 partials: bucket b owns slots
// [item_off[b], item_off[b+1]); after the launches with stride 1, 2, 4, ...
// slot item_off[b] holds the bucket sum.  One quad per slot (xyzz_add_quad), no
// host syncs.
template <class F>
__global__ void __launch_bounds__(256) k_seg_tree(Xyzz<F>* part, const uint32_t* item_off,
                                                  const uint32_t* item_bucket, size_t T,
                                                  uint32_t stride, uint32_t fan) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = (uint32_t)g & 3;
    const size_t p = g >> 2;
    if (p >= T) return;  // every branch below is uniform over the quad
    uint32_t b = item_bucket[p];
    uint32_t o = item_off[b];
    uint32_t j = (uint32_t)p - o;
    uint32_t cnt = item_off[b + 1] - o;
    if (cnt <= LIGHT) return;  // done by k_bucket_sum
    if (j % (fan * stride)) return;
    if (j + stride >= cnt) return;
    Xyzz<F> acc = ld(part + p);
    for (uint32_t k = 1; k < fan && j + k * stride < cnt; k++) xyzz_add_quad(acc, ld(part + p + k * stride), lane);
    if (lane == 0) st(part + p, acc);
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

// Level 2 for light buckets (2..LIGHT partials): QB quads per bucket.  Quad j
// adds partials j, j + QB, ... of its bucket with quad adds, then log2(QB)
// xor-shuffle rounds (lane masks 4, 8, ...) combine the quads.  Every lane
// takes part in the shuffles; only the adds are predicated.
template <class F, uint32_t QB>
__global__ void __launch_bounds__(256) k_bucket_sum(Xyzz<F>* part, const uint32_t* item_off, size_t nb) {
    static_assert(QB == 1 || QB == 2 || QB == 4, "quads per bucket");
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t b = t / (4 * QB);
    const uint32_t k = (uint32_t)t & 3, j = (uint32_t)(t >> 2) & (QB - 1);
    uint32_t o = 0, cnt = 0;
    if (b < nb) {
        o = item_off[b];
        cnt = item_off[b + 1] - o;
    }
    const bool act = cnt >= 2 && cnt <= LIGHT;
    Xyzz<F> acc = Xyzz<F>::inf();
    if (act)
        for (uint32_t i = j; i < cnt; i += QB) xyzz_add_quad(acc, ld(part + o + i), k);
    for (int s = 4; s < (int)(4 * QB); s <<= 1) {
        const Xyzz<F> other = shfl_xor_words(acc, s);
        if (act) xyzz_add_quad(acc, other, k);
    }
    if (act && j == 0 && k == 0) st(part + o, acc);
}

// ------------------------------------------------------------ reduction v2
// Dense bucket sums: S[b] = partial of bucket b (or infinity)
// (item_off is indexed in sort order pi(b) = bitrev_{c-1}(b), see sort_entries)
template <class F>
__global__ void k_gather_buckets(const Xyzz<F>* partial, const uint32_t* item_off, size_t nb, int c,
                                 Xyzz<F>* S) {
    size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    uint32_t q = __brev((uint32_t)b) >> (33 - c);
    uint32_t o = item_off[q], e = item_off[q + 1];
    Xyzz<F> v = (e > o) ? ld(partial + o) : Xyzz<F>::inf();
    if (kMergeInBlock<F> && e - o > 1 && e - o <= LIGHT) {  // second in-block head
        uint32_t k = ((o >> 8) + 1) << 8;
        if (k < e) xyzz_add_inplace(v, ld(partial + k));
    }
    st(S + b, v);
}

// copy a list of small device arrays into one contiguous staging buffer
template <class F>
struct GatherList {
    const Xyzz<F>* src[64];
    uint32_t off[65];
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
// Sorted entries + work items of one scalar vector over a base shape (n, c, W,
// scalar index map).  Bases with identical shapes can share one: the Groth16
// prover sorts the wires once for A/K and once for B1/G2.
struct MsmSort {
    DevBuf sorted, counts, offsets, itemcnt, item_off, item_bucket, maxcnt;
    DevBuf keys, tmp_entry, tmp_key, hist, hoff, bin_start, seg2, chunk_start, chunk_hist, chunk_pos,
        chunk_desc;
    std::vector<DevBuf> scan_tmp;
    uint32_t* pin = nullptr;          // pinned (n_items, max_items) read-back
    hipEvent_t pin_ev = nullptr;      // after the read-back copy
    hipEvent_t ready_ev = nullptr;    // after the item -> bucket map
    int K1 = 32;
    size_t items_ub = 0;
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
}  // namespace gg

struct gg_msm_base {
    int group = GG_G1;
    size_t n = 0;  // resident points
    int c = 0, W = 0;
    gg::WinSpec win{};  // per-window bit widths / offsets
    size_t nb = 0;
    DevBuf pts;   // W * n affine points, window-major
    DevBuf sidx;  // n u32 or empty
    bool has_sidx = false;
    bool has_inf = false;  // wire-indexed table with infinity holes (skipped)
    int scurve = 0;        // scalar field: 0 = BN254 fr, 1 = BLS12-381 fr
    uint32_t max_sidx = 0;
    std::mutex mu;
    gg::MsmSort own;                  // this base's sort state
    DevBuf partA, segs, segs2, scal;  // per-base accumulation / reduction scratch
};

namespace gg {

template <class F>
inline void precompute(gg_msm_base* b, const Affine<F>* dev_in, hipStream_t st) {
    const size_t n = b->n;
    b->pts.alloc((size_t)b->W * n * sizeof(Affine<F>));
    Affine<F>* out = b->pts.as<Affine<F>>();
    DevBuf cur(n * sizeof(Xyzz<F>));
    // ~64 elements per thread amortise one Fermat inversion, >= 16K threads
    const size_t T = std::min<size_t>(n, std::max<size_t>(16384, n / 64));
    DevBuf prefix(n * sizeof(F));
    hipLaunchKernelGGL(k_pre_init<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, dev_in, n, out,
                       cur.as<Xyzz<F>>());
    GG_HIP(hipGetLastError());
    for (int w = 1; w < b->W; w++) {
        hipLaunchKernelGGL(k_pre_dbl<F>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                           cur.as<Xyzz<F>>(), n, (int)b->win.bits[w - 1]);
        GG_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_pre_normalize<F>, dim3(grid_for(T, 256)), dim3(256), 0, st,
                           (const Xyzz<F>*)cur.p, n, T, prefix.as<F>(), out + (size_t)w * n);
        GG_HIP(hipGetLastError());
    }
    GG_HIP(hipStreamSynchronize(st));
}

// Weighted bucket sum sum_{b<nb} (b+1) S_b with log-depth, wide tree sums
// (DESIGN.md "MSM / bucket reduction"): a weighted sum WS(X, off) =
// sum_j (j + off) X_j over n = 2^k elements is split as j = q*M + r into
// M * WS(H, 0) + WS(G, off) with row sums H_q and column sums G_r -- both plain
// tree sums that run wide on the GPU.  Pieces of <= 16 elements finish on the
// host, combined by Horner over their 2^mlog factors.
template <class F>
inline Xyzz<F> bucket_reduce_2d(gg_msm_base* b, const Xyzz<F>* partials, const uint32_t* item_off,
                                hipStream_t st) {
    const size_t nb = b->nb;
    const size_t XB = sizeof(Xyzz<F>);
    b->segs.reserve(nb * XB);
    const size_t arena_elems = 3 * nb + 1024;
    b->segs2.reserve(arena_elems * XB);
    Xyzz<F>* S = b->segs.as<Xyzz<F>>();
    hipLaunchKernelGGL(k_gather_buckets<F>, dim3(grid_for(nb, 256)), dim3(256), 0, st, partials,
                       item_off, nb, b->c, S);
    GG_HIP(hipGetLastError());
    Xyzz<F>* arena = b->segs2.as<Xyzz<F>>();
    size_t used = 0;
    auto alloc = [&](size_t cnt) {
        GG_CHECK(used + cnt <= arena_elems, GG_ERR_INTERNAL, "bucket reduction arena overflow");
        Xyzz<F>* p = arena + used;
        used += cnt;
        return p;
    };
    struct Item { const Xyzz<F>* X; uint32_t n, off; int mlog; };
    struct Job { const Xyzz<F>* in; uint32_t A, Bc, sa, sb; Item dest; };
    std::vector<Item> items{{S, (uint32_t)nb, 1u, 0}};
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
            jobs.push_back({it.X, M, rows, 1u, M, Item{nullptr, rows, 0u, it.mlog + mlg}});
            jobs.push_back({it.X, rows, M, M, 1u, Item{nullptr, M, it.off, it.mlog}});
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
    // host: tiny weighted sums + Horner over the 2^mlog factors
    GG_CHECK(host_items.size() <= 64, GG_ERR_INTERNAL, "too many host reduction items");
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
    GG_HIP(hipStreamSynchronize(st));
    std::vector<std::vector<Xyzz<F>>> hx(host_items.size());
    for (size_t k = 0; k < host_items.size(); k++)
        hx[k].assign(flat.begin() + GL.off[k], flat.begin() + GL.off[k + 1]);
    std::vector<std::pair<int, Xyzz<F>>> vals;
    for (size_t k = 0; k < host_items.size(); k++) {
        const auto& X = hx[k];
        Xyzz<F> run = Xyzz<F>::inf(), acc = Xyzz<F>::inf();
        for (size_t j = X.size(); j-- > 1;) {
            run = xyzz_add(run, X[j]);
            acc = xyzz_add(acc, run);
        }
        if (host_items[k].off) {
            run = xyzz_add(run, X[0]);  // run = sum of all
            for (uint32_t o = 0; o < host_items[k].off; o++) acc = xyzz_add(acc, run);
        }
        vals.push_back({host_items[k].mlog, acc});
    }
    std::sort(vals.begin(), vals.end(), [](const auto& x, const auto& y) { return x.first > y.first; });
    Xyzz<F> acc = Xyzz<F>::inf();
    int cur = vals.empty() ? 0 : vals[0].first;
    for (auto& v : vals) {
        for (; cur > v.first; cur--) acc = acc.is_inf() ? acc : xyzz_dbl(acc);
        acc = xyzz_add(acc, v.second);
    }
    for (; cur > 0; cur--) acc = acc.is_inf() ? acc : xyzz_dbl(acc);
    return acc;
}

// Accumulation + reduction of base b over a prepared sort s (its own or one
// shared with a base of identical shape).  Waits (device side) for s->ready_ev.
template <class F>
inline Xyzz<F> msm_finish(gg_msm_base* b, MsmSort* s, hipStream_t st) {
    const size_t n = b->n, nb = b->nb;
    if (n == 0) return Xyzz<F>::inf();
    GG_HIP(hipStreamWaitEvent(st, s->ready_ev, 0));
    const uint32_t* offs = s->offsets.as<uint32_t>();
    const uint32_t* ioff = s->item_off.as<uint32_t>();
    const size_t items_ub = s->items_ub;
    b->partA.reserve((items_ub + 1) * sizeof(Xyzz<F>));
    {
        // per-group names: the Groth16 prove runs G1 and G2 accumulations at once
        const char* acc_name = sizeof(F) == sizeof(Fp) ? "msm_accum" : (sizeof(F) == sizeof(Fp2) ? "msm_accum_g2" : "msm_accum_bls");
        ProfScope ps_acc(acc_name, st, (double)n);
        hipLaunchKernelGGL(k_accum_affine<F>, dim3(grid_for(items_ub, 256)), dim3(256),
                           kMergeInBlock<F> ? 256 * sizeof(Xyzz<F>) : 0, st, (const Affine<F>*)b->pts.p,
                           s->sorted.as<uint32_t>(), offs, ioff, s->item_bucket.as<uint32_t>(),
                           ioff + nb, s->K1, (int)b->has_inf, b->partA.as<Xyzz<F>>());
        GG_HIP(hipGetLastError());
        ps_acc.stop(st);
    }
    GG_HIP(hipEventSynchronize(s->pin_ev));
    const size_t n_items = s->pin[0];
    const uint32_t max_items = s->pin[1];
    GG_CHECK(n_items <= items_ub, GG_ERR_INTERNAL, "item count above its bound");
    // ---- level 2: light buckets summed by a thread each, heavy buckets (> LIGHT
    // items) by a per-bucket tree (skew-robust: log2(items) launches)
    ProfScope ps_acc2("msm_accum2", st, (double)n);
    if (!kMergeInBlock<F> && max_items > 1) {
        // quads per bucket (MI355X sweep: one quad per bucket at 2^20; more
        // lanes make the level throughput-bound)
        static const int l2qb = getenv("GG_L2_QB") ? atoi(getenv("GG_L2_QB")) : 1;
        Xyzz<F>* pa = b->partA.as<Xyzz<F>>();
        if (l2qb >= 4) hipLaunchKernelGGL((k_bucket_sum<F, 4>), dim3(grid_for(16 * nb, 256)), dim3(256), 0, st, pa, ioff, nb);
        else if (l2qb == 2) hipLaunchKernelGGL((k_bucket_sum<F, 2>), dim3(grid_for(8 * nb, 256)), dim3(256), 0, st, pa, ioff, nb);
        else hipLaunchKernelGGL((k_bucket_sum<F, 1>), dim3(grid_for(4 * nb, 256)), dim3(256), 0, st, pa, ioff, nb);
        GG_HIP(hipGetLastError());
    }
    for (uint32_t stride = 1; max_items > LIGHT && stride < max_items;) {
        uint32_t fan = (stride == 1) ? 4u : 2u;
        hipLaunchKernelGGL(k_seg_tree<F>, dim3(grid_for(4 * n_items, 256)), dim3(256), 0, st,
                           b->partA.as<Xyzz<F>>(), ioff, s->item_bucket.as<uint32_t>(), n_items, stride,
                           fan);
        GG_HIP(hipGetLastError());
        stride *= fan;
    }
    ps_acc2.stop(st);
    // ---- bucket reduction: sum_b (b+1) S_b
    ProfScope ps_red("msm_reduce", st, (double)nb);
    Xyzz<F> res = bucket_reduce_2d<F>(b, (const Xyzz<F>*)b->partA.p, ioff, st);
    ps_red.stop(st);
    return res;
}

template <class F>
inline Xyzz<F> msm_run(gg_msm_base* b, const Fr* scalars_dev, hipStream_t st) {
    if (b->n == 0) return Xyzz<F>::inf();
    msm_prepare(b, &b->own, scalars_dev, st);
    return msm_finish<F>(b, &b->own, st);
}

template <class F>
inline void create_base(gg_msm_base* b, const void* points, size_t n, int on_device,
                        const uint32_t* sidx, int window_bits, bool keep_inf = false,
                        int scurve = 0) {
    b->scurve = scurve;
    const int total = scalar_total_bits(scurve);
    const size_t pb = sizeof(Affine<F>);
    std::vector<uint8_t> host;
    const uint8_t* src;
    if (on_device) {
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
    b->c = window_bits ? window_bits : choose_c(std::max<size_t>(b->n, 1), pb, total);
    GG_CHECK(b->c >= 2 && b->c <= 24, GG_ERR_INVALID_ARG, "window_bits out of range [2, 24]");
    b->W = (total + b->c - 1) / b->c;
    b->c = (total + b->W - 1) / b->W;  // widest balanced window for this W
    GG_CHECK(b->W <= 64, GG_ERR_INVALID_ARG, "too many windows");
    b->win = make_windows(b->c, b->W, total);
    b->nb = (size_t)1 << (b->c - 1);
    GG_CHECK((double)b->W * (double)b->n < 2147483648.0, GG_ERR_UNSUPPORTED,
             "too many points x windows for 31-bit entry ids");
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

