// Non-template MSM kernels: scalar digits, counting sort, scan, work items.
#include "msm_impl.cuh"
#include <atomic>
#include <cstdlib>

namespace gg {
// ------------------------------------------------------------------ scan
__global__ void k_scan_block(const uint32_t* in, uint32_t* out, uint32_t* sums, size_t n) {
    __shared__ uint32_t s[256];
    const int PER = 8;
    size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x) * PER;
    uint32_t v[PER];
    uint32_t tot = 0;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        v[i] = (base + i < n) ? in[base + i] : 0u;
        tot += v[i];
    }
    s[threadIdx.x] = tot;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        uint32_t x = (threadIdx.x >= (unsigned)off) ? s[threadIdx.x - off] : 0u;
        __syncthreads();
        s[threadIdx.x] += x;
        __syncthreads();
    }
    uint32_t run = s[threadIdx.x] - tot;  // exclusive
#pragma unroll
    for (int i = 0; i < PER; i++) {
        if (base + i < n) out[base + i] = run;
        run += v[i];
    }
    if (threadIdx.x == 255 && sums) sums[blockIdx.x] = s[255];
}

__global__ void k_scan_add(uint32_t* out, const uint32_t* sums, size_t n) {
    size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
    uint32_t a = sums[blockIdx.x];
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (base + i < n) out[base + i] += a;
}

// k_scan_add with each block's prefix summed from the block sums directly (no
// scan of the sums: one launch fewer; for up to kScanPrefixMax blocks, <= 16
// loads a thread)
constexpr size_t kScanPrefixMax = 4096;
__global__ void __launch_bounds__(256) k_scan_add_prefix(uint32_t* out, const uint32_t* sums, size_t n) {
    __shared__ uint32_t wsum[4];
    uint32_t acc = 0;
    for (uint32_t i = threadIdx.x; i < blockIdx.x; i += 256) acc += sums[i];
    for (int off = 32; off > 0; off >>= 1) acc += (uint32_t)__shfl_xor((int)acc, off);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
    __syncthreads();
    const uint32_t a = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (!a) return;
    const size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (base + i < n) out[base + i] += a;
}

// exclusive scan of n >= 1 u32: out[0..n) (out[n] is set by k_set_total)
void exclusive_scan(const uint32_t* in, uint32_t* out, size_t n, hipStream_t st,
                    std::vector<DevBuf>& tmp, int depth) {
    const size_t per_block = 256 * 8;
    size_t blocks = (n + per_block - 1) / per_block;
    if (blocks <= 1) {
        hipLaunchKernelGGL(k_scan_block, dim3(1), dim3(256), 0, st, in, out, nullptr, n);
        GG_HIP(hipGetLastError());
        return;
    }
    if (blocks <= kScanPrefixMax) {  // two launches (round 6: the sort's launch count)
        if (tmp.size() < (size_t)(depth + 1) * 2) tmp.resize((size_t)(depth + 1) * 2);
        tmp[2 * depth].reserve(blocks * 4);
        uint32_t* sums = tmp[2 * depth].as<uint32_t>();
        hipLaunchKernelGGL(k_scan_block, dim3((unsigned)blocks), dim3(256), 0, st, in, out, sums, n);
        GG_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_scan_add_prefix, dim3((unsigned)blocks), dim3(256), 0, st, out, sums, n);
        GG_HIP(hipGetLastError());
        return;
    }
    if (tmp.size() < (size_t)(depth + 1) * 2) tmp.resize((size_t)(depth + 1) * 2);
    tmp[2 * depth].reserve(blocks * 4);
    tmp[2 * depth + 1].reserve(blocks * 4);
    uint32_t* sums = tmp[2 * depth].as<uint32_t>();
    uint32_t* scanned = tmp[2 * depth + 1].as<uint32_t>();
    hipLaunchKernelGGL(k_scan_block, dim3((unsigned)blocks), dim3(256), 0, st, in, out, sums, n);
    GG_HIP(hipGetLastError());
    exclusive_scan(sums, scanned, blocks, st, tmp, depth + 1);
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)blocks), dim3(256), 0, st, out, scanned, n);
    GG_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ kernels
__global__ void k_set_total(uint32_t* out, const uint32_t* in, size_t n) {
    // out[n] = out[n-1] + in[n-1]
    if (n) out[n] = out[n - 1] + in[n - 1];
    else out[0] = 0;
}

template <class E>
__device__ __forceinline__ uint32_t extract_bits(const E& k, int bit, int c) {
    if (bit >= 256) return 0;
    int limb = bit >> 5, off = bit & 31;
    uint64_t v = k.v[limb] >> off;
    if (off + c > 32 && limb < 7) v |= (uint64_t)k.v[limb + 1] << (32 - off);
    return (uint32_t)(v & ((1u << c) - 1));
}

// entries of the fullest bucket: block-level max, one atomic per block
__global__ void __launch_bounds__(256) k_bucket_max(const uint32_t* offsets, size_t nb, uint32_t* maxcnt) {
    __shared__ uint32_t wmax[4];
    size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v = b < nb ? offsets[b + 1] - offsets[b] : 0u;
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        if (m) atomicMax(maxcnt, m);
    }
}

int choose_c(size_t n, size_t point_bytes, int total_bits) {
    if (const char* e = getenv("GG_MSM_WINDOW")) {  // tuning override
        int c = atoi(e);
        if (c >= 4 && c <= 24) return c;
    }
    // cost ~ bucket additions (n*W) + per-bucket level-2 / reduction work, fitted
    // to MI355X sweeps (2^20: c=17; 2^24 G1: c=22; G2 and G1 bases sharing a G2
    // sort, point_bytes = 128: c=20 -- the Fp2 bucket reduction weighs twice);
    // epb > 512 (entries per bucket) makes heavy buckets (+25 %).  With balanced
    // accumulation ranges short buckets cost nothing extra.  Window widths are
    // balanced (make_windows), so every c is usable.
    const double per_bucket = point_bytes >= 128 ? 12.0 : 6.0;
    int best = 16;
    double bc = 1e300;
    for (int c = 4; c <= 23; c++) {
        int W = (total_bits + c - 1) / c;
        if ((total_bits + W - 1) / W != c) continue;  // same W as a narrower c
        double mem = (double)W * (double)n * (double)point_bytes;
        if (mem > 48e9) continue;  // precomputed table budget per base
        const double entries = (double)n * W, buckets = (double)(1u << (c - 1));
        const double epb = entries / buckets;
        double f = 1.0 + (epb > 512 ? 0.25 : 0.0);
        double cost = entries * f + buckets * per_bucket;
        if (cost < bc) { bc = cost; best = c; }
    }
    return best;
}

// process-wide cap on what precompute tables may take (gg_set_hbm_budget; 0 = none)
static std::atomic<unsigned long long> g_hbm_budget{0};

int choose_groups(double bytes, double extra, int W) { return choose_groups_multi(&bytes, &W, 1, extra); }

int choose_groups_multi(const double* bytes, const int* W, int k, double extra) {
    if (const char* e = getenv("GG_MSM_GROUPS")) {  // override (tests, tuning)
        const int g = atoi(e);
        if (g == 1 || g == 2 || g == 4 || g == 8 || g == 16) return g;
    }
    int wmax = 1;
    for (int i = 0; i < k; i++) wmax = std::max(wmax, W[i]);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
        (void)hipGetLastError();
        return 1;
    }
    // keep 4 GiB or 3 % of the card for the per-proof scratch of other work
    double avail = (double)fr - std::max(4.0 * (1ull << 30), 0.03 * (double)tot);
    const unsigned long long cap = g_hbm_budget.load();
    if (cap) avail = std::min(avail, (double)cap);
    int g = 1;
    while (g < 16 && g < wmax) {
        double need = extra;
        for (int i = 0; i < k; i++) need += bytes[i] * (double)((W[i] + g - 1) / g) / (double)W[i];
        if (need <= avail) break;
        g <<= 1;
    }
    return g;
}

}  // namespace gg

extern "C" int gg_set_hbm_budget(size_t bytes) {
    gg::g_hbm_budget.store((unsigned long long)bytes);
    return GG_OK;
}

extern "C" size_t gg_get_hbm_budget(void) { return (size_t)gg::g_hbm_budget.load(); }

// ===================================================================== sort v2
// Counting sort of the (window, scalar) entries by bucket without global
// atomics (DESIGN.md "MSM / sort"):
//   A. k_digits_hist : signed digits -> keys[w*n+i]; per-block LDS histogram of
//                      the bucket's top h bits ("bins"), written bin-major.
//   B. exclusive scan of the [bin][block] histogram -> per-(bin, block) bases.
//   C. k_bin_scatter : entries scattered into their bin, ranks from LDS atomics.
//   D. k_bin_sort    : one workgroup per bin, LDS counting sort on the low bits,
//                      writes the final per-bucket offsets.
namespace gg {

// scalars per block in phases A / C: spb = min(512, pow2 <= 8192 / W) so the
// LDS-staged tile of phase C holds <= 8192 entries (64 KiB)
inline int sort_spb(int W) {
    int s = 512;
    while (s > 32 && s * W > 8192) s >>= 1;
    return s;
}

// Sort order is by pi(b) = bitrev_{c-1}(b): bins take the LOW bits of the bucket
// id, so the small ids of a narrow top window spread over all bins.
// With precompute groups the bucket id B = j 2^(c-1) + b carries the group in
// its top bits (kbits = c - 1 + log2 G key bits): sort key = bucket_perm(B).
__device__ __forceinline__ uint32_t bin_of(uint32_t B, int c, int kbits, int h) {
    return bucket_perm(B, c) >> (kbits - h);
}

// exclusive scan of v over a 256-thread block (4 wave scans + one barrier);
// `wsum` is 4 words of LDS.  Returns the exclusive prefix; *total = block sum.
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const int lane = __lane_id(), wv = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t w = wsum[i];
        if (i < wv) pre += w;
        tot += w;
    }
    *total = tot;
    return pre + x - v;
}

// Wave-level multisplit rank: lanes with equal digit d form a group (found with
// rbits ballots); one LDS atomic per group, the rank within the group comes from
// a popcount.  Removes same-address LDS atomic serialisation.  Must be called by
// all lanes of the wave (inactive lanes pass valid = false).
__device__ __forceinline__ uint32_t wave_rank(uint32_t* cnt, uint32_t d, bool valid, int rbits) {
    uint64_t match = __ballot(valid);
    for (int bb = 0; bb < rbits; bb++) {
        const bool bit = (d >> bb) & 1u;
        const uint64_t bal = __ballot(bit);
        match &= bit ? bal : ~bal;
    }
    const int lane = __lane_id();
    const uint32_t rank = (uint32_t)__popcll(match & ((1ull << lane) - 1));
    const int leader = match ? __ffsll((unsigned long long)match) - 1 : lane;
    uint32_t b = 0;
    if (valid && lane == leader) b = atomicAdd(&cnt[d], (uint32_t)__popcll(match));
    b = __shfl(b, leader);
    return b + rank;
}

// The sort key of every window of one scalar, in window order (the signed digits
// carry upward): fn(w, key), key = bucket | sign bit, or 0xffffffff for a zero
// digit or (bucket stripes, slog > 0) a bucket outside stripe sres.
template <class SC, class Fn>
__device__ __forceinline__ void scalar_keys(const Fe<SC>& scl, int c, int W, const WinSpec& ws, int G, int slog,
                                            uint32_t sres, uint32_t gofs, Fn&& fn) {
    const uint32_t smask = (1u << slog) - 1u;
    const Fe<SC> k = from_mont(scl);
    int carry = 0;
    for (int w = 0; w < W; w++) {
        const int bw = ws.bits[w];
        int d = (int)extract_bits(k, ws.off[w], bw) + carry;
        if (d > (1 << (bw - 1))) { d -= (1 << bw); carry = 1; } else carry = 0;
        uint32_t key = 0xffffffffu;
        const uint32_t bb = (uint32_t)((d > 0 ? d : -d) - 1);  // bucket |d| - 1 of group w mod G
        if (d && (bb & smask) == sres) {
            // bucket stripe (slog > 0): only buckets bb = 2^slog j + sres, renumbered j;
            // c is then the stripe's c - slog
            const uint32_t bk = ((gofs + (uint32_t)(w & (G - 1))) << (c - 1)) | (bb >> slog);
            key = bk | (d < 0 ? 0x80000000u : 0u);
        }
        fn(w, key);
    }
}

// Phase A: the block's bin histogram and every entry's key for phase C.  (Round
// 4 measured phase C deriving the keys again from the scalars instead: 3.37 vs
// 3.14 ms per 2^24 sort, profiles/r04_c_sort_ab.txt -- the key array stays.)
// A batch of nvec scalar vectors over one base (same-base commitments): block
// column = v vblocks + tile, vector v's keys in rows v W + w, its buckets in
// groups v G .. v G + G - 1 (sort_entries).
// SPT = scalars per thread (spb <= 256 SPT), all loaded before any digit work
template <class SC, int SPT>
__global__ void __launch_bounds__(256) k_digits_hist(VecPtrs vp, const uint32_t* sidx,
                                                     size_t n, int c, int W, WinSpec ws, int G, int kbits,
                                                     int spb, int nbins, int h, uint32_t* keys, size_t kst,
                                                     uint32_t* hist, uint32_t nblocks, uint32_t vblocks, int slog,
                                                     uint32_t sres) {
    extern __shared__ uint32_t hh[];
    const uint32_t col = blockIdx.x;        // histogram column
    const uint32_t v = col / vblocks;       // scalar vector of the batch
    const uint32_t tile = col - v * vblocks;  // its scalar range
    const Fe<SC>* scalars = static_cast<const Fe<SC>*>(vp.p[v]);
    uint32_t* vkeys = keys + (size_t)v * W * kst;
    for (int j = threadIdx.x; j < nbins; j += blockDim.x) hh[j] = 0;
    __syncthreads();
    Fe<SC> scl[SPT];
    size_t idx[SPT];
#pragma unroll
    for (int s = 0; s < SPT; s++) {
        idx[s] = ~(size_t)0;
        if (s * 256 + (int)threadIdx.x < spb) {
            size_t i = (size_t)tile * spb + s * 256 + threadIdx.x;
            if (i < n) {
                idx[s] = i;
                scl[s] = ld(scalars + (sidx ? sidx[i] : i));
            }
        }
    }
#pragma unroll
    for (int s = 0; s < SPT; s++) {
        if (idx[s] == ~(size_t)0) continue;
        const size_t i = idx[s];
        scalar_keys<SC>(scl[s], c, W, ws, G, slog, sres, v * (uint32_t)G, [&](int w, uint32_t key) {
            if (key != 0xffffffffu) atomicAdd(&hh[bin_of(key & 0x7fffffffu, c, kbits, h)], 1u);
            vkeys[(size_t)w * kst + i] = key;
        });
    }
    __syncthreads();
    for (int j = threadIdx.x; j < nbins; j += blockDim.x) hist[(size_t)j * nblocks + col] = hh[j];
}

// Phase C, LDS-staged: the block's entries are first partitioned by bin in LDS
// (ranks from LDS atomics, bin bases from this block's own histogram), then
// written out as contiguous per-bin runs -> coalesced stores.
__global__ void __launch_bounds__(256) k_bin_scatter(const uint32_t* keys, size_t kst, size_t n, int W, int c, int G,
                                                     int kbits, int spb, int nbins, int h, const uint32_t* hist,
                                                     const uint32_t* hoff, uint32_t nblocks, uint32_t vblocks,
                                                     uint32_t* tmp_entry, void* tmp_key, int key16) {
    extern __shared__ uint32_t sm[];
    const uint32_t col = xcd_swizzle(blockIdx.x, gridDim.x);  // histogram column (k_digits_hist)
    const uint32_t v = col / vblocks;
    const uint32_t tile = col - v * vblocks;
    keys += (size_t)v * W * kst;
    uint32_t* lbase = sm;             // nbins: local exclusive offsets
    uint32_t* lcur = sm + nbins;      // nbins: local cursors
    uint32_t* s_entry = sm + 2 * nbins;
    uint32_t* s_key = s_entry + spb * W;
    const int lowbits = kbits - h;
    // this block's column of the histogram and of the global bin offsets, one bin
    // per thread (nbins <= 256), both loads in flight together; the local
    // exclusive scan is a wave scan + one barrier
    const uint32_t jb = threadIdx.x;
    const bool has = (int)jb < nbins;
    const uint32_t cnt = has ? hist[(size_t)jb * nblocks + col] : 0u;
    const uint32_t gof = has ? hoff[(size_t)jb * nblocks + col] : 0u;
    __shared__ uint32_t wsum[4];
    uint32_t tot;
    const uint32_t ex = block_excl_scan256(cnt, wsum, &tot);
    if (has) {
        lbase[jb] = ex;
        lcur[jb] = ex;
    }
    __syncthreads();
    const size_t i0 = (size_t)tile * spb;
    const int ns = (int)min((size_t)spb, n - i0);
    const int tot_e = ns * W;
    // flat (window, scalar) index j = w * ns + t; keys loaded 8 per batch before
    // the LDS atomics so the loads overlap
    for (int jb0 = 0; jb0 < tot_e; jb0 += 8 * 256) {
        uint32_t kk[8];
        uint32_t ee[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            int j = jb0 + (int)threadIdx.x + u * 256;
            kk[u] = 0xffffffffu;
            if (j < tot_e) {
                int w = j / ns, t = j - w * ns;
                kk[u] = keys[(size_t)w * kst + i0 + t];
                ee[u] = (uint32_t)((size_t)(w / G) * n + i0 + t);  // the stored copy of window w
            }
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            uint32_t key = kk[u];
            if (key == 0xffffffffu) continue;
            uint32_t pk = bucket_perm(key & 0x7fffffffu, c);
            uint32_t q = atomicAdd(&lcur[pk >> lowbits], 1u);
            s_entry[q] = ee[u] | (key & 0x80000000u);
            s_key[q] = pk;
        }
    }
    __syncthreads();
    // staged slot q of bin b goes to hoff[b][tile] + (q - lbase[b]): the
    // difference per bin, from LDS
    if (has) lbase[jb] = gof - ex;
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < tot; q += blockDim.x) {
        const uint32_t pk = s_key[q];
        const uint32_t pos = lbase[pk >> lowbits] + q;
        tmp_entry[pos] = s_entry[q];
        if (tmp_key) {
            if (key16) static_cast<uint16_t*>(tmp_key)[pos] = (uint16_t)pk;  // the low kbits - h <= 16 bits
            else static_cast<uint32_t*>(tmp_key)[pos] = pk;
        }
    }
}

// bin_start[j] = hoff[j * nblocks] (j < nbins), bin_start[nbins] = total
__global__ void k_bin_starts(const uint32_t* hoff, const uint32_t* hist, uint32_t nblocks, int nbins,
                             uint32_t* bin_start) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < nbins) bin_start[j] = hoff[(size_t)j * nblocks];
    if (j == 0) {
        size_t last = (size_t)nbins * nblocks - 1;
        bin_start[nbins] = hoff[last] + hist[last];
    }
}

// ---- phase D: segmented MSD passes.  Each pass splits every segment (a run of
// entries sharing the bucket's high bits) on the next r <= 8 bits, in chunks of
// <= SEG_CH entries that never straddle a segment, so any skew (a bucket holding
// half of all entries, as 0/1-heavy witnesses produce) spreads over many
// workgroups.  The scatter is LDS-staged: a chunk is first ordered by digit in
// LDS, then written as per-digit runs of ~SEG_CH / 2^r entries (coalesced).
// 2048 (round 4, r04_v): 2^24 G1 sort 3.29 -> 3.12 ms against 4096 (half the
// registers and LDS per workgroup: twice the resident scatter waves); 1024 slower
#ifndef GG_SEG_CH
#define GG_SEG_CH 2048
#endif
constexpr uint32_t SEG_CH = GG_SEG_CH;
constexpr int SEG_PER = SEG_CH / 256;  // entries per thread

// chunk_start[0..nseg] (exclusive scan of the segments' chunk counts, total at
// [nseg]) in one block, for nseg <= 2048: the first segmented pass's 256 bins
__global__ void __launch_bounds__(256) k_seg_plan_small(const uint32_t* seg_start, uint32_t nseg,
                                                        uint32_t* chunk_start) {
    __shared__ uint32_t wsum[4];
    uint32_t c[8], t = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t sg = threadIdx.x * 8 + i;
        c[i] = sg < nseg ? (seg_start[sg + 1] - seg_start[sg] + SEG_CH - 1) / SEG_CH : 0u;
        t += c[i];
    }
    uint32_t tot;
    uint32_t run = block_excl_scan256(t, wsum, &tot);
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t sg = threadIdx.x * 8 + i;
        if (sg < nseg) chunk_start[sg] = run;
        run += c[i];
    }
    if (threadIdx.x == 0) chunk_start[nseg] = tot;
}

// a chunk's descriptor {lo, hi, g0, nch} -- its entry range, the first chunk of
// its segment, the segment's chunks; nch = 0 marks a grid slot past the last
// chunk -- computed by one thread of the block that works on the chunk
__device__ __forceinline__ uint4 chunk_desc_block(const uint32_t* seg_start, const uint32_t* chunk_start,
                                                  uint32_t nseg, uint32_t g) {
    __shared__ uint4 d;
    if (threadIdx.x == 0) {
        uint4 r = make_uint4(0, 0, 0, 0);
        if (g < chunk_start[nseg]) {
            uint32_t lo = 0, hi = nseg;  // largest s with chunk_start[s] <= g
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (chunk_start[mid] <= g) lo = mid;
                else hi = mid;
            }
            const uint32_t g0 = chunk_start[lo], nch = chunk_start[lo + 1] - g0, k = g - g0;
            const uint32_t a = seg_start[lo] + k * SEG_CH, b = min(seg_start[lo + 1], a + SEG_CH);
            r = make_uint4(a, b, g0, nch);
        }
        d = r;
    }
    __syncthreads();
    return d;
}

__global__ void k_seg_chunk_counts(const uint32_t* seg_start, uint32_t nseg, uint32_t* cnt) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < nseg) cnt[s] = (seg_start[s + 1] - seg_start[s] + SEG_CH - 1) / SEG_CH;
}


// counters laid out [segment][digit][chunk-in-segment]: one global exclusive
// scan then yields absolute output positions.
// KT: the key word of the segmented passes -- u16 once the bins hold the high
// bits and <= 16 remain (the usual case: c - 1 = 21 bucket bits, 8 of them bins),
// halving the key traffic of every later pass
template <class KT>
__global__ void __launch_bounds__(256) k_seg_hist(const KT* keys, const uint32_t* seg_start,
                                                  const uint32_t* chunk_start, uint32_t nseg, int shift,
                                                  int rbits, uint32_t* ch) {
    __shared__ uint32_t hist[256];
    const uint32_t g = xcd_swizzle(blockIdx.x, gridDim.x);
    const uint4 dsc = chunk_desc_block(seg_start, chunk_start, nseg, g);
    const uint32_t lo = dsc.x, hi = dsc.y, g0 = dsc.z, nch = dsc.w, k = g - g0;
    if (nch == 0) return;
    const uint32_t R = 1u << rbits;
    if (threadIdx.x < R) hist[threadIdx.x] = 0;
    __syncthreads();
    // the chunk's aligned middle in 4-key vectors, the unaligned ends one key a lane
    // (round 4: 2^24 G1 sort 3.53 -> 3.29 ms against one key a lane, profiles/r04_u_*)
    const uint32_t a0 = min(hi, (lo + 3u) & ~3u), a1 = max(a0, hi & ~3u);
    for (uint32_t e = lo + threadIdx.x; e < a0; e += blockDim.x)
        atomicAdd(&hist[(keys[e] >> shift) & (R - 1)], 1u);
    for (uint32_t e = a1 + threadIdx.x; e < hi; e += blockDim.x)
        atomicAdd(&hist[(keys[e] >> shift) & (R - 1)], 1u);
    struct alignas(4 * sizeof(KT)) K4 { KT k[4]; };
    const K4* kv = reinterpret_cast<const K4*>(keys + a0);
    const uint32_t nv = (a1 - a0) >> 2;
    for (uint32_t q = threadIdx.x; q < nv; q += blockDim.x) {
        const K4 x = kv[q];
#pragma unroll
        for (int u = 0; u < 4; u++) atomicAdd(&hist[(x.k[u] >> shift) & (R - 1)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < R) ch[(size_t)g0 * R + (size_t)threadIdx.x * nch + k] = hist[threadIdx.x];
}

template <class KT>
__global__ void __launch_bounds__(256) k_seg_scatter(const uint32_t* ent_in, const KT* key_in,
                                                     const uint32_t* seg_start, const uint32_t* chunk_start,
                                                     uint32_t nseg, int shift, int rbits,
                                                     const uint32_t* chpos, uint32_t* ent_out,
                                                     KT* key_out) {
    __shared__ uint32_t cnt[256], base[256], part[256];
    extern __shared__ uint32_t stage[];  // SEG_CH entries, SEG_CH digits (u8) [, SEG_CH keys]
    const uint32_t g = xcd_swizzle(blockIdx.x, gridDim.x);
    const uint4 dsc = chunk_desc_block(seg_start, chunk_start, nseg, g);
    const uint32_t lo = dsc.x, hi = dsc.y, g0 = dsc.z, nch = dsc.w, k = g - g0;
    if (nch == 0) return;
    const uint32_t R = 1u << rbits;
    const uint32_t m = hi - lo;
    if (threadIdx.x < R) cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t ek[SEG_PER], ee[SEG_PER], rk[SEG_PER];
#pragma unroll
    for (int j = 0; j < SEG_PER; j++) {
        uint32_t q = threadIdx.x + 256u * j;
        ek[j] = 0;
        ee[j] = 0;
        if (q < m) {
            ek[j] = key_in[lo + q];
            ee[j] = ent_in[lo + q];
        }
    }
#pragma unroll
    for (int j = 0; j < SEG_PER; j++) {
        uint32_t q = threadIdx.x + 256u * j;
        rk[j] = wave_rank(cnt, (ek[j] >> shift) & (R - 1), q < m, rbits);
    }
    __syncthreads();
    // exclusive scan of the chunk's digit counts
    uint32_t tot_unused;
    const uint32_t v = threadIdx.x < R ? cnt[threadIdx.x] : 0u;
    const uint32_t ex = block_excl_scan256(v, part, &tot_unused);
    if (threadIdx.x < R) base[threadIdx.x] = ex;
    uint8_t* s_dig = (uint8_t*)(stage + SEG_CH);
    uint32_t* s_key = stage + SEG_CH + SEG_CH / 4;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SEG_PER; j++) {
        uint32_t q = threadIdx.x + 256u * j;
        if (q < m) {
            const uint32_t d = (ek[j] >> shift) & (R - 1);
            uint32_t p = base[d] + rk[j];
            stage[p] = ee[j];
            s_dig[p] = (uint8_t)d;
            if (key_out) s_key[p] = ek[j];
        }
    }
    // global position of each digit's run
    if (threadIdx.x < R) cnt[threadIdx.x] = chpos[(size_t)g0 * R + (size_t)threadIdx.x * nch + k];
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < m; q += blockDim.x) {
        uint32_t kk = key_out ? s_key[q] : 0u;
        const uint32_t dl = s_dig[q];
        uint32_t pos = cnt[dl] + (q - base[dl]);
        ent_out[pos] = stage[q];
        if (key_out) key_out[pos] = (KT)kk;
    }
}

// start of every sub-segment: next[s * R + d]; next[nseg * R] = total
__global__ void k_seg_next(const uint32_t* seg_start, const uint32_t* chunk_start, const uint32_t* chpos,
                           uint32_t nseg, int rbits, uint32_t* next) {
    size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t R = 1u << rbits;
    if (q >= (size_t)nseg * R) return;
    uint32_t sg = (uint32_t)(q >> rbits), d = (uint32_t)(q & (R - 1));
    uint32_t g0 = chunk_start[sg], nch = chunk_start[sg + 1] - g0;
    next[q] = nch ? chpos[(size_t)g0 * R + (size_t)d * nch] : seg_start[sg];
    if (q == 0) next[(size_t)nseg * R] = seg_start[nseg];
}

// number of bits of the first (bin) pass and the split of the rest into passes
static void sort_plan(int c, int& h, std::vector<int>& rs) {
    h = std::min(8, c - 1);
    if (const char* e = getenv("GG_SORT_H")) h = std::max(1, std::min(atoi(e), std::min(8, c - 1)));
    int rmax = 8;  // one segmented pass for c <= 17 (MI355X sweep: 2^20 sort 0.38 -> 0.26 ms)
    if (const char* e = getenv("GG_SORT_RMAX")) rmax = std::max(1, std::min(atoi(e), 8));
    int low = (c - 1) - h;
    rs.clear();
    if (low <= 0) return;
    int np = (low + rmax - 1) / rmax;
    for (int i = 0; i < np; i++) {
        int r = low / (np - i);
        rs.push_back(r);
        low -= r;
    }
}

void sort_entries(const gg_msm_base* b, MsmSort* s, const VecPtrs& vp, hipStream_t st) {
    // a bucket stripe sorts a 2^-slog share of the buckets, renumbered densely:
    // the bucket ids (and every sort key) are those of a c - slog window.  A
    // batch of s->nvec vectors sorts into s->kp (power of two >= nvec) copies of
    // the bucket space, vector v in groups v G .. v G + G - 1.
    const size_t n = b->n, nb = (b->nb >> s->slog) * (size_t)s->kp;
    const int c = b->c - s->slog, W = b->W, G = b->G;
    const size_t total = (size_t)W * n * (size_t)s->nvec;
    const int kbits = (c - 1) + __builtin_ctz((unsigned)(G * s->kp));  // sort key bits
    int h;
    std::vector<int> rs;
    sort_plan(kbits + 1, h, rs);
    const int nbins = 1 << h;
    int spb = sort_spb(W);
    if (const char* e = getenv("GG_SORT_SPB")) {  // tuning override: a power of two, 32..1024,
        const int v = atoi(e);                     // the bin-scatter tile spb W <= 16384 entries
        if (v >= 32 && v <= 1024 && (v & (v - 1)) == 0 && v * W <= 16384) spb = v;
    }
    const uint32_t vblocks = (uint32_t)((n + spb - 1) / spb);  // per vector
    const uint32_t nblocks = vblocks * (uint32_t)s->nvec;
    const size_t nh = (size_t)nbins * nblocks;
    // all scratch reserved up front (no reallocation between launches)
    size_t ch_max = 0;
    {
        size_t ns = (size_t)nbins;
        for (int r : rs) {
            ch_max = std::max(ch_max, ((total + SEG_CH - 1) / SEG_CH + ns) << r);
            ns <<= r;
        }
    }
    // key rows of phase A, stride kst = n (round 4: rows padded to 256-B
    // boundaries and XCD-aware histogram tiles measured no change, r04_u)
    const size_t kst = n;
    s->keys.reserve(total * 4);
    s->tmp_entry.reserve(total * 4);
    s->tmp_key.reserve(total * 4);
    s->sorted.reserve(total * 4 + 64);  // + 64: the accumulation reads 16-B chunks past its last entry
    s->hist.reserve(nh * 4);
    s->hoff.reserve((nh + 1) * 4);
    s->bin_start.reserve(((size_t)nb + 1) * 4);
    s->seg2.reserve(((size_t)nb + 1) * 4);
    s->offsets.reserve((nb + 1) * 4);
    s->counts.reserve(nb * 4);
    s->chunk_start.reserve(((size_t)nb + 1) * 4);
    if (ch_max) {
        s->chunk_hist.reserve(ch_max * 4);
        s->chunk_pos.reserve((ch_max + 1) * 4);
    }
    {
        auto* const hk = b->scurve ? (spb > 512 ? &k_digits_hist<FrBlsCfg, 4> : &k_digits_hist<FrBlsCfg, 2>)
                                   : (spb > 512 ? &k_digits_hist<FrCfg, 4> : &k_digits_hist<FrCfg, 2>);
        hipLaunchKernelGGL(hk, dim3(nblocks), dim3(256), nbins * 4, st, vp,
                           b->has_sidx ? b->sidx.as<uint32_t>() : nullptr, n, c, W, b->win, G, kbits, spb, nbins,
                           h, s->keys.as<uint32_t>(), kst, s->hist.as<uint32_t>(), nblocks, vblocks, s->slog,
                           s->sres);
        GG_HIP(hipGetLastError());
    }
    exclusive_scan(s->hist.as<uint32_t>(), s->hoff.as<uint32_t>(), nh, st, s->scan_tmp);
    // segment starts ping-pong between bin_start and seg2; the last pass writes offsets
    DevBuf* segb[2] = {&s->bin_start, &s->seg2};
    hipLaunchKernelGGL(k_bin_starts, dim3(grid_for(nbins, 256)), dim3(256), 0, st,
                       s->hoff.as<uint32_t>(), s->hist.as<uint32_t>(), nblocks, nbins,
                       rs.empty() ? s->offsets.as<uint32_t>() : segb[0]->as<uint32_t>());
    GG_HIP(hipGetLastError());
    const size_t lds_c = (2 * (size_t)nbins + 2 * (size_t)spb * W) * 4;
    GG_CHECK(lds_c <= 160 * 1024, GG_ERR_INTERNAL, "bin scatter LDS tile too large");
    if (lds_c > 64 * 1024)  // GG_SORT_SPB tiles past 64 KiB: opt in to the CU's 160 KiB
        GG_HIP(hipFuncSetAttribute((const void*)k_bin_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_c));
    GG_CHECK(nbins <= 256, GG_ERR_INTERNAL, "bin scatter: one bin per thread");
    // scatter stage j (0 = bin scatter) writes entries to `sorted` when the number
    // of stages after it is even, else tmp_entry; keys to tmp_key (j even) / keys (j odd)
    const int S = 1 + (int)rs.size();
    auto ent_out = [&](int j) { return ((S - 1 - j) % 2 == 0) ? &s->sorted : &s->tmp_entry; };
    auto key_out = [&](int j) { return (j % 2 == 0) ? &s->tmp_key : &s->keys; };
    const bool key16 = kbits - h <= 16;
    hipLaunchKernelGGL(k_bin_scatter, dim3(nblocks), dim3(256), lds_c, st, s->keys.as<uint32_t>(), kst,
                       n, W, c, G, kbits, spb, nbins, h, s->hist.as<uint32_t>(), s->hoff.as<uint32_t>(), nblocks,
                       vblocks, ent_out(0)->as<uint32_t>(), S > 1 ? key_out(0)->p : nullptr, (int)key16);
    GG_HIP(hipGetLastError());
    uint32_t nseg = (uint32_t)nbins;
    int shift = kbits - h;
    for (int j = 1; j < S; j++) {
        const int r = rs[j - 1];
        const bool last = j == S - 1;
        shift -= r;
        const uint32_t R = 1u << r;
        const size_t max_chunks = (total + SEG_CH - 1) / SEG_CH + nseg;
        const uint32_t* segp = segb[(j - 1) & 1]->as<uint32_t>();
        const uint32_t* cst = s->chunk_start.as<uint32_t>();
        // round 6: fewer launches per pass (each costs ~5 us of dependent-launch
        // gap on the sort's stream, 24 per sort before): the chunk plan in one
        // block when it fits, the descriptors inside the hist / scatter blocks,
        // no zeroing of the chunk histogram (every real chunk's counters are
        // written and the scan's stale tail lies past them)
        if (nseg <= 2048) {
            hipLaunchKernelGGL(k_seg_plan_small, dim3(1), dim3(256), 0, st, segp, nseg, s->chunk_start.as<uint32_t>());
            GG_HIP(hipGetLastError());
        } else {
            hipLaunchKernelGGL(k_seg_chunk_counts, dim3(grid_for(nseg, 256)), dim3(256), 0, st, segp, nseg,
                               s->counts.as<uint32_t>());
            GG_HIP(hipGetLastError());
            exclusive_scan(s->counts.as<uint32_t>(), s->chunk_start.as<uint32_t>(), nseg, st, s->scan_tmp);
            hipLaunchKernelGGL(k_set_total, dim3(1), dim3(1), 0, st, s->chunk_start.as<uint32_t>(),
                               s->counts.as<uint32_t>(), (size_t)nseg);
            GG_HIP(hipGetLastError());
        }
        const void* kin = key_out(j - 1)->p;
        if (key16)
            hipLaunchKernelGGL(k_seg_hist<uint16_t>, dim3((unsigned)max_chunks), dim3(256), 0, st,
                               (const uint16_t*)kin, segp, cst, nseg, shift, r, s->chunk_hist.as<uint32_t>());
        else
            hipLaunchKernelGGL(k_seg_hist<uint32_t>, dim3((unsigned)max_chunks), dim3(256), 0, st,
                               (const uint32_t*)kin, segp, cst, nseg, shift, r, s->chunk_hist.as<uint32_t>());
        GG_HIP(hipGetLastError());
        exclusive_scan(s->chunk_hist.as<uint32_t>(), s->chunk_pos.as<uint32_t>(), max_chunks * R, st,
                       s->scan_tmp);
        const size_t lds_s = (size_t)SEG_CH * (last ? 5 : 9);
        if (key16)
            hipLaunchKernelGGL(k_seg_scatter<uint16_t>, dim3((unsigned)max_chunks), dim3(256), lds_s, st,
                               ent_out(j - 1)->as<uint32_t>(), (const uint16_t*)kin, segp, cst, nseg,
                               shift, r, s->chunk_pos.as<uint32_t>(), ent_out(j)->as<uint32_t>(),
                               last ? nullptr : key_out(j)->as<uint16_t>());
        else
            hipLaunchKernelGGL(k_seg_scatter<uint32_t>, dim3((unsigned)max_chunks), dim3(256), lds_s, st,
                               ent_out(j - 1)->as<uint32_t>(), (const uint32_t*)kin, segp, cst, nseg,
                               shift, r, s->chunk_pos.as<uint32_t>(), ent_out(j)->as<uint32_t>(),
                               last ? nullptr : key_out(j)->as<uint32_t>());
        GG_HIP(hipGetLastError());
        uint32_t* next = last ? s->offsets.as<uint32_t>() : segb[j & 1]->as<uint32_t>();
        hipLaunchKernelGGL(k_seg_next, dim3(grid_for((size_t)nseg * R, 256)), dim3(256), 0, st, segp,
                           s->chunk_start.as<uint32_t>(), s->chunk_pos.as<uint32_t>(), nseg, r, next);
        GG_HIP(hipGetLastError());
        nseg *= R;
    }
}

// ---- a sort derived from another base's (Groth16: B1 / G2 from the A / K sort).
// Base a indexes the scalars directly (entry = w' n_a + i, i = the scalar's
// index), base b through its map (entry = w' n_b + j, scalar sidx_b[j]), with
// the same window layout.  bmap[i] = j for the scalars b uses, else ~0.  The
// entries of a's sorted list whose scalar b uses, renumbered and kept in order,
// are b's sorted list: same digits, same buckets.  A stable filter (flags,
// exclusive scan, scatter) instead of a second sort; b's bucket offsets are the
// kept counts before a's.
__global__ void k_derive_flags(const uint32_t* sorted, const uint32_t* offsets, uint32_t nb, size_t cap, uint32_t n,
                               const uint32_t* bmap, uint32_t* flags) {
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= cap) return;
    uint32_t f = 0;
    if (e < offsets[nb]) f = bmap[(sorted[e] & 0x7fffffffu) % n] != 0xffffffffu;
    flags[e] = f;
}
__global__ void k_derive_scatter(const uint32_t* sorted, const uint32_t* offsets, uint32_t nb, uint32_t n, uint32_t nb_pts,
                                 const uint32_t* bmap, const uint32_t* pos, uint32_t* out) {
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= offsets[nb]) return;
    const uint32_t v = sorted[e], idx = v & 0x7fffffffu;
    const uint32_t j = bmap[idx % n];
    if (j == 0xffffffffu) return;
    out[pos[e]] = ((idx / n) * nb_pts + j) | (v & 0x80000000u);
}
__global__ void k_derive_offsets(const uint32_t* offa, const uint32_t* pos, uint32_t nb, uint32_t* offb) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q <= nb) offb[q] = pos[offa[q]];
}

void msm_prepare_derived(const gg_msm_base* a, const MsmSort* sa, const gg_msm_base* b, MsmSort* sb,
                         const uint32_t* bmap, hipStream_t st) {
    GG_CHECK(a->c == b->c && a->W == b->W && a->G == b->G && !a->has_sidx && sa->nvec == 1, GG_ERR_INTERNAL,
             "derived sort: the bases' window layouts differ (or a batch sort)");
    sb->nvec = 1;
    sb->kp = 1;
    const size_t cap = (size_t)a->W * a->n, nb = a->nb >> sa->slog;
    sb->slog = sa->slog;
    sb->sres = sa->sres;
    sb->ensure_events();
    sb->keys.reserve(std::max<size_t>(cap, 1) * 4);           // flags
    sb->tmp_entry.reserve((std::max<size_t>(cap, 1) + 1) * 4);  // kept positions (+ the total)
    sb->sorted.reserve(std::max<size_t>((size_t)b->W * b->n, 1) * 4 + 64);  // 16-B chunk reads
    sb->offsets.reserve((nb + 1) * 4);
    sb->maxcnt.reserve(4);
    GG_HIP(hipStreamWaitEvent(st, sa->ready_ev, 0));
    {
        ProfScope ps_sort("msm_sort", st, (double)b->n);
        uint32_t* flags = sb->keys.as<uint32_t>();
        uint32_t* pos = sb->tmp_entry.as<uint32_t>();
        const uint32_t* offa = sa->offsets.as<uint32_t>();
        hipLaunchKernelGGL(k_derive_flags, dim3(grid_for(cap, 256)), dim3(256), 0, st, sa->sorted.as<uint32_t>(),
                           offa, (uint32_t)nb, cap, (uint32_t)a->n, bmap, flags);
        GG_HIP(hipGetLastError());
        exclusive_scan(flags, pos, cap, st, sb->scan_tmp);
        hipLaunchKernelGGL(k_set_total, dim3(1), dim3(1), 0, st, pos, flags, cap);
        GG_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_derive_scatter, dim3(grid_for(cap, 256)), dim3(256), 0, st, sa->sorted.as<uint32_t>(),
                           offa, (uint32_t)nb, (uint32_t)a->n, (uint32_t)b->n, bmap, pos, sb->sorted.as<uint32_t>());
        GG_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_derive_offsets, dim3(grid_for(nb + 1, 256)), dim3(256), 0, st, offa, pos, (uint32_t)nb,
                           sb->offsets.as<uint32_t>());
        GG_HIP(hipGetLastError());
        ps_sort.stop(st);
    }
    GG_HIP(hipMemsetAsync(sb->maxcnt.p, 0, 4, st));
    hipLaunchKernelGGL(k_bucket_max, dim3(grid_for(nb, 256)), dim3(256), 0, st, sb->offsets.as<uint32_t>(), nb,
                       sb->maxcnt.as<uint32_t>());
    GG_HIP(hipGetLastError());
    GG_HIP(hipMemcpyAsync(sb->pin, sb->maxcnt.p, 4, hipMemcpyDeviceToHost, st));
    GG_HIP(hipMemcpyAsync(sb->pin + 1, sb->offsets.as<uint32_t>() + nb, 4, hipMemcpyDeviceToHost, st));
    GG_HIP(hipEventRecord(sb->pin_ev, st));
    GG_HIP(hipEventRecord(sb->ready_ev, st));
}

// Sort of one scalar vector over b's shape into s; records s->ready_ev (sort
// done) and s->pin_ev (the fullest bucket's entry count on the host).
void msm_prepare(const gg_msm_base* b, MsmSort* s, const Fr* scalars_dev, hipStream_t st, int slog,
                 uint32_t sres) {
    VecPtrs vp{};
    vp.p[0] = scalars_dev;
    msm_prepare_batch(b, s, vp, 1, st, slog, sres);
}

// the sort of nvec scalar vectors over b's points in one pass (same-base
// commitments: PlonK's L, R, O and H1, H2, H3, prove.go:425-502, 1199-1218)
void msm_prepare_batch(const gg_msm_base* b, MsmSort* s, const VecPtrs& vp, int nvec, hipStream_t st, int slog,
                       uint32_t sres) {
    GG_CHECK(slog >= 0 && slog <= b->c - 2 && sres < (1u << slog), GG_ERR_INVALID_ARG,
             "bucket stripe out of range (stripe_log <= window_bits - 2, part < 2^stripe_log)");
    GG_CHECK(nvec >= 1 && nvec <= kMaxBatch && (nvec == 1 || slog == 0), GG_ERR_INVALID_ARG,
             "batch of 1..4 scalar vectors (no bucket stripes)");
    GG_CHECK(nvec == 1 || msm_batch_fits(b->n, b->W, b->c, b->G, nvec), GG_ERR_UNSUPPORTED,
             "MSM batch too large for 32-bit sort indices (gg_msm_batch_shape)");
    s->slog = slog;
    s->sres = sres;
    s->nvec = nvec;
    s->kp = 1;
    while (s->kp < nvec) s->kp <<= 1;
    const size_t n = b->n, nb = (b->nb >> slog) * (size_t)s->kp;
    s->ensure_events();
    s->counts.reserve(nb * 4);
    s->offsets.reserve((nb + 1) * 4);
    s->maxcnt.reserve(4);
    {
        ProfScope ps_sort("msm_sort", st, (double)n);
        sort_entries(b, s, vp, st);
        ps_sort.stop(st);
    }
    GG_HIP(hipMemsetAsync(s->maxcnt.p, 0, 4, st));
    hipLaunchKernelGGL(k_bucket_max, dim3(grid_for(nb, 256)), dim3(256), 0, st, s->offsets.as<uint32_t>(), nb,
                       s->maxcnt.as<uint32_t>());
    GG_HIP(hipGetLastError());
    GG_HIP(hipMemcpyAsync(s->pin, s->maxcnt.p, 4, hipMemcpyDeviceToHost, st));
    GG_HIP(hipMemcpyAsync(s->pin + 1, s->offsets.as<uint32_t>() + nb, 4, hipMemcpyDeviceToHost, st));
    GG_HIP(hipEventRecord(s->pin_ev, st));
    GG_HIP(hipEventRecord(s->ready_ev, st));
}

}  // namespace gg
