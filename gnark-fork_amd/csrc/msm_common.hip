// Non-template MSM kernels: scalar digits, counting sort, scan, work items.
#include "msm_impl.cuh"
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
// total count of entries for out[n] of the scan is handled by k_total.
// out[n] = total, out[n+1] = *maxcnt (one 8-byte read-back per level)
__global__ void k_set_total_max(uint32_t* out, const uint32_t* in, size_t n, const uint32_t* maxcnt) {
    out[n] = n ? out[n - 1] + in[n - 1] : 0u;
    out[n + 1] = *maxcnt;
}

__global__ void k_set_total(uint32_t* out, const uint32_t* in, size_t n) {
    // out[n] = out[n-1] + in[n-1]
    if (n) out[n] = out[n - 1] + in[n - 1];
    else out[0] = 0;
}

__device__ __forceinline__ uint32_t extract_bits(const Fr& k, int bit, int c) {
    if (bit >= 256) return 0;
    int limb = bit >> 5, off = bit & 31;
    uint64_t v = k.v[limb] >> off;
    if (off + c > 32 && limb < 7) v |= (uint64_t)k.v[limb + 1] << (32 - off);
    return (uint32_t)(v & ((1u << c) - 1));
}

// items per bucket = ceil(cnt / K); block-level max, one atomic per block
__global__ void __launch_bounds__(256) k_item_counts(const uint32_t* offsets, size_t nb, int K,
                                                     uint32_t* itemcnt, uint32_t* maxcnt) {
    __shared__ uint32_t wmax[4];
    size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v = 0;
    if (b < nb) {
        uint32_t cnt = offsets[b + 1] - offsets[b];
        v = (cnt + K - 1) / K;
        itemcnt[b] = v;
    }
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        if (m) atomicMax(maxcnt, m);
    }
}

// item -> bucket map: one thread per item, upper_bound over item_off (a heavy
// bucket's thousands of items no longer serialise on one thread)
__global__ void k_item_buckets(const uint32_t* item_off, size_t nb, size_t n_items,
                               uint32_t* item_bucket) {
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_items) return;
    size_t lo = 0, hi = nb;  // largest b with item_off[b] <= t (item_off[0] = 0)
    while (hi - lo > 1) {
        size_t mid = (lo + hi) >> 1;
        if (item_off[mid] <= (uint32_t)t) lo = mid; else hi = mid;
    }
    item_bucket[t] = (uint32_t)lo;
}

int choose_c(size_t n, size_t point_bytes) {
    if (const char* e = getenv("GG_MSM_WINDOW")) {  // tuning override
        int c = atoi(e);
        if (c >= 4 && c <= 24) return c;
    }
    // cost ~ bucket additions (n*W) + reduction (~6 madd-equivalents per bucket:
    // its tail is latency- not throughput-bound).  The top window holds only
    // 254 - c(W-1) bits; if that is much narrower than c, all n of its entries
    // pile into a few buckets (long chains, skewed sort bins): require
    // top_bits >= c - 6 (measured on MI355X: c=18/19/21 at 2^20 are 2-3x slower).
    int best = 16;
    double bc = 1e300;
    for (int c = 4; c <= 23; c++) {
        int W = (255 + c - 1) / c;
        int top_bits = 254 - c * (W - 1);
        if (c > 8 && top_bits < c - 6) continue;
        double mem = (double)W * (double)n * (double)point_bytes;
        if (mem > 48e9) continue;  // precomputed table budget per base
        double cost = (double)n * W + (double)(1u << (c - 1)) * 6.0;
        if (cost < bc) { bc = cost; best = c; }
    }
    return best;
}

}  // namespace gg

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
__device__ __forceinline__ uint32_t pi_of(uint32_t b, int c) { return __brev(b) >> (33 - c); }
__device__ __forceinline__ uint32_t bin_of(uint32_t b, int c) { return pi_of(b, c) >> (c - 1 - min(8, c - 1)); }

__global__ void __launch_bounds__(256) k_digits_hist(const Fr* scalars, const uint32_t* sidx,
                                                     size_t n, int c, int W, int spb, int nbins,
                                                     uint32_t* keys, uint32_t* hist,
                                                     uint32_t nblocks) {
    extern __shared__ uint32_t h[];
    for (int j = threadIdx.x; j < nbins; j += blockDim.x) h[j] = 0;
    __syncthreads();
    const int half = 1 << (c - 1);
    for (int s = 0; s * 256 < spb; s++) {
        if (s * 256 + (int)threadIdx.x >= spb) break;
        size_t i = (size_t)blockIdx.x * spb + s * 256 + threadIdx.x;
        if (i >= n) break;
        Fr sc = ld(scalars + (sidx ? sidx[i] : i));
        Fr k = from_mont(sc);
        int carry = 0;
        for (int w = 0; w < W; w++) {
            int d = (int)extract_bits(k, w * c, c) + carry;
            if (d > half) { d -= (1 << c); carry = 1; } else carry = 0;
            uint32_t key = 0xffffffffu;
            if (d) {
                uint32_t bk = (uint32_t)((d > 0 ? d : -d) - 1);
                key = bk | (d < 0 ? 0x80000000u : 0u);
                atomicAdd(&h[bin_of(bk, c)], 1u);
            }
            keys[(size_t)w * n + i] = key;
        }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < nbins; j += blockDim.x) hist[(size_t)j * nblocks + blockIdx.x] = h[j];
}

// Phase C, LDS-staged: the block's entries are first partitioned by bin in LDS
// (ranks from LDS atomics, bin bases from this block's own histogram), then
// written out as contiguous per-bin runs -> coalesced stores.
__global__ void __launch_bounds__(256) k_bin_scatter(const uint32_t* keys, size_t n, int W, int c, int spb,
                                                     int nbins, const uint32_t* hist,
                                                     const uint32_t* hoff, uint32_t nblocks,
                                                     uint32_t* tmp_entry, uint32_t* tmp_key) {
    extern __shared__ uint32_t sm[];
    uint32_t* lbase = sm;             // nbins: local exclusive offsets
    uint32_t* lcur = sm + nbins;      // nbins: local cursors
    uint32_t* s_entry = sm + 2 * nbins;
    uint32_t* s_key = s_entry + spb * W;
    const int lowbits = (c - 1) - min(8, c - 1);
    // local exclusive scan of this block's histogram (column of hist)
    __shared__ uint32_t part[256];
    const int per = (nbins + 255) / 256;
    uint32_t s = 0;
    for (int k = 0; k < per; k++) {
        int j = threadIdx.x * per + k;
        if (j < nbins) s += hist[(size_t)j * nblocks + blockIdx.x];
    }
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        uint32_t x = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += x;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
    for (int k = 0; k < per; k++) {
        int j = threadIdx.x * per + k;
        if (j < nbins) {
            lbase[j] = run;
            lcur[j] = run;
            run += hist[(size_t)j * nblocks + blockIdx.x];
        }
    }
    __syncthreads();
    const size_t i0 = (size_t)blockIdx.x * spb;
    const int ns = (int)min((size_t)spb, n - i0);
    for (int w = 0; w < W; w++) {
        for (int t = threadIdx.x; t < ns; t += blockDim.x) {
            size_t e = (size_t)w * n + i0 + t;
            uint32_t key = keys[e];
            if (key == 0xffffffffu) continue;
            uint32_t pk = pi_of(key & 0x7fffffffu, c);
            uint32_t q = atomicAdd(&lcur[pk >> lowbits], 1u);
            s_entry[q] = (uint32_t)e | (key & 0x80000000u);
            s_key[q] = pk;
        }
    }
    __syncthreads();
    const uint32_t tot = part[255];
    for (uint32_t q = threadIdx.x; q < tot; q += blockDim.x) {
        uint32_t pk = s_key[q];
        uint32_t bin = pk >> lowbits;
        uint32_t pos = hoff[(size_t)bin * nblocks + blockIdx.x] + (q - lbase[bin]);
        tmp_entry[pos] = s_entry[q];
        tmp_key[pos] = pk;
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

// ---- phase D: chunked counting sort of every bin on its low bits.  Chunks of
// <= SORT_CH entries never straddle a bin, so any skew (a bucket holding half of
// all entries, as 0/1-heavy witnesses produce) spreads over many workgroups.
constexpr uint32_t SORT_CH = 4096;

// chunk_start[b] = first chunk of bin b, chunk_start[nbins] = total chunks
__global__ void __launch_bounds__(256) k_chunk_setup(const uint32_t* bin_start, int nbins,
                                                     uint32_t* chunk_start) {
    __shared__ uint32_t part[256];
    const int per = (nbins + 255) / 256;
    const int b0 = threadIdx.x * per;
    uint32_t s = 0;
    for (int k = 0; k < per; k++) {
        int b = b0 + k;
        if (b < nbins) s += (bin_start[b + 1] - bin_start[b] + SORT_CH - 1) / SORT_CH;
    }
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        uint32_t x = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += x;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
    for (int k = 0; k < per; k++) {
        int b = b0 + k;
        if (b < nbins) {
            chunk_start[b] = run;
            run += (bin_start[b + 1] - bin_start[b] + SORT_CH - 1) / SORT_CH;
        }
    }
    if (threadIdx.x == 255) chunk_start[nbins] = part[255];
}

__device__ __forceinline__ int find_bin(const uint32_t* chunk_start, int nbins, uint32_t g) {
    int lo = 0, hi = nbins;  // largest b with chunk_start[b] <= g
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (chunk_start[mid] <= g) lo = mid; else hi = mid;
    }
    return lo;
}

// counters laid out [bin][low][chunk-in-bin]: one global exclusive scan then
// yields absolute output positions.
__global__ void __launch_bounds__(256) k_chunk_hist(const uint32_t* tmp_key, const uint32_t* bin_start,
                                                    const uint32_t* chunk_start, int nbins, int lowbits,
                                                    uint32_t* ch) {
    extern __shared__ uint32_t hist[];
    const uint32_t g = blockIdx.x;
    if (g >= chunk_start[nbins]) return;
    const int L = 1 << lowbits;
    const int b = find_bin(chunk_start, nbins, g);
    const uint32_t g0 = chunk_start[b], nch = chunk_start[b + 1] - g0, k = g - g0;
    const uint32_t lo = bin_start[b] + k * SORT_CH, hi = min(bin_start[b + 1], lo + SORT_CH);
    for (int j = threadIdx.x; j < L; j += blockDim.x) hist[j] = 0;
    __syncthreads();
    for (uint32_t e = lo + threadIdx.x; e < hi; e += blockDim.x) atomicAdd(&hist[tmp_key[e] & (L - 1)], 1u);
    __syncthreads();
    for (int j = threadIdx.x; j < L; j += blockDim.x) ch[(size_t)g0 * L + (size_t)j * nch + k] = hist[j];
}

__global__ void __launch_bounds__(256) k_chunk_scatter(const uint32_t* tmp_entry, const uint32_t* tmp_key,
                                                       const uint32_t* bin_start,
                                                       const uint32_t* chunk_start, int nbins,
                                                       int lowbits, const uint32_t* chs,
                                                       uint32_t* sorted) {
    extern __shared__ uint32_t cur[];
    const uint32_t g = blockIdx.x;
    if (g >= chunk_start[nbins]) return;
    const int L = 1 << lowbits;
    const int b = find_bin(chunk_start, nbins, g);
    const uint32_t g0 = chunk_start[b], nch = chunk_start[b + 1] - g0, k = g - g0;
    const uint32_t lo = bin_start[b] + k * SORT_CH, hi = min(bin_start[b + 1], lo + SORT_CH);
    for (int j = threadIdx.x; j < L; j += blockDim.x) cur[j] = chs[(size_t)g0 * L + (size_t)j * nch + k];
    __syncthreads();
    for (uint32_t e = lo + threadIdx.x; e < hi; e += blockDim.x) {
        uint32_t pos = atomicAdd(&cur[tmp_key[e] & (L - 1)], 1u);
        sorted[pos] = tmp_entry[e];
    }
}

// offsets[(bin << lowbits) + low] = start of that bucket (in pi order); [nb] = total
__global__ void k_bucket_offsets(const uint32_t* bin_start, const uint32_t* chunk_start,
                                 const uint32_t* chs, int nbins, int lowbits, uint32_t* offsets) {
    size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int L = 1 << lowbits;
    if (q >= ((size_t)nbins << lowbits)) return;
    int b = (int)(q >> lowbits), l = (int)(q & (L - 1));
    uint32_t g0 = chunk_start[b], nch = chunk_start[b + 1] - g0;
    offsets[q] = nch ? chs[(size_t)g0 * L + (size_t)l * nch] : bin_start[b];
    if (q == 0) offsets[(size_t)nbins << lowbits] = bin_start[nbins];
}

void sort_entries(gg_msm_base* b, const Fr* scalars_dev, hipStream_t st) {
    const size_t n = b->n, nb = b->nb;
    const int c = b->c, W = b->W;
    const size_t total = (size_t)W * n;
    const int h = std::min(8, c - 1);
    const int nbins = 1 << h;
    const int lowbits = (c - 1) - h;
    const int spb = sort_spb(W);
    const uint32_t nblocks = (uint32_t)((n + spb - 1) / spb);
    const size_t nh = (size_t)nbins * nblocks;
    b->keys.reserve(total * 4);
    b->tmp_entry.reserve(total * 4);
    b->tmp_key.reserve(total * 4);
    b->sorted.reserve(total * 4);
    b->hist.reserve(nh * 4);
    b->hoff.reserve((nh + 1) * 4);
    b->bin_start.reserve((nbins + 1) * 4);
    b->offsets.reserve((nb + 1) * 4);
    hipLaunchKernelGGL(k_digits_hist, dim3(nblocks), dim3(256), nbins * 4, st, scalars_dev,
                       b->has_sidx ? b->sidx.as<uint32_t>() : nullptr, n, c, W, spb, nbins,
                       b->keys.as<uint32_t>(), b->hist.as<uint32_t>(), nblocks);
    GG_HIP(hipGetLastError());
    exclusive_scan(b->hist.as<uint32_t>(), b->hoff.as<uint32_t>(), nh, st, b->scan_tmp);
    hipLaunchKernelGGL(k_bin_starts, dim3(grid_for(nbins, 256)), dim3(256), 0, st,
                       b->hoff.as<uint32_t>(), b->hist.as<uint32_t>(), nblocks, nbins,
                       b->bin_start.as<uint32_t>());
    GG_HIP(hipGetLastError());
    const size_t lds_c = (2 * (size_t)nbins + 2 * (size_t)spb * W) * 4;
    GG_CHECK(lds_c <= 160 * 1024, GG_ERR_INTERNAL, "bin scatter LDS tile too large");
    hipLaunchKernelGGL(k_bin_scatter, dim3(nblocks), dim3(256), lds_c, st, b->keys.as<uint32_t>(),
                       n, W, c, spb, nbins, b->hist.as<uint32_t>(), b->hoff.as<uint32_t>(), nblocks,
                       b->tmp_entry.as<uint32_t>(), b->tmp_key.as<uint32_t>());
    GG_HIP(hipGetLastError());
    const size_t L = (size_t)1 << lowbits;
    const size_t max_chunks = (total + SORT_CH - 1) / SORT_CH + nbins;
    b->chunk_start.reserve((nbins + 1) * 4);
    b->chunk_hist.reserve(max_chunks * L * 4);
    b->chunk_pos.reserve((max_chunks * L + 1) * 4);
    hipLaunchKernelGGL(k_chunk_setup, dim3(1), dim3(256), 0, st, b->bin_start.as<uint32_t>(), nbins,
                       b->chunk_start.as<uint32_t>());
    GG_HIP(hipGetLastError());
    GG_HIP(hipMemsetAsync(b->chunk_hist.p, 0, max_chunks * L * 4, st));
    hipLaunchKernelGGL(k_chunk_hist, dim3((unsigned)max_chunks), dim3(256), L * 4, st,
                       b->tmp_key.as<uint32_t>(), b->bin_start.as<uint32_t>(),
                       b->chunk_start.as<uint32_t>(), nbins, lowbits, b->chunk_hist.as<uint32_t>());
    GG_HIP(hipGetLastError());
    exclusive_scan(b->chunk_hist.as<uint32_t>(), b->chunk_pos.as<uint32_t>(), max_chunks * L, st,
                   b->scan_tmp);
    hipLaunchKernelGGL(k_chunk_scatter, dim3((unsigned)max_chunks), dim3(256), L * 4, st,
                       b->tmp_entry.as<uint32_t>(), b->tmp_key.as<uint32_t>(),
                       b->bin_start.as<uint32_t>(), b->chunk_start.as<uint32_t>(), nbins, lowbits,
                       b->chunk_pos.as<uint32_t>(), b->sorted.as<uint32_t>());
    GG_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_bucket_offsets, dim3(grid_for((size_t)nbins << lowbits, 256)), dim3(256), 0, st,
                       b->bin_start.as<uint32_t>(), b->chunk_start.as<uint32_t>(),
                       b->chunk_pos.as<uint32_t>(), nbins, lowbits, b->offsets.as<uint32_t>());
    GG_HIP(hipGetLastError());
}

}  // namespace gg
