// Non-template MSM kernels: scalar digits, counting sort, scan, work items.
#include "msm_impl.cuh"

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

// digits[w*n + i]: signed digit of scalar i in window w; histogram into counts
__global__ void k_digits(const Fr* scalars, const uint32_t* sidx, size_t n, int c, int W,
                         int32_t* digits, uint32_t* counts) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr s = ld(scalars + (sidx ? sidx[i] : i));
    Fr k = from_mont(s);
    int carry = 0;
    const int half = 1 << (c - 1);
    for (int w = 0; w < W; w++) {
        int d = (int)extract_bits(k, w * c, c) + carry;
        if (d > half) { d -= (1 << c); carry = 1; } else carry = 0;
        digits[(size_t)w * n + i] = d;
        if (d) atomicAdd(&counts[(d > 0 ? d : -d) - 1], 1u);
    }
}

__global__ void k_scatter(const int32_t* digits, size_t total, uint32_t* cursor, uint32_t* sorted) {
    size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    int d = digits[e];
    if (!d) return;
    uint32_t b = (uint32_t)((d > 0 ? d : -d) - 1);
    uint32_t pos = atomicAdd(&cursor[b], 1u);
    sorted[pos] = (uint32_t)e | (d < 0 ? 0x80000000u : 0u);
}

// items per bucket = ceil(cnt / K)
__global__ void k_item_counts(const uint32_t* offsets, size_t nb, int K, uint32_t* itemcnt,
                              uint32_t* maxcnt) {
    size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v = 0;
    if (b < nb) {
        uint32_t cnt = offsets[b + 1] - offsets[b];
        v = (cnt + K - 1) / K;
        itemcnt[b] = v;
    }
    // wave max then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
    if ((threadIdx.x & 63) == 0 && v) atomicMax(maxcnt, v);
}

__global__ void k_item_buckets(const uint32_t* item_off, size_t nb, uint32_t* item_bucket) {
    size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    for (uint32_t t = item_off[b]; t < item_off[b + 1]; t++) item_bucket[t] = (uint32_t)b;
}

int choose_c(size_t n, size_t point_bytes) {
    int best = 4;
    double bc = 1e300;
    for (int c = 4; c <= 23; c++) {
        int W = (255 + c - 1) / c;
        double mem = (double)W * (double)n * (double)point_bytes;
        if (mem > 48e9) continue;  // precomputed table budget per base
        double cost = (double)n * W + (double)(1u << (c - 1)) * 2.8;
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

constexpr int SORT_SPB = 1024;  // scalars per block in A / C (256 threads x 4)

__global__ void __launch_bounds__(256) k_digits_hist(const Fr* scalars, const uint32_t* sidx,
                                                     size_t n, int c, int W, int hshift, int nbins,
                                                     uint32_t* keys, uint32_t* hist,
                                                     uint32_t nblocks) {
    extern __shared__ uint32_t h[];
    for (int j = threadIdx.x; j < nbins; j += blockDim.x) h[j] = 0;
    __syncthreads();
    const int half = 1 << (c - 1);
    for (int s = 0; s < SORT_SPB / 256; s++) {
        size_t i = (size_t)blockIdx.x * SORT_SPB + s * 256 + threadIdx.x;
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
                atomicAdd(&h[bk >> hshift], 1u);
            }
            keys[(size_t)w * n + i] = key;
        }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < nbins; j += blockDim.x) hist[(size_t)j * nblocks + blockIdx.x] = h[j];
}

__global__ void __launch_bounds__(256) k_bin_scatter(const uint32_t* keys, size_t n, int W, int hshift,
                                                     int nbins, const uint32_t* hoff, uint32_t nblocks,
                                                     uint32_t* tmp_entry, uint32_t* tmp_key) {
    extern __shared__ uint32_t cur[];
    for (int j = threadIdx.x; j < nbins; j += blockDim.x) cur[j] = hoff[(size_t)j * nblocks + blockIdx.x];
    __syncthreads();
    for (int s = 0; s < SORT_SPB / 256; s++) {
        size_t i = (size_t)blockIdx.x * SORT_SPB + s * 256 + threadIdx.x;
        if (i >= n) break;
        for (int w = 0; w < W; w++) {
            size_t e = (size_t)w * n + i;
            uint32_t key = keys[e];
            if (key == 0xffffffffu) continue;
            uint32_t bk = key & 0x7fffffffu;
            uint32_t pos = atomicAdd(&cur[bk >> hshift], 1u);
            tmp_entry[pos] = (uint32_t)e | (key & 0x80000000u);
            tmp_key[pos] = bk;
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

__global__ void __launch_bounds__(1024) k_bin_sort(const uint32_t* tmp_entry, const uint32_t* tmp_key,
                                                   const uint32_t* bin_start, int lowbits, int nbins,
                                                   uint32_t* sorted, uint32_t* offsets) {
    extern __shared__ uint32_t sm[];
    const int nk = 1 << lowbits;
    uint32_t* cnt = sm;          // nk
    uint32_t* part = sm + nk;    // 1024
    const uint32_t mask = (uint32_t)nk - 1;
    const int bin = blockIdx.x;
    const uint32_t lo = bin_start[bin], hi = bin_start[bin + 1];
    for (int j = threadIdx.x; j < nk; j += blockDim.x) cnt[j] = 0;
    __syncthreads();
    for (uint32_t e = lo + threadIdx.x; e < hi; e += blockDim.x) atomicAdd(&cnt[tmp_key[e] & mask], 1u);
    __syncthreads();
    // exclusive scan of cnt[0..nk): thread t owns a contiguous chunk
    const int per = (nk + 1023) / 1024;
    const int c0 = threadIdx.x * per;
    uint32_t s = 0;
    for (int k = 0; k < per; k++)
        if (c0 + k < nk) s += cnt[c0 + k];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        uint32_t x = (threadIdx.x >= (unsigned)off) ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += x;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
    for (int k = 0; k < per; k++) {
        int j = c0 + k;
        if (j < nk) {
            uint32_t v = cnt[j];
            cnt[j] = run;  // becomes the cursor
            offsets[((size_t)bin << lowbits) + j] = lo + run;
            run += v;
        }
    }
    if (bin == nbins - 1 && threadIdx.x == 0) offsets[(size_t)nbins << lowbits] = hi;
    __syncthreads();
    for (uint32_t e = lo + threadIdx.x; e < hi; e += blockDim.x) {
        uint32_t pos = atomicAdd(&cnt[tmp_key[e] & mask], 1u);
        sorted[lo + pos] = tmp_entry[e];
    }
}

void sort_entries(gg_msm_base* b, const Fr* scalars_dev, hipStream_t st) {
    const size_t n = b->n, nb = b->nb;
    const int c = b->c, W = b->W;
    const size_t total = (size_t)W * n;
    const int h = std::min(8, c - 1);
    const int nbins = 1 << h;
    const int lowbits = (c - 1) - h;
    const uint32_t nblocks = (uint32_t)((n + SORT_SPB - 1) / SORT_SPB);
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
                       b->has_sidx ? b->sidx.as<uint32_t>() : nullptr, n, c, W, lowbits, nbins,
                       b->keys.as<uint32_t>(), b->hist.as<uint32_t>(), nblocks);
    GG_HIP(hipGetLastError());
    exclusive_scan(b->hist.as<uint32_t>(), b->hoff.as<uint32_t>(), nh, st, b->scan_tmp);
    hipLaunchKernelGGL(k_bin_starts, dim3(grid_for(nbins, 256)), dim3(256), 0, st,
                       b->hoff.as<uint32_t>(), b->hist.as<uint32_t>(), nblocks, nbins,
                       b->bin_start.as<uint32_t>());
    GG_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_bin_scatter, dim3(nblocks), dim3(256), nbins * 4, st, b->keys.as<uint32_t>(),
                       n, W, lowbits, nbins, b->hoff.as<uint32_t>(), nblocks,
                       b->tmp_entry.as<uint32_t>(), b->tmp_key.as<uint32_t>());
    GG_HIP(hipGetLastError());
    size_t lds = ((size_t)(1 << lowbits) + 1024) * 4;
    hipLaunchKernelGGL(k_bin_sort, dim3(nbins), dim3(1024), lds, st, b->tmp_entry.as<uint32_t>(),
                       b->tmp_key.as<uint32_t>(), b->bin_start.as<uint32_t>(), lowbits, nbins,
                       b->sorted.as<uint32_t>(), b->offsets.as<uint32_t>());
    GG_HIP(hipGetLastError());
}

}  // namespace gg
