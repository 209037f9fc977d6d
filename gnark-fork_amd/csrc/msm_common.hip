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
