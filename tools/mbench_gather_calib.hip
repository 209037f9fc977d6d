// FETCH_SIZE calibration for the MSM accumulation's access widths
// (MI355X_MICROARCH.md "HBM": "Other access widths are uncalibrated: calibrate
// on a known byte count in your own access pattern").
//
// One dispatch per pattern, each over a table of argv[1] GiB (default 4; >> the
// 256 MiB Infinity Cache; 16 covers the 12.9-GB G1 tables of the 2^24 key, where
// address translation of random gathers costs extra fetches), every byte read
// exactly once:
//   k_stream16   : 16 B per lane, coalesced (the guide's calibrated case: raw = 1/2)
//   k_gather<64> : 64-B points gathered through a shuffled permutation (G1 BN254)
//   k_gather<128>: 128-B points, same (G2 BN254 / the G2 accumulation)
//   k_gather<96> : 96-B points (BLS12-381 G1)
// The permutation (4 B per point) is read coalesced by the gathers too, so
// known bytes = table + 4 * points.  Run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/mbench_gather_calib
// and divide the known bytes by FETCH_SIZE x 1024 per dispatch.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

template <int BYTES>
struct Pt {
    uint32_t w[BYTES / 4];
};

__global__ void k_stream16(const uint4* p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x + v.y + v.z + v.w;
    }
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int BYTES>
__global__ void k_gather(const Pt<BYTES>* pts, const uint32_t* idx, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const Pt<BYTES> p = pts[idx[i]];
#pragma unroll
        for (int k = 0; k < BYTES / 4; k++) acc ^= p.w[k];
    }
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int BYTES>
static void gather(const void* tab, size_t table, uint32_t* idx, uint32_t* out, int grid) {
    const size_t n = table / BYTES;
    std::vector<uint32_t> h(n);
    std::iota(h.begin(), h.end(), 0u);
    std::shuffle(h.begin(), h.end(), std::mt19937_64(BYTES));
    (void)hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_gather<BYTES>, dim3(grid), dim3(256), 0, 0, (const Pt<BYTES>*)tab, idx, n, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("{\"kernel\": \"k_gather<%d>\", \"points\": %zu, \"known_bytes\": %zu, \"ms\": %.3f}\n", BYTES, n,
           n * BYTES + n * 4, ms);
}

int main(int argc, char** argv) {
    const size_t gib = argc > 1 ? (size_t)atoi(argv[1]) : 4;
    const size_t table = gib << 30;
    printf("{\"table_bytes\": %zu}\n", table);
    void* tab;
    uint32_t *idx, *out;
    const int grid = 256 * 8 * 4;
    if (hipMalloc(&tab, table) != hipSuccess || hipMalloc(&idx, (table / 64) * 4) != hipSuccess ||
        hipMalloc(&out, (size_t)grid * 256 * 4) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(tab, 1, table);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(256), 0, 0, (const uint4*)tab, table / 16, out);
    (void)hipDeviceSynchronize();
    printf("{\"kernel\": \"k_stream16\", \"known_bytes\": %zu}\n", table);
    gather<64>(tab, table, idx, out, grid);
    gather<96>(tab, table - table % 96, idx, out, grid);
    gather<128>(tab, table, idx, out, grid);
    return 0;
}
