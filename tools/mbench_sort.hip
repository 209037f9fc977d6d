// Microbenchmark: rocPRIM radix_sort_pairs on MSM-shaped keys (13.6M entries,
// 19-bit bucket ids) -- reference point for the hand-written bucket sort.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <vector>
#include <random>

int main() {
    const size_t n = 13ull << 20;
    const int bits = 19;
    std::vector<uint32_t> hk(n), hv(n);
    std::mt19937 rng(1);
    for (size_t i = 0; i < n; i++) { hk[i] = rng() & ((1u << bits) - 1); hv[i] = (uint32_t)i; }
    uint32_t *k0, *k1, *v0, *v1;
    (void)hipMalloc(&k0, n * 4); (void)hipMalloc(&k1, n * 4); (void)hipMalloc(&v0, n * 4); (void)hipMalloc(&v1, n * 4);
    (void)hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice);
    size_t tmp_bytes = 0;
    (void)rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0, k1, v0, v1, n, 0, bits);
    void* tmp; (void)hipMalloc(&tmp, tmp_bytes);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 5; rep++) {
        (void)hipEventRecord(e0);
        (void)rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, k1, v0, v1, n, 0, bits);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("{\"rocprim_radix_sort_pairs_ms\": %.4f, \"n\": %zu, \"bits\": %d}\n", ms, n, bits);
    }
    return 0;
}
