// Microbenchmark: BN254 Fp Montgomery multiplication throughput on gfx950,
// plus raw v_mad_u64_u32 throughput, to calibrate the MSM/NTT rooflines.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../gnark-fork_amd/csrc/field.cuh"
using namespace gg;

__global__ void __launch_bounds__(256) k_mulchain(Fp* data, int iters) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    Fp a = data[2 * i], b = data[2 * i + 1], c = a, d = b;
    for (int k = 0; k < iters; k++) { a = a * b; c = c * d; b = b * a; d = d * c; }
    data[2 * i] = a + c; data[2 * i + 1] = b + d;
}

__global__ void __launch_bounds__(256) k_mad(uint64_t* out, int iters) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a = (uint32_t)i * 2654435761u + 1, b = a ^ 0x9e3779b9u;
    uint64_t x0 = i, x1 = i + 1, x2 = i + 2, x3 = i + 3, x4 = 5, x5 = 6, x6 = 7, x7 = 8;
    for (int k = 0; k < iters; k++) {
        x0 = (uint64_t)a * b + x0; x1 = (uint64_t)b * a + x1; x2 = (uint64_t)a * a + x2; x3 = (uint64_t)b * b + x3;
        x4 = (uint64_t)(a + 1) * b + x4; x5 = (uint64_t)b * (a + 3) + x5; x6 = (uint64_t)(a ^ 5) * a + x6; x7 = (uint64_t)(b ^ 7) * b + x7;
        a ^= (uint32_t)x0; b += (uint32_t)(x1 >> 32);
    }
    out[i] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
}

int main() {
    const int blocks = 256 * 16, threads = 256;
    size_t n = (size_t)blocks * threads;
    std::vector<Fp> h(2 * n);
    for (size_t i = 0; i < 2 * n; i++) for (int l = 0; l < 8; l++) h[i].v[l] = (uint32_t)(i * 2654435761u + l * 40503u) & (l == 7 ? 0x0fffffffu : 0xffffffffu);
    Fp* d; hipMalloc(&d, 2 * n * sizeof(Fp));
    hipMemcpy(d, h.data(), 2 * n * sizeof(Fp), hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    int iters = 256;
    k_mulchain<<<blocks, threads>>>(d, 4);
    hipEventRecord(e0);
    k_mulchain<<<blocks, threads>>>(d, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double muls = (double)n * iters * 4;
    printf("{\"fp_mont_mul_per_s\": %.4e, \"ms\": %.3f}\n", muls / (ms * 1e-3), ms);
    uint64_t* o; hipMalloc(&o, n * 8);
    k_mad<<<blocks, threads>>>(o, 4);
    hipEventRecord(e0);
    k_mad<<<blocks, threads>>>(o, 4096);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double mads = (double)n * 4096 * 8;
    printf("{\"mad_u64_u32_per_s\": %.4e, \"ms\": %.3f}\n", mads / (ms * 1e-3), ms);
    return 0;
}
