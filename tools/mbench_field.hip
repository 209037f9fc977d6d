// Microbenchmark: BN254 Fp Montgomery multiplication throughput on gfx950
// (product-scanning asm form vs portable CIOS), plus raw v_mad_u64_u32 rate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../gnark-fork_amd/csrc/field29.cuh"
using namespace gg;

template <class C>
__device__ __forceinline__ Fe<C> mul_cios(const Fe<C>& a, const Fe<C>& b) {
    uint32_t t[8];
#pragma unroll
    for (int j = 0; j < 8; j++) t[j] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t acc = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) { acc = (uint64_t)a.v[j] * b.v[i] + t[j] + (acc >> 32); t[j] = (uint32_t)acc; }
        uint32_t t8 = (uint32_t)(acc >> 32);
        uint32_t m = t[0] * C::INV;
        acc = (uint64_t)m * C::P[0] + t[0];
#pragma unroll
        for (int j = 1; j < 8; j++) { acc = (uint64_t)m * C::P[j] + t[j] + (acc >> 32); t[j - 1] = (uint32_t)acc; }
        t[7] = t8 + (uint32_t)(acc >> 32);
    }
    Fe<C> r, s; uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = __builtin_subc(t[i], C::P[i], br, &br);
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = br ? t[i] : s.v[i];
    return r;
}

// radix-29 product with the column shift done on 32-bit halves (v_alignbit_b32
// + v_lshrrev_b32 in asm, so the compiler cannot fold it back into a 64-bit shift)
__device__ __forceinline__ uint64_t shr29(uint64_t acc) {
    uint32_t lo = (uint32_t)acc, hi = (uint32_t)(acc >> 32), nlo, nhi;
    asm volatile("v_alignbit_b32 %0, %2, %3, 29\n\tv_lshrrev_b32 %1, 29, %2" : "=v"(nlo), "=v"(nhi) : "v"(hi), "v"(lo));
    return ((uint64_t)nhi << 32) | nlo;
}
__device__ __forceinline__ Fp29 mul_alt(const Fp29& a, const Fp29& b) {
    constexpr int N = 9;
    uint32_t m[N];
    Fp29 r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k - 1 : N - 1); i++) acc += (uint64_t)m[i] * Fp29Cfg::P[k - i];
        if (k < N) {
            m[k] = ((uint32_t)acc * Fp29Cfg::INV) & Fp29Cfg::MASK;
            acc += (uint64_t)m[k] * Fp29Cfg::P[0];
        } else {
            r.l[k - N] = (uint32_t)acc & Fp29Cfg::MASK;
        }
        acc = shr29(acc);
    }
    r.l[N - 1] = (uint32_t)acc;
    return r;
}

template <int V>
__global__ void __launch_bounds__(256) k_mulchain(Fp* data, int iters) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    Fp a = data[2 * i], b = data[2 * i + 1], c = a, d = b;
    if (V == 3) {  // radix 29 with 32-bit column shifts
        Fp29 a2 = unpack29(to_r261(a)), b2 = unpack29(to_r261(b)), c2 = a2, d2 = b2;
        for (int k = 0; k < iters; k++) { a2 = mul_alt(a2, b2); c2 = mul_alt(c2, d2); b2 = mul_alt(b2, a2); d2 = mul_alt(d2, c2); }
        data[2 * i] = to_std(a2) + to_std(c2); data[2 * i + 1] = to_std(b2) + to_std(d2);
        return;
    }
    if (V == 2) {  // 29-bit reduced-radix form (field29.cuh)
        Fp29 a2 = unpack29(to_r261(a)), b2 = unpack29(to_r261(b)), c2 = a2, d2 = b2;
        for (int k = 0; k < iters; k++) { a2 = mul(a2, b2); c2 = mul(c2, d2); b2 = mul(b2, a2); d2 = mul(d2, c2); }
        if (iters == 7) { a2 = sqr(a2); c2 = mul(c2, c2); a2 = mul(a2, c2); c2 = sqr(c2); }
        data[2 * i] = to_std(a2) + to_std(c2); data[2 * i + 1] = to_std(b2) + to_std(d2);
        return;
    }
    for (int k = 0; k < iters; k++) {
        if (V == 0) { a = mul_cios(a, b); c = mul_cios(c, d); b = mul_cios(b, a); d = mul_cios(d, c); }
        else { a = a * b; c = c * d; b = b * a; d = d * c; }
    }
    if (iters == 7) { a = a * a; c = c * c; a = a * c; c = c * c; }
    data[2 * i] = a + c; data[2 * i + 1] = b + d;
}

// single-wave latency probe: one wave, dependent chain
template <int V>
__global__ void k_latency(Fp* data, int iters) {
    Fp a = data[threadIdx.x], b = data[64 + threadIdx.x];
    for (int k = 0; k < iters; k++) { if (V == 0) a = mul_cios(a, b); else a = a * b; }
    data[threadIdx.x] = a;
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

// pure v_mad_u64_u32 throughput: 16 independent accumulators; MIX adds 16
// independent 32-bit add chains per iteration (do they co-issue with the mads?)
template <int MIX>
__global__ void __launch_bounds__(256) k_mad_tp(uint64_t* out, int iters) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a[16], b = (uint32_t)i ^ 0x9e3779b9u;
    uint64_t x[16];
    uint32_t y[16];
#pragma unroll
    for (int j = 0; j < 16; j++) a[j] = (uint32_t)i * 2654435761u + j;
#pragma unroll
    for (int j = 0; j < 16; j++) { x[j] = i + j; y[j] = (uint32_t)i ^ (j * 77u); }
    for (int k = 0; k < iters; k++) {
#pragma unroll
        for (int j = 0; j < 16; j++) asm volatile("" : "+v"(a[j]));
#pragma unroll
        for (int j = 0; j < 16; j++) {
            x[j] = (uint64_t)a[j] * b + x[j];
            if (MIX) asm volatile("v_add_u32 %0, %0, %1\n\tv_xor_b32 %0, %0, %2" : "+v"(y[j]) : "v"(a[j]), "v"(b));
        }
    }
    uint64_t r = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) r ^= x[j] + y[j];
    out[i] = r;
}

int main() {
    const int blocks = 256 * 16, threads = 256;
    size_t n = (size_t)blocks * threads;
    std::vector<Fp> h(2 * n);
    for (size_t i = 0; i < 2 * n; i++) for (int l = 0; l < 8; l++) h[i].v[l] = (uint32_t)(i * 2654435761u + l * 40503u) & (l == 7 ? 0x0fffffffu : 0xffffffffu);
    Fp* d; (void)hipMalloc(&d, 2 * n * sizeof(Fp));
    Fp* d2; (void)hipMalloc(&d2, 2 * n * sizeof(Fp));
    (void)hipMemcpy(d, h.data(), 2 * n * sizeof(Fp), hipMemcpyHostToDevice);
    (void)hipMemcpy(d2, h.data(), 2 * n * sizeof(Fp), hipMemcpyHostToDevice);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    int iters = 256;
    float ms;
    for (int rep = 0; rep < 3; rep++) {
        k_mulchain<0><<<blocks, threads>>>(d, 4);
        (void)hipEventRecord(e0); k_mulchain<0><<<blocks, threads>>>(d, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("{\"variant\": \"cios\", \"fp_mont_mul_per_s\": %.4e}\n", (double)n * iters * 4 / (ms * 1e-3));
        k_mulchain<1><<<blocks, threads>>>(d2, 4);
        (void)hipEventRecord(e0); k_mulchain<1><<<blocks, threads>>>(d2, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("{\"variant\": \"product_scanning\", \"fp_mont_mul_per_s\": %.4e}\n", (double)n * iters * 4 / (ms * 1e-3));
    }
    Fp* d3; (void)hipMalloc(&d3, 2 * n * sizeof(Fp));
    (void)hipMemcpy(d3, h.data(), 2 * n * sizeof(Fp), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; rep++) {
        k_mulchain<2><<<blocks, threads>>>(d3, 4);
        (void)hipEventRecord(e0); k_mulchain<2><<<blocks, threads>>>(d3, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("{\"variant\": \"radix29\", \"fp_mont_mul_per_s\": %.4e}\n", (double)n * iters * 4 / (ms * 1e-3));
    }
    {
        Fp* d4; (void)hipMalloc(&d4, 2 * n * sizeof(Fp));
        (void)hipMemcpy(d4, h.data(), 2 * n * sizeof(Fp), hipMemcpyHostToDevice);
        for (int rep = 0; rep < 3; rep++) {
            k_mulchain<3><<<blocks, threads>>>(d4, 4);
            (void)hipEventRecord(e0); k_mulchain<3><<<blocks, threads>>>(d4, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("{\"variant\": \"radix29_shift32\", \"fp_mont_mul_per_s\": %.4e}\n", (double)n * iters * 4 / (ms * 1e-3));
        }
    }
    // equality of the variants on the same data
    (void)hipMemcpy(d, h.data(), 2 * n * sizeof(Fp), hipMemcpyHostToDevice);
    (void)hipMemcpy(d2, h.data(), 2 * n * sizeof(Fp), hipMemcpyHostToDevice);
    (void)hipMemcpy(d3, h.data(), 2 * n * sizeof(Fp), hipMemcpyHostToDevice);
    k_mulchain<0><<<blocks, threads>>>(d, 7); k_mulchain<1><<<blocks, threads>>>(d2, 7); k_mulchain<2><<<blocks, threads>>>(d3, 7);
    {
        std::vector<Fp> r1(2 * n), r3(2 * n);
        (void)hipMemcpy(r1.data(), d, 2 * n * sizeof(Fp), hipMemcpyDeviceToHost);
        (void)hipMemcpy(r3.data(), d3, 2 * n * sizeof(Fp), hipMemcpyDeviceToHost);
        size_t diff = 0; for (size_t i = 0; i < 2 * n; i++) diff += !(r1[i] == r3[i]);
        printf("{\"radix29_differs\": %zu}\n", diff);
    }
    std::vector<Fp> r1(2 * n), r2(2 * n);
    (void)hipMemcpy(r1.data(), d, 2 * n * sizeof(Fp), hipMemcpyDeviceToHost);
    (void)hipMemcpy(r2.data(), d2, 2 * n * sizeof(Fp), hipMemcpyDeviceToHost);
    size_t diff = 0; for (size_t i = 0; i < 2 * n; i++) diff += !(r1[i] == r2[i]);
    printf("{\"variants_differ\": %zu}\n", diff);
    for (int v = 0; v < 2; v++) {
        (void)hipEventRecord(e0);
        if (v == 0) k_latency<0><<<1, 64>>>(d, 2000); else k_latency<1><<<1, 64>>>(d, 2000);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
        printf("{\"variant\": \"%s\", \"single_wave_mul_latency_ns\": %.1f}\n", v ? "product_scanning" : "cios", ms * 1e6 / 2000);
    }
    uint64_t* o; (void)hipMalloc(&o, n * 8);
    k_mad<<<blocks, threads>>>(o, 4);
    (void)hipEventRecord(e0); k_mad<<<blocks, threads>>>(o, 4096); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("{\"mad_u64_u32_per_s\": %.4e}\n", (double)n * 4096 * 8 / (ms * 1e-3));
    for (int mix = 0; mix < 2; mix++) {
        for (int rep = 0; rep < 2; rep++) {
            if (mix) k_mad_tp<1><<<blocks, threads>>>(o, 4); else k_mad_tp<0><<<blocks, threads>>>(o, 4);
            (void)hipEventRecord(e0);
            if (mix) k_mad_tp<1><<<blocks, threads>>>(o, 2048); else k_mad_tp<0><<<blocks, threads>>>(o, 2048);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("{\"mad_tp_mix\": %d, \"mad_per_s\": %.4e, \"wave_cycles_per_iter_at_2.4GHz\": %.1f}\n", mix,
                   (double)n * 2048 * 16 / (ms * 1e-3), ms * 1e-3 * 2.4e9 * 1024 / ((double)n / 64 * 2048));
        }
    }
    return 0;
}
