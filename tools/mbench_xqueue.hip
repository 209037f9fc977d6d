// Does an exchange copy wait for an MSM kernel on another stream? (round-4
// VERDICT "next" 1, DESIGN.md §5 "hardware queues").
//
// HIP maps streams onto at most GPU_MAX_HW_QUEUES (4) hardware queues per
// device; two streams that share a queue are serialised by it.  A one-process
// multi-GPU key creates, per device, the prove streams of every shard's key
// (s0..s4, groth16.hip pk_finish), the shard stream and its copy streams
// (groth16_multi.hip), in that order.  This tool creates streams in a given
// order, starts a long accumulation-shaped kernel (256-thread blocks, two waves
// per SIMD with ~200 VGPRs each, several rounds of blocks) on one of them,
// then a 176-MB device copy (the 8-shard 2^24 exchange-1 push) on another, and
// reports when the copy completes relative to the kernel:
//
//   copy_end_ms   : copy completion, ms after the kernel's start event
//   kernel_ms     : the kernel alone (its start to end events)
//   overlapped    : copy_end_ms < kernel_ms (the copy did not wait)
//
// Variants (one line each):
//   plain-K<k>-X<x>   : S plain streams, kernel on stream k, copy on stream x,
//                       hipMemcpyDeviceToDevice (a blit kernel: needs CU slots)
//   nocu-K<k>-X<x>    : same, hipMemcpyDeviceToDeviceNoCU (SDMA engine)
//   prio-...          : the copy stream created with the greatest priority
//   peer-...          : hipMemcpyPeerAsync (device to itself, the rehearsal)
// Usage: mbench_xqueue [streams=8] [copy_MB=176] [kernel_rounds=12]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

// ~200 live VGPRs, two waves per SIMD: the accumulation's occupancy shape
__global__ void __launch_bounds__(256, 2) k_busy(uint64_t* out, uint32_t iters, uint32_t seed) {
    uint64_t a[48];
#pragma unroll
    for (int i = 0; i < 48; i++) a[i] = (uint64_t)(threadIdx.x * 48 + i) * 0x9e3779b97f4a7c15ull + seed;
    for (uint32_t k = 0; k < iters; k++) {
#pragma unroll
        for (int i = 0; i < 48; i++) a[i] = (a[i] >> 7) * (uint64_t)(uint32_t)a[(i + 5) % 48] + (a[(i + 11) % 48] >> 3);
    }
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 48; i++) s ^= a[i];
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

struct Result {
    float copy_end, kernel, copy_alone;
};

static int g_cus = 256;

static Result run(int S, int kidx, int xidx, int mode, size_t bytes, int rounds, uint32_t iters) {
    std::vector<hipStream_t> st(S);
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    for (int i = 0; i < S; i++) {
        if (i == xidx && mode == 2) CK(hipStreamCreateWithPriority(&st[i], hipStreamNonBlocking, hi));
        else CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    }
    void *src, *dst;
    CK(hipMalloc(&src, bytes));
    CK(hipMalloc(&dst, bytes));
    CK(hipMemset(src, 1, bytes));
    const int blocks = g_cus * 2 * rounds;
    uint64_t* out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 8));
    hipEvent_t k0, k1, x1, c0, c1;
    for (hipEvent_t* e : {&k0, &k1, &x1, &c0, &c1}) CK(hipEventCreate(e));
    auto copy = [&](hipStream_t s) {
        if (mode == 1) CK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDeviceNoCU, s));
        else if (mode == 3) CK(hipMemcpyPeerAsync(dst, 0, src, 0, bytes, s));
        else CK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
    };
    // warm both paths
    hipLaunchKernelGGL(k_busy, dim3(g_cus * 2), dim3(256), 0, st[kidx], out, 16u, 1u);
    copy(st[xidx]);
    CK(hipDeviceSynchronize());
    // the copy alone
    CK(hipEventRecord(c0, st[xidx]));
    copy(st[xidx]);
    CK(hipEventRecord(c1, st[xidx]));
    CK(hipDeviceSynchronize());
    // kernel, then the copy issued right behind its launch on the other stream
    CK(hipEventRecord(k0, st[kidx]));
    hipLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, st[kidx], out, iters, 2u);
    CK(hipGetLastError());
    CK(hipEventRecord(k1, st[kidx]));
    copy(st[xidx]);
    CK(hipEventRecord(x1, st[xidx]));
    CK(hipDeviceSynchronize());
    Result r;
    CK(hipEventElapsedTime(&r.kernel, k0, k1));
    CK(hipEventElapsedTime(&r.copy_end, k0, x1));
    CK(hipEventElapsedTime(&r.copy_alone, c0, c1));
    for (hipEvent_t e : {k0, k1, x1, c0, c1}) CK(hipEventDestroy(e));
    CK(hipFree(out));
    CK(hipFree(src));
    CK(hipFree(dst));
    for (auto s : st) CK(hipStreamDestroy(s));
    return r;
}

int main(int argc, char** argv) {
    const int S = argc > 1 ? atoi(argv[1]) : 8;
    const size_t mb = argc > 2 ? (size_t)atoi(argv[2]) : 176;
    const int rounds = argc > 3 ? atoi(argv[3]) : 12;
    const uint32_t iters = argc > 4 ? (uint32_t)atoi(argv[4]) : 400;
    CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
    const char* q = getenv("GPU_MAX_HW_QUEUES");
    printf("{\"tool\": \"mbench_xqueue\", \"streams\": %d, \"copy_MB\": %zu, \"rounds\": %d, \"cus\": %d, "
           "\"GPU_MAX_HW_QUEUES\": \"%s\"}\n",
           S, mb, rounds, g_cus, q ? q : "unset(4)");
    const char* names[4] = {"plain", "nocu", "prio", "peer"};
    const int pairs[][2] = {{0, 1}, {0, 4}, {1, 5}, {0, S - 1}, {S - 1, 0}};
    for (int mode = 0; mode < 4; mode++)
        for (const auto& p : pairs) {
            if (p[0] >= S || p[1] >= S || p[0] == p[1]) continue;
            const Result r = run(S, p[0], p[1], mode, mb << 20, rounds, iters);
            printf("{\"variant\": \"%s-K%d-X%d\", \"kernel_ms\": %.3f, \"copy_end_ms\": %.3f, \"copy_alone_ms\": %.3f, "
                   "\"overlapped\": %s}\n",
                   names[mode], p[0], p[1], r.kernel, r.copy_end, r.copy_alone,
                   r.copy_end < r.kernel ? "true" : "false");
            fflush(stdout);
        }
    return 0;
}
