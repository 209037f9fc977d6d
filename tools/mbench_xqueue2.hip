// Exchange copies vs a long MSM kernel, timed from the host the way the
// library waits for them (hipStreamSynchronize on the copy stream, as
// groth16_multi.hip mpk_exchange does) -- round-4 VERDICT "next" 1.
//
// A kernel shaped like the G1 accumulation (256-thread blocks, ~225 VGPRs, two
// waves per SIMD, several rounds of blocks) runs on stream K; right behind its
// launch a 176-MB copy (the 8-shard 2^24 exchange-1 push) is issued on stream
// X.  The host then synchronises X and records when that returned and whether
// K was still running (hipStreamQuery), then synchronises K.
//
// Stream setups (S streams created, kernel on the first, copy on the last
// unless said otherwise -- with S > GPU_MAX_HW_QUEUES (4) some share a queue):
//   plain   : hipStreamCreateWithFlags for all
//   prio    : the copy stream with the greatest priority
//   cumask  : the copy stream from hipExtStreamCreateWithCUMask (all CUs)
//   first   : the copy stream created FIRST, then the others
// Copy kinds: d2d (hipMemcpyDeviceToDevice: a blit kernel, needs CU slots),
// nocu (hipMemcpyDeviceToDeviceNoCU: the SDMA engines), peer
// (hipMemcpyPeerAsync device -> itself, what a one-GPU rehearsal issues).
// Also: 7 pushes of 25 MB (an 8-way exchange) on one stream vs 7 streams,
// with no kernel running, per copy kind.
// Usage: mbench_xqueue2 [S=8] [copy_MB=176] [rounds=12] [iters=400]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

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

static int g_cus = 256;
using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
}

enum Setup { PLAIN, PRIO, CUMASK, FIRST };
enum Kind { D2D, NOCU, PEER };
static const char* setup_name[] = {"plain", "prio", "cumask", "first"};
static const char* kind_name[] = {"d2d", "nocu", "peer"};

static void make_streams(int S, Setup su, std::vector<hipStream_t>& st, int& kidx, int& xidx) {
    st.assign(S, nullptr);
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    xidx = S - 1;
    kidx = 0;
    if (su == FIRST) {
        xidx = 0;
        kidx = S - 1;
    }
    for (int i = 0; i < S; i++) {
        if (i == xidx && su == PRIO) {
            CK(hipStreamCreateWithPriority(&st[i], hipStreamNonBlocking, hi));
        } else if (i == xidx && su == CUMASK) {
            std::vector<uint32_t> mask((g_cus + 31) / 32, 0xffffffffu);
            CK(hipExtStreamCreateWithCUMask(&st[i], (uint32_t)mask.size(), mask.data()));
        } else {
            CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
        }
    }
}

static void copy(void* dst, const void* src, size_t bytes, Kind k, hipStream_t s) {
    if (k == NOCU) CK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDeviceNoCU, s));
    else if (k == PEER) CK(hipMemcpyPeerAsync(dst, 0, src, 0, bytes, s));
    else CK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
}

int main(int argc, char** argv) {
    const int S = argc > 1 ? atoi(argv[1]) : 8;
    const size_t bytes = (size_t)(argc > 2 ? atoi(argv[2]) : 176) << 20;
    const int rounds = argc > 3 ? atoi(argv[3]) : 12;
    const uint32_t iters = argc > 4 ? (uint32_t)atoi(argv[4]) : 400;
    CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
    const char* q = getenv("GPU_MAX_HW_QUEUES");
    printf("{\"tool\": \"mbench_xqueue2\", \"streams\": %d, \"copy_MB\": %zu, \"rounds\": %d, \"cus\": %d, "
           "\"GPU_MAX_HW_QUEUES\": \"%s\"}\n",
           S, bytes >> 20, rounds, g_cus, q ? q : "unset");
    void *src, *dst;
    CK(hipMalloc(&src, bytes));
    CK(hipMalloc(&dst, bytes));
    CK(hipMemset(src, 1, bytes));
    const int blocks = g_cus * 2 * rounds;
    uint64_t* out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 8));
    for (int su = 0; su < 4; su++)
        for (int kd = 0; kd < 3; kd++) {
            std::vector<hipStream_t> st;
            int ki, xi;
            make_streams(S, (Setup)su, st, ki, xi);
            // warm: kernel alone, copy alone (timed from the host)
            hipLaunchKernelGGL(k_busy, dim3(g_cus * 2), dim3(256), 0, st[ki], out, 16u, 1u);
            copy(dst, src, bytes, (Kind)kd, st[xi]);
            CK(hipDeviceSynchronize());
            auto a = clk::now();
            copy(dst, src, bytes, (Kind)kd, st[xi]);
            CK(hipStreamSynchronize(st[xi]));
            const double copy_alone = ms(a, clk::now());
            a = clk::now();
            hipLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, st[ki], out, iters, 2u);
            CK(hipStreamSynchronize(st[ki]));
            const double kernel_alone = ms(a, clk::now());
            // kernel, then the copy right behind its launch
            a = clk::now();
            hipLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, st[ki], out, iters, 3u);
            CK(hipGetLastError());
            copy(dst, src, bytes, (Kind)kd, st[xi]);
            CK(hipStreamSynchronize(st[xi]));
            const double copy_done = ms(a, clk::now());
            const hipError_t kq = hipStreamQuery(st[ki]);
            const bool kernel_running = kq == hipErrorNotReady;
            CK(hipStreamSynchronize(st[ki]));
            const double kernel_done = ms(a, clk::now());
            (void)hipGetLastError();
            printf("{\"setup\": \"%s\", \"kind\": \"%s\", \"copy_alone_ms\": %.3f, \"kernel_alone_ms\": %.3f, "
                   "\"copy_done_ms\": %.3f, \"kernel_done_ms\": %.3f, \"kernel_still_running_at_copy_done\": %s}\n",
                   setup_name[su], kind_name[kd], copy_alone, kernel_alone, copy_done, kernel_done,
                   kernel_running ? "true" : "false");
            fflush(stdout);
            for (auto s : st) CK(hipStreamDestroy(s));
        }
    // an 8-way exchange: 7 pushes of bytes / 7, one stream vs seven streams, no kernel
    const size_t part = bytes / 7;
    for (int kd = 0; kd < 3; kd++)
        for (int nst : {1, 7}) {
            std::vector<hipStream_t> st(nst);
            for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            for (int rep = 0; rep < 2; rep++) {
                auto a = clk::now();
                for (int j = 0; j < 7; j++)
                    copy((char*)dst + j * part, (const char*)src + j * part, part, (Kind)kd, st[j % nst]);
                for (auto s : st) CK(hipStreamSynchronize(s));
                if (rep)
                    printf("{\"pushes\": 7, \"MB_each\": %.1f, \"kind\": \"%s\", \"streams\": %d, \"ms\": %.3f}\n",
                           part / 1e6, kind_name[kd], nst, ms(a, clk::now()));
            }
            fflush(stdout);
            for (auto s : st) CK(hipStreamDestroy(s));
        }
    CK(hipFree(out));
    CK(hipFree(src));
    CK(hipFree(dst));
    return 0;
}
