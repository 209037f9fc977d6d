// Microbenchmark: random 64-B / 128-B point gathers over a multi-GB table on
// gfx950 -- the access pattern of the MSM bucket accumulation (each sorted
// entry reads one precomputed affine point, every point exactly once).
// Sweeps table size, loads in flight per lane (prefetch depth D) and waves per
// SIMD (register budget via launch bounds), and an ALU filler of F dependent
// ops per gather so the overlap of gathers with compute can be read off.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>

template <int BYTES>
struct Pt {
    uint4 q[BYTES / 16];
};

template <int BYTES, int D, int WAVES>
__global__ void __launch_bounds__(256, WAVES) k_gather(const Pt<BYTES>* pts, const uint32_t* idx, uint32_t K, size_t E,
                                                       int filler, uint32_t* out) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t e0 = t * K;
    if (e0 >= E) return;
    const size_t e1 = e0 + K < E ? e0 + K : E;
    uint32_t acc = 0, f = (uint32_t)t;
    Pt<BYTES> buf[D];
#pragma unroll
    for (int d = 0; d < D; d++) buf[d] = pts[idx[e0 + d < e1 ? e0 + d : e0]];
    for (size_t e = e0; e < e1; e += D) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            const Pt<BYTES> p = buf[d];
            const size_t en = e + D + d;
            if (en < e1) buf[d] = pts[idx[en]];
#pragma unroll
            for (int i = 0; i < BYTES / 16; i++) acc ^= p.q[i].x + p.q[i].y + p.q[i].z + p.q[i].w;
            for (int k = 0; k < filler; k++) f = f * 1664525u + acc;
        }
    }
    out[t] = acc + f;
}

template <int BYTES, int D, int WAVES>
void run(const void* pts, const uint32_t* idx, size_t E, size_t table, int filler, uint32_t* out) {
    const uint32_t K = 64;
    const size_t T = (E + K - 1) / K;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto launch = [&] {
        hipLaunchKernelGGL((k_gather<BYTES, D, WAVES>), dim3((T + 255) / 256), dim3(256), 0, 0,
                           (const Pt<BYTES>*)pts, idx, K, E, filler, out);
    };
    launch();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; r++) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 3;
    printf("{\"point_bytes\": %d, \"table_GB\": %.2f, \"depth\": %d, \"waves_per_simd\": %d, \"filler\": %d, "
           "\"ms\": %.3f, \"Ggathers_per_s\": %.2f, \"GBps\": %.0f}\n",
           BYTES, table / 1e9, D, WAVES, filler, ms, E / (ms * 1e6), E * (double)BYTES / (ms * 1e6));
    fflush(stdout);
}

int main(int argc, char** argv) {
    const size_t table = (size_t)(argc > 1 ? atof(argv[1]) : 12.9) * 1e9;
    const size_t E = (size_t)(argc > 2 ? atof(argv[2]) : 201e6);
    void* pts;
    if (hipMalloc(&pts, table) != hipSuccess) { printf("alloc failed\n"); return 1; }
    (void)hipMemset(pts, 1, table);
    uint32_t *idx, *out;
    (void)hipMalloc(&idx, E * 4);
    (void)hipMalloc(&out, (E / 64 + 1) * 4);
    const bool quick = argc > 3;
    for (int bytes : {64, 128}) {
        if (quick && bytes == 128) break;
        const size_t npts = table / bytes;
        std::vector<uint32_t> h(E);
        std::mt19937_64 rng(7);
        // every point at most once while E <= npts, like the MSM's entries
        for (size_t i = 0; i < E; i++) h[i] = (uint32_t)(rng() % npts);
        (void)hipMemcpy(idx, h.data(), E * 4, hipMemcpyHostToDevice);
        if (quick) {
            run<64, 1, 2>(pts, idx, E, table, 0, out);
        } else if (bytes == 64) {
            run<64, 1, 2>(pts, idx, E, table, 0, out);
            run<64, 2, 2>(pts, idx, E, table, 0, out);
            run<64, 4, 2>(pts, idx, E, table, 0, out);
            run<64, 1, 4>(pts, idx, E, table, 0, out);
            run<64, 4, 4>(pts, idx, E, table, 0, out);
            run<64, 1, 2>(pts, idx, E, table, 400, out);
            run<64, 2, 2>(pts, idx, E, table, 400, out);
            run<64, 4, 2>(pts, idx, E, table, 400, out);
        } else {
            run<128, 1, 1>(pts, idx, E, table, 0, out);
            run<128, 2, 1>(pts, idx, E, table, 0, out);
            run<128, 1, 2>(pts, idx, E, table, 0, out);
        }
    }
    return 0;
}
