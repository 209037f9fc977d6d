// Host-side cost of starting GPU work from a fresh std::thread (what each
// std::async(launch::async) task of the provers pays) against a thread that
// already ran HIP calls: spawn -> hipSetDevice -> one empty kernel enqueued on a
// shared stream, timed on the host, 200 rounds each.  tools/gpu_r06n.sh
#include <hip/hip_runtime.h>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <thread>
#include <vector>
#include <algorithm>

__global__ void k_empty(int* p) { if (threadIdx.x == 0 && p) p[0] = 1; }

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    if (hipSetDevice(0) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
    if (hipStreamSynchronize(s) != hipSuccess) return 1;
    const int R = 200;
    std::vector<double> fresh, warm;
    for (int r = 0; r < R; r++) {
        const double t0 = now_us();
        double t1 = 0;
        std::thread th([&] {
            (void)hipSetDevice(0);
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
            t1 = now_us();
        });
        th.join();
        fresh.push_back(t1 - t0);
        (void)hipStreamSynchronize(s);
    }
    // one persistent worker fed through a condition variable
    std::mutex mu;
    std::condition_variable cv, done_cv;
    bool go = false, done = false, quit = false;
    double t0 = 0, t1 = 0;
    std::thread w([&] {
        for (;;) {
            std::unique_lock<std::mutex> l(mu);
            cv.wait(l, [&] { return go || quit; });
            if (quit) return;
            go = false;
            l.unlock();
            (void)hipSetDevice(0);
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
            t1 = now_us();
            l.lock();
            done = true;
            done_cv.notify_one();
        }
    });
    for (int r = 0; r < R; r++) {
        std::unique_lock<std::mutex> l(mu);
        t0 = now_us();
        go = true;
        done = false;
        cv.notify_one();
        done_cv.wait(l, [&] { return done; });
        warm.push_back(t1 - t0);
        l.unlock();
        (void)hipStreamSynchronize(s);
    }
    {
        std::lock_guard<std::mutex> l(mu);
        quit = true;
    }
    cv.notify_one();
    w.join();
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    auto p90 = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() * 9 / 10]; };
    printf("fresh thread: median %.1f us, p90 %.1f us; persistent worker: median %.1f us, p90 %.1f us (%d rounds)\n",
           med(fresh), p90(fresh), med(warm), p90(warm), R);
    (void)hipStreamDestroy(s);
    return 0;
}
