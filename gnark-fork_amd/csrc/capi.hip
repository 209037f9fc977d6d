// C-ABI runtime entry points: errors, devices, memory, host-side point helpers.
#include "common.h"
#include "curve.cuh"
#include <cstring>
#include <atomic>
#include <chrono>
#include <deque>
#include <map>
#include <thread>
#include <mutex>
#include <string>

namespace gg {
static thread_local std::string g_last_error;
void set_last_error(const std::string& m) { g_last_error = m; }
}  // namespace gg

using namespace gg;

std::vector<int> gg::enable_peer_access(const std::vector<int>& devs) {
    const int k = (int)devs.size();
    std::vector<int> code((size_t)k * k, GG_PEER_SAME_DEVICE);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (int i = 0; i < k; i++)
        for (int j = 0; j < k; j++) {
            if (devs[i] == devs[j]) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, devs[i], devs[j]) != hipSuccess || !can) {
                (void)hipGetLastError();
                code[(size_t)i * k + j] = GG_PEER_UNAVAILABLE;
                continue;
            }
            if (hipSetDevice(devs[i]) != hipSuccess) {
                (void)hipGetLastError();
                code[(size_t)i * k + j] = GG_PEER_FAILED;
                continue;
            }
            const hipError_t e = hipDeviceEnablePeerAccess(devs[j], 0);
            if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) {
                code[(size_t)i * k + j] = GG_PEER_ENABLED;
            } else {
                code[(size_t)i * k + j] = GG_PEER_FAILED;
            }
            (void)hipGetLastError();
        }
    (void)hipSetDevice(cur);
    return code;
}

namespace {
std::mutex g_tq_mu;
struct DedQueue {
    hipStream_t s;
    bool used;
};
std::map<int, std::vector<DedQueue>> g_tq;  // device -> its dedicated task queues (CU-masked streams)
int task_queue_cap() {
    const char* e = getenv("GG_TASK_QUEUES");  // read per borrow: tests switch budgets between keys
    return e ? std::max(0, atoi(e)) : 8;
}
// a dedicated queue of `device` (the set grows up to the budget), or null
hipStream_t borrow_task_queue(int device) {
    std::lock_guard<std::mutex> g(g_tq_mu);
    auto& v = g_tq[device];
    int used = 0;
    for (auto& d : v) used += d.used;
    if (used >= task_queue_cap()) return nullptr;
    for (auto& d : v)
        if (!d.used) {
            d.used = true;
            if (gg::trace_streams()) fprintf(stderr, "[gg] borrow dedicated queue %p (device %d)\n", (void*)d.s, device);
            return d.s;
        }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
    for (int c = 0; c < cus; c++) mask[(size_t)c / 32] |= 1u << (c % 32);
    int cur = 0;
    (void)hipGetDevice(&cur);
    hipStream_t s = nullptr;
    const bool ok = hipSetDevice(device) == hipSuccess &&
                    hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) == hipSuccess;
    (void)hipSetDevice(cur);
    if (!ok) {
        (void)hipGetLastError();
        return nullptr;
    }
    v.push_back({s, true});
    if (gg::trace_streams()) fprintf(stderr, "[gg] new dedicated queue %p (device %d, %zu)\n", (void*)s, device, v.size());
    return s;
}
void return_task_queue(hipStream_t s) {
    std::lock_guard<std::mutex> g(g_tq_mu);
    for (auto& kv : g_tq)
        for (auto& d : kv.second)
            if (d.s == s) {
                d.used = false;
                if (gg::trace_streams()) fprintf(stderr, "[gg] return dedicated queue %p\n", (void*)s);
                return;
            }
}
// destroy every dedicated queue of `device` that no task slot holds (all of
// them idle: a returned queue was waited for)
void drop_idle_task_queues(int device) {
    std::lock_guard<std::mutex> g(g_tq_mu);
    auto it = g_tq.find(device);
    if (it == g_tq.end()) return;
    auto& v = it->second;
    for (auto& d : v) if (d.used) return;  // a key still runs on this device's set
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    for (auto& d : v) {
        if (gg::trace_streams()) fprintf(stderr, "[gg] destroy dedicated queue %p (device %d)\n", (void*)d.s, device);
        (void)hipStreamDestroy(d.s);
    }
    v.clear();
    (void)hipSetDevice(cur);
}
void wait_idle(hipStream_t s) {
    GG_WAIT_STREAM(s);                    // bounded
    GG_HIP(hipStreamSynchronize(s));      // returns at once; settles the runtime's view of the stream
}
}  // namespace

// GG_TRACE_STREAMS=1: a stderr line per borrowed / returned dedicated queue
bool gg::trace_streams() {
    static const bool on = getenv("GG_TRACE_STREAMS") && atoi(getenv("GG_TRACE_STREAMS")) == 1;
    return on;
}

void gg::task_streams_init(hipStream_t* const* active, TaskQueue* q, int n, int device, bool dedicated) {
    int cur = 0;
    GG_HIP(hipGetDevice(&cur));
    GG_HIP(hipSetDevice(device));
    for (int i = 0; i < n; i++) {
        if (!q[i].own) GG_HIP(hipStreamCreateWithFlags(&q[i].own, hipStreamNonBlocking));
        q[i].ded = dedicated ? borrow_task_queue(device) : nullptr;
        *active[i] = q[i].ded ? q[i].ded : q[i].own;
    }
    GG_HIP(hipSetDevice(cur));
}

void gg::task_streams_switch(hipStream_t* const* active, TaskQueue* q, int n, int device, bool dedicated) {
    int cur = 0;
    GG_HIP(hipGetDevice(&cur));
    GG_HIP(hipSetDevice(device));
    for (int i = 0; i < n; i++) {
        wait_idle(q[i].own);
        if (q[i].ded) wait_idle(q[i].ded);
    }
    for (int i = 0; i < n; i++)
        if (q[i].ded && !dedicated) {
            return_task_queue(q[i].ded);
            q[i].ded = nullptr;
        }
    for (int i = 0; i < n; i++) {
        if (dedicated && !q[i].ded) q[i].ded = borrow_task_queue(device);
        *active[i] = q[i].ded ? q[i].ded : q[i].own;
    }
    GG_HIP(hipSetDevice(cur));
}

void gg::task_streams_release(TaskQueue* q, int n, int device) {
    for (int i = 0; i < n; i++) {
        if (q[i].ded) {
            (void)hipStreamSynchronize(q[i].ded);
            return_task_queue(q[i].ded);
            q[i].ded = nullptr;
        }
        if (q[i].own) (void)hipStreamDestroy(q[i].own);
        q[i].own = nullptr;
    }
    // the last key on the device gone: its dedicated queues too (as round 5
    // destroyed them with their keys -- none outlives the process's keys, so
    // none is left for the runtime's teardown at exit, which crashed under
    // rocprofv3 --pmc, r06e)
    drop_idle_task_queues(device);
}

extern "C" int gg_release_task_queues(void) {
    GG_CAPI_BEGIN
    std::vector<int> devs;
    {
        std::lock_guard<std::mutex> g(g_tq_mu);
        for (auto& kv : g_tq) devs.push_back(kv.first);
    }
    for (int d : devs) drop_idle_task_queues(d);
    GG_CAPI_END
}

// ---- kept worker threads (common.h run_task)
namespace {
struct WorkerPool {
    std::mutex m;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    int idle = 0;
};
WorkerPool& worker_pool() {
    static WorkerPool* p = new WorkerPool();  // never destroyed: its workers outlive static teardown
    return *p;
}
void pool_worker() {
    WorkerPool& P = worker_pool();
    std::unique_lock<std::mutex> l(P.m);
    for (;;) {
        P.idle++;
        P.cv.wait(l, [&] { return !P.q.empty(); });
        P.idle--;
        std::function<void()> fn = std::move(P.q.front());
        P.q.pop_front();
        l.unlock();
        fn();  // TaskState::run catches everything
        l.lock();
    }
}
}  // namespace

bool gg::pool_enabled() {
    static const bool on = !(getenv("GG_TASK_POOL") && atoi(getenv("GG_TASK_POOL")) == 0);
    return on;
}

void gg::pool_post(std::function<void()> fn) {
    if (!pool_enabled()) {  // A/B: a fresh thread per task, as std::async
        std::thread(std::move(fn)).detach();
        return;
    }
    WorkerPool& P = worker_pool();
    std::lock_guard<std::mutex> l(P.m);
    P.q.push_back(std::move(fn));
    // every queued task has a worker to take it: an idle one, else a new one
    if (P.idle >= (int)P.q.size()) P.cv.notify_one();
    else std::thread(pool_worker).detach();
}

// ---- bounded waits (common.h)
namespace {
std::atomic<double> g_wait_timeout{-1.0};  // < 0: GG_WAIT_TIMEOUT_S or the default
thread_local std::string g_wait_label;
}  // namespace

double gg::wait_timeout_s() {
    const double t = g_wait_timeout.load();
    if (t > 0) return t;
    static const double env = [] {
        const char* e = getenv("GG_WAIT_TIMEOUT_S");
        const double v = e ? atof(e) : 0.0;
        return v > 0 ? v : 300.0;
    }();
    return env;
}

gg::WaitScope::WaitScope(const std::string& label) : prev(g_wait_label) { g_wait_label = label; }
gg::WaitScope::~WaitScope() { g_wait_label = prev; }

namespace {
std::string wait_where(const char* what, const char* fn, int line) {
    std::string w = g_wait_label.empty() ? std::string() : g_wait_label + ": ";
    return w + fn + ":" + std::to_string(line) + " waiting for " + what;
}
// poll q() (hipEventQuery / hipStreamQuery) until it is no longer NotReady: a
// yield loop for the first 2 ms (the latency of hipEventSynchronize's spin), then
// 20-us sleeps, up to the deadline
template <class Q>
void poll_ready(Q q, const char* what, const char* fn, int line) {
    hipError_t e = q();
    if (e == hipErrorNotReady) {
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        const double lim = gg::wait_timeout_s();
        while (e == hipErrorNotReady) {
            const double el = std::chrono::duration<double>(clk::now() - t0).count();
            if (el > lim) {
                char b[64];
                snprintf(b, sizeof b, "timed out after %.0f s: ", el);
                throw gg::Error(GG_ERR_TIMEOUT, b + wait_where(what, fn, line) +
                                                    " (GG_WAIT_TIMEOUT_S / gg_set_wait_timeout)");
            }
            if (el < 0.002) std::this_thread::yield();
            else std::this_thread::sleep_for(std::chrono::microseconds(20));
            e = q();
        }
    }
    if (e != hipSuccess) {
        const int code = e == hipErrorOutOfMemory ? GG_ERR_OOM : GG_ERR_DEVICE;
        throw gg::Error(code, std::string(hipGetErrorString(e)) + " at " + wait_where(what, fn, line));
    }
}
}  // namespace

void gg::wait_event_(hipEvent_t e, const char* what, const char* fn, int line) {
    poll_ready([e] { return hipEventQuery(e); }, what, fn, line);
}
void gg::wait_stream_(hipStream_t s, const char* what, const char* fn, int line) {
    poll_ready([s] { return hipStreamQuery(s); }, what, fn, line);
}

int gg::PartBarrier::wait(const char* what) {
    std::unique_lock<std::mutex> l(mu);
    if (broken) return why.empty() ? GG_ERR_INTERNAL : GG_ERR_TIMEOUT;
    const uint64_t g = gen;
    if (++count == n) {
        count = 0;
        gen++;
        cv.notify_all();
        return GG_OK;
    }
    const auto lim = std::chrono::duration<double>(wait_timeout_s());
    if (!cv.wait_for(l, lim, [&] { return gen != g || broken; })) {
        broken = true;
        char b[96];
        snprintf(b, sizeof b, "timed out after %.0f s at a barrier of %d (%d arrived): ", lim.count(), n, count);
        why = b + wait_where(what, "barrier", 0);
        cv.notify_all();
        set_last_error(why);
        return GG_ERR_TIMEOUT;
    }
    if (broken && !why.empty()) set_last_error(why);
    return broken ? (why.empty() ? GG_ERR_INTERNAL : GG_ERR_TIMEOUT) : GG_OK;
}
void gg::PartBarrier::abort() {
    std::lock_guard<std::mutex> l(mu);
    broken = true;
    cv.notify_all();
}
void gg::PartBarrier::reset() {
    std::lock_guard<std::mutex> l(mu);
    broken = false;
    count = 0;
    why.clear();
}

extern "C" int gg_set_wait_timeout(double seconds) {
    GG_CAPI_BEGIN
    GG_CHECK(seconds >= 0, GG_ERR_INVALID_ARG, "timeout must be >= 0 (0: GG_WAIT_TIMEOUT_S or 300 s)");
    g_wait_timeout.store(seconds > 0 ? seconds : -1.0);
    GG_CAPI_END
}
extern "C" double gg_get_wait_timeout(void) { return gg::wait_timeout_s(); }

// host-only self-test of the bounded barrier (no GPU): `parties` threads are
// expected, `arriving` of them come; with arriving < parties every waiter must
// return GG_ERR_TIMEOUT after timeout_s instead of blocking
extern "C" int gg_wait_selftest(int parties, int arriving, double timeout_s) {
    GG_CAPI_BEGIN
    GG_CHECK(parties >= 1 && parties <= 64 && arriving >= 1 && arriving <= parties && timeout_s > 0,
             GG_ERR_INVALID_ARG, "1 <= arriving <= parties <= 64, timeout_s > 0");
    const double saved = g_wait_timeout.load();
    g_wait_timeout.store(timeout_s);
    gg::PartBarrier bar;
    bar.n = parties;
    std::vector<int> rc(arriving, GG_OK);
    std::vector<std::string> msg(arriving);
    {
        std::vector<std::thread> th;
        for (int i = 0; i < arriving; i++)
            th.emplace_back([&, i] {
                gg::WaitScope ws("selftest part " + std::to_string(i));
                rc[i] = bar.wait("the other parts");
                if (rc[i]) msg[i] = gg_last_error();
            });
        for (auto& t : th) t.join();
    }
    g_wait_timeout.store(saved);
    for (int i = 0; i < arriving; i++) GG_CHECK(rc[i] == GG_OK, rc[i], msg[i]);
    GG_CAPI_END
}

// host-only self-test of the kept worker threads (common.h run_task): n tasks
// that all wait at one barrier (they need n workers at once: the set grows),
// the last of them failing after it; its error comes back through get().  A
// dropped deferred task never runs, a waited one runs once.
extern "C" int gg_task_selftest(int n) {
    GG_CAPI_BEGIN
    GG_CHECK(n >= 1 && n <= 256, GG_ERR_INVALID_ARG, "1 <= n <= 256");
    const double saved = g_wait_timeout.load();
    g_wait_timeout.store(20.0);
    gg::PartBarrier bar;
    bar.n = n;
    std::atomic<int> ran{0};
    std::vector<gg::Task<int>> t;
    for (int i = 0; i < n; i++)
        t.push_back(gg::run_task([i, n, &bar, &ran]() -> int {
            gg::WaitScope ws("selftest task " + std::to_string(i));
            const int rc = bar.wait("the other tasks");
            if (rc) throw gg::Error(rc, gg_last_error());
            ran++;
            if (i == n - 1) throw gg::Error(GG_ERR_INTERNAL, "selftest: the last task fails");
            return i;
        }));
    int code = GG_OK;
    std::string msg;
    for (int i = 0; i < n; i++) {
        try {
            GG_CHECK(t[i].get() == i, GG_ERR_INTERNAL, "selftest: a task returned the wrong value");
        } catch (const gg::Error& e) {
            if (code == GG_OK) {
                code = e.code;
                msg = e.what();
            }
        }
    }
    g_wait_timeout.store(saved);
    GG_CHECK(ran.load() == n, code ? code : GG_ERR_INTERNAL, "selftest: not every task passed the barrier: " + msg);
    GG_CHECK(code == GG_ERR_INTERNAL && msg.find("the last task fails") != std::string::npos, GG_ERR_INTERNAL,
             "selftest: the failing task's error did not come back: " + msg);
    bool dropped_ran = false;
    { auto d = gg::run_task([&dropped_ran] { dropped_ran = true; return 0; }, true); }
    GG_CHECK(!dropped_ran, GG_ERR_INTERNAL, "selftest: a dropped deferred task ran");
    int calls = 0;
    auto w = gg::run_task([&calls] { return ++calls; }, true);
    GG_CHECK(w.get() == 1 && w.get() == 1 && calls == 1, GG_ERR_INTERNAL, "selftest: a deferred task did not run once");
    GG_CAPI_END
}

namespace {
// one wave that sleeps `sleeps` times (s_sleep 127: ~8k cycles each) and
// writes a flag; every wave reaches the end on its own
__global__ void k_sleep_wave(uint32_t sleeps, uint32_t* done) {
    for (uint32_t i = 0; i < sleeps; i++) __builtin_amdgcn_s_sleep(127);
    if (threadIdx.x == 0) done[0] = sleeps;
}
}  // namespace

// the same deadline on a real stream wait: a one-wave kernel that sleeps
// `sleeps` x ~3.4 us on the calling thread's stream, waited for with the
// library's bounded stream wait (GG_WAIT_STREAM) under timeout_s.  The kernel
// always drains before the call returns (it ends on its own), so a timeout here
// leaves nothing in flight
extern "C" int gg_wait_selftest_device(uint32_t sleeps, double timeout_s) {
    GG_CAPI_BEGIN
    GG_CHECK(timeout_s > 0 && sleeps <= (1u << 20), GG_ERR_INVALID_ARG, "timeout_s > 0, sleeps <= 2^20");
    hipStream_t st = hipStreamPerThread;
    DevBuf done(4);
    hipLaunchKernelGGL(k_sleep_wave, dim3(1), dim3(64), 0, st, sleeps, done.as<uint32_t>());
    GG_HIP(hipGetLastError());
    const double saved = g_wait_timeout.load();
    g_wait_timeout.store(timeout_s);
    int rc = GG_OK;
    std::string msg;
    try {
        gg::WaitScope ws("device selftest");
        GG_WAIT_STREAM(st);
    } catch (const gg::Error& e) {
        rc = e.code;
        msg = e.what();
    }
    g_wait_timeout.store(saved);
    GG_HIP(hipStreamSynchronize(st));  // the wave ends by itself: drain before `done` goes
    uint32_t got = 0;
    GG_HIP(hipMemcpy(&got, done.p, 4, hipMemcpyDeviceToHost));
    GG_CHECK(got == sleeps, GG_ERR_INTERNAL, "selftest wave did not finish");
    GG_CHECK(rc == GG_OK, rc, msg);
    GG_CAPI_END
}

extern "C" const char* gg_last_error(void) { return g_last_error.c_str(); }

extern "C" int gg_version(void) { return 100; }  // 0.1.0

extern "C" int gg_build_flags(void) { return kAccumProbe ? GG_BUILD_ACCUM_PROBE : 0; }

extern "C" int gg_device_count(int* count) {
    GG_CAPI_BEGIN
    GG_CHECK(count, GG_ERR_INVALID_ARG, "null argument");
    GG_HIP(hipGetDeviceCount(count));
    GG_CAPI_END
}

extern "C" int gg_set_device(int device) {
    GG_CAPI_BEGIN
    GG_HIP(hipSetDevice(device));
    GG_CAPI_END
}

extern "C" int gg_malloc(void** dev_ptr, size_t bytes) {
    GG_CAPI_BEGIN
    GG_CHECK(dev_ptr, GG_ERR_INVALID_ARG, "null argument");
    GG_HIP(hipMalloc(dev_ptr, bytes ? bytes : 1));
    GG_CAPI_END
}

extern "C" int gg_free(void* dev_ptr) {
    GG_CAPI_BEGIN
    if (dev_ptr) GG_HIP(hipFree(dev_ptr));
    GG_CAPI_END
}

extern "C" int gg_copy_to_device(void* dev_dst, const void* host_src, size_t bytes) {
    GG_CAPI_BEGIN
    if (bytes) GG_HIP(hipMemcpy(dev_dst, host_src, bytes, hipMemcpyHostToDevice));
    GG_CAPI_END
}

extern "C" int gg_copy_to_host(void* host_dst, const void* dev_src, size_t bytes) {
    GG_CAPI_BEGIN
    if (bytes) GG_HIP(hipMemcpy(host_dst, dev_src, bytes, hipMemcpyDeviceToHost));
    GG_CAPI_END
}

extern "C" int gg_copy_device(void* dev_dst, const void* dev_src, size_t bytes) {
    GG_CAPI_BEGIN
    if (bytes) GG_HIP(hipMemcpy(dev_dst, dev_src, bytes, hipMemcpyDeviceToDevice));
    GG_CAPI_END
}

extern "C" int gg_memset_device(void* dev_dst, int value, size_t bytes) {
    GG_CAPI_BEGIN
    if (bytes) GG_HIP(hipMemset(dev_dst, value, bytes));
    GG_CAPI_END
}

extern "C" int gg_synchronize(void) {
    GG_CAPI_BEGIN
    GG_HIP(hipDeviceSynchronize());
    GG_CAPI_END
}

template <class F>
static void jac_to_aff_bytes(const void* jac, void* aff) {
    Jac<F> j;
    memcpy(&j, jac, sizeof(j));
    Affine<F> a = jac_to_affine(j);
    memcpy(aff, &a, sizeof(a));
}

template <class F>
static void jac_add_bytes(const void* a, const void* b, void* out) {
    Jac<F> x, y;
    memcpy(&x, a, sizeof(x));
    memcpy(&y, b, sizeof(y));
    Jac<F> r = jac_add(x, y);
    memcpy(out, &r, sizeof(r));
}

template <class F, class S = Fr>
static void scalar_mul_bytes(const void* p_aff, const void* k_mont, void* out) {
    Affine<F> p;
    memcpy(&p, p_aff, sizeof(p));
    S k;
    memcpy(&k, k_mont, 32);
    S kc = from_mont(k);
    Jac<F> r = jac_mul(Jac<F>::from_affine(p), kc.v);
    memcpy(out, &r, sizeof(r));
}

extern "C" int gg_g1_jac_to_affine(const void* jac, void* aff) {
    GG_CAPI_BEGIN
    GG_CHECK(jac && aff, GG_ERR_INVALID_ARG, "null argument");
    jac_to_aff_bytes<Fp>(jac, aff);
    GG_CAPI_END
}
extern "C" int gg_g2_jac_to_affine(const void* jac, void* aff) {
    GG_CAPI_BEGIN
    GG_CHECK(jac && aff, GG_ERR_INVALID_ARG, "null argument");
    jac_to_aff_bytes<Fp2>(jac, aff);
    GG_CAPI_END
}
extern "C" int gg_g1_jac_add(const void* a, const void* b, void* out) {
    GG_CAPI_BEGIN
    GG_CHECK(a && b && out, GG_ERR_INVALID_ARG, "null argument");
    jac_add_bytes<Fp>(a, b, out);
    GG_CAPI_END
}
extern "C" int gg_g2_jac_add(const void* a, const void* b, void* out) {
    GG_CAPI_BEGIN
    GG_CHECK(a && b && out, GG_ERR_INVALID_ARG, "null argument");
    jac_add_bytes<Fp2>(a, b, out);
    GG_CAPI_END
}
extern "C" int gg_bls12_381_g1_jac_to_affine(const void* jac, void* aff) {
    GG_CAPI_BEGIN
    GG_CHECK(jac && aff, GG_ERR_INVALID_ARG, "null argument");
    jac_to_aff_bytes<FpBls>(jac, aff);
    GG_CAPI_END
}
extern "C" int gg_bls12_381_g1_jac_add(const void* a, const void* b, void* out) {
    GG_CAPI_BEGIN
    GG_CHECK(a && b && out, GG_ERR_INVALID_ARG, "null argument");
    jac_add_bytes<FpBls>(a, b, out);
    GG_CAPI_END
}
extern "C" int gg_g1_scalar_mul(const void* p, const void* k, void* out) {
    GG_CAPI_BEGIN
    GG_CHECK(p && k && out, GG_ERR_INVALID_ARG, "null argument");
    scalar_mul_bytes<Fp>(p, k, out);
    GG_CAPI_END
}
extern "C" int gg_bls12_381_g1_scalar_mul(const void* p, const void* k, void* out) {
    GG_CAPI_BEGIN
    GG_CHECK(p && k && out, GG_ERR_INVALID_ARG, "null argument");
    scalar_mul_bytes<FpBls, FrBls>(p, k, out);
    GG_CAPI_END
}
extern "C" int gg_bls12_381_g2_jac_to_affine(const void* jac, void* aff) {
    GG_CAPI_BEGIN
    GG_CHECK(jac && aff, GG_ERR_INVALID_ARG, "null argument");
    jac_to_aff_bytes<Fp2Bls>(jac, aff);
    GG_CAPI_END
}
extern "C" int gg_bls12_381_g2_jac_add(const void* a, const void* b, void* out) {
    GG_CAPI_BEGIN
    GG_CHECK(a && b && out, GG_ERR_INVALID_ARG, "null argument");
    jac_add_bytes<Fp2Bls>(a, b, out);
    GG_CAPI_END
}
extern "C" int gg_bls12_381_g2_scalar_mul(const void* p, const void* k, void* out) {
    GG_CAPI_BEGIN
    GG_CHECK(p && k && out, GG_ERR_INVALID_ARG, "null argument");
    scalar_mul_bytes<Fp2Bls, FrBls>(p, k, out);
    GG_CAPI_END
}
extern "C" int gg_g2_scalar_mul(const void* p, const void* k, void* out) {
    GG_CAPI_BEGIN
    GG_CHECK(p && k && out, GG_ERR_INVALID_ARG, "null argument");
    scalar_mul_bytes<Fp2>(p, k, out);
    GG_CAPI_END
}
