// Shared runtime plumbing: error propagation into the C ABI, HIP checks,
// device buffers with RAII.
#pragma once
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>
#include <cstdio>
#include <vector>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <type_traits>
#include "../../include/gnark_amd.h"

// -DGG_ACCUM_PROBE=1 builds a traffic-attribution variant (build_var/, never
// the product library): the MSM accumulation reads its points from <= 1024
// cached entries, so its sums are wrong.  gg_build_flags() reports it and the
// provers of such a build return GG_REHEARSAL, never GG_OK.
#ifndef GG_ACCUM_PROBE
#define GG_ACCUM_PROBE 0
#endif

namespace gg {

constexpr bool kAccumProbe = GG_ACCUM_PROBE != 0;

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& m);

#define GG_HIP(x)                                                                         \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            int code_ = (e_ == hipErrorOutOfMemory) ? GG_ERR_OOM : GG_ERR_DEVICE;         \
            throw ::gg::Error(code_, std::string(#x) + " failed: " + hipGetErrorString(e_) + \
                                         " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
        }                                                                                 \
    } while (0)

#define GG_CHECK(cond, code, msg)                       \
    do {                                                \
        if (!(cond)) throw ::gg::Error((code), (msg));  \
    } while (0)

// a probe build's results are wrong by design: every entry point that returns
// MSM sums or proof parts ends with this instead of GG_OK
#define GG_PROBE_GUARD()                                                                         \
    do {                                                                                         \
        if (::gg::kAccumProbe) {                                                                 \
            ::gg::set_last_error("traffic-probe build (GG_ACCUM_PROBE): the MSM sums are wrong"); \
            return GG_REHEARSAL;                                                                 \
        }                                                                                        \
    } while (0)

#define GG_CAPI_BEGIN try {
#define GG_CAPI_END                                      \
    return GG_OK;                                        \
    }                                                    \
    catch (const ::gg::Error& e) {                       \
        ::gg::set_last_error(e.what());                  \
        return e.code;                                   \
    }                                                    \
    catch (const std::bad_alloc&) {                      \
        ::gg::set_last_error("host out of memory");      \
        return GG_ERR_OOM;                               \
    }                                                    \
    catch (const std::exception& e) {                    \
        ::gg::set_last_error(e.what());                  \
        return GG_ERR_INTERNAL;                          \
    }

// owning device buffer
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    explicit DevBuf(size_t b) { alloc(b); }
    void alloc(size_t b) {
        release();
        if (b) GG_HIP(hipMalloc(&p, b));
        bytes = b;
    }
    // grow-only
    void reserve(size_t b) {
        if (b > bytes) alloc(b);
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
    ~DevBuf() { release(); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; bytes = o.bytes; o.p = nullptr; o.bytes = 0; }
        return *this;
    }
};

// bump allocator over one device buffer: per-task scratch that is reused across
// calls (no hipMalloc / hipFree -- which synchronise the device -- inside a
// prove).  get() hands out 256-B aligned slices; reset() recycles them all.
struct Arena {
    DevBuf buf;
    size_t off = 0;
    void reserve(size_t b) {
        if (b > buf.bytes) buf.alloc(b);
        off = 0;
    }
    void reset() { off = 0; }
    template <class T>
    T* get(size_t count) {
        const size_t b = (count * sizeof(T) + 255) & ~(size_t)255;
        GG_CHECK(off + b <= buf.bytes, GG_ERR_INTERNAL, "device arena overflow");
        T* p = reinterpret_cast<T*>((char*)buf.p + off);
        off += b;
        return p;
    }
};

inline bool is_device_ptr(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

// XCD-aware block swizzle (bijective for any nwg): consecutive logical blocks run
// on one XCD (blocks b and b + 8 share an XCD under round-robin dispatch), so
// neighbouring blocks' partial-line writes merge in that XCD's L2.  Speed only.
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t bid, uint32_t nwg) {
    const uint32_t q = nwg >> 3, r = nwg & 7, x = bid & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// Enables xGMI peer access from every listed device to every other one and
// returns the outcome per ordered pair (i, j) as GG_PEER_* codes (row-major,
// devs.size()^2): a pair whose access failed still copies, staged through host
// memory by the runtime, so callers report it (capi.hip).
std::vector<int> enable_peer_access(const std::vector<int>& devs);

// A stream for copies that must not wait behind kernels of other streams: HIP
// maps the streams of a device round-robin onto GPU_MAX_HW_QUEUES (4) hardware
// queues per priority, and a queue runs its packets in order -- with 8 streams
// the 5th shares the 1st's queue and a copy on it waits for the 1st's MSM
// kernel (tools/mbench_xqueue, profiles/r05_a_xqueue.txt: 6.3 ms instead of
// 0.1 ms behind a 6-ms kernel).  Streams of the greatest priority live in their
// own queues, so copies on them start at once whatever the compute streams run.
inline void create_copy_stream(hipStream_t* s) {
    int lo = 0, hi = 0;
    GG_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    GG_HIP(hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi));
}

// The compute streams of a prove's concurrent tasks.  HIP maps a device's
// streams onto 4 hardware queues per priority, so with 5 tasks on 4 queues two
// tasks share a queue and the second one's kernels wait for the first one's
// whole chain (the 8-shard Groth16 trace, profiles/r05_g_groth16_shard0.md: the
// G2 accumulation started 7 ms late behind the A-MSM's reduction).  A stream
// with a CU mask (all CUs here) gets a hardware queue of its own (r05_b_xqueue2).
// Each task slot (TaskQueue) has a plain stream of its own, created once with
// its key, and while the device has one to give a DEDICATED queue borrowed from
// the process's per-device set: at most GG_TASK_QUEUES (default 8) CU-masked
// streams per device and process, created on first use and never destroyed.
// Handing the dedicated queues from one key (shard, part) to another -- the
// timing rehearsals -- is a pointer swap between idle streams: no stream is
// created or destroyed then.  (Round 6: re-creating streams in the rehearsal
// stalled inside hipStreamDestroy of a pool stream after CU-masked streams had
// been destroyed, profiles/r06_d_restream_stall.md, the r05k stall's pattern.)
struct TaskQueue {
    hipStream_t own = nullptr;  // plain non-blocking stream of the slot (the key's)
    hipStream_t ded = nullptr;  // borrowed dedicated queue, or null
};
// active[i] <- slot i's stream: dedicated if `dedicated` and the budget allows
void task_streams_init(hipStream_t* const* active, TaskQueue* q, int n, int device, bool dedicated);
// between proofs: wait until the slots' streams are idle, return / borrow the
// dedicated queues, repoint active[] (never creates or destroys a stream)
void task_streams_switch(hipStream_t* const* active, TaskQueue* q, int n, int device, bool dedicated);
// the key goes away: dedicated queues back to the set, own streams destroyed;
// a device's set is destroyed once no key holds any of it
void task_streams_release(TaskQueue* q, int n, int device);
bool trace_streams();

// ---- bounded host waits (round 6, VERDICT r5: a stall must end in an error,
// not a hang).  Every wait of the library's host threads for GPU work or for
// another part / shard of a proof has a deadline: gg_set_wait_timeout or
// GG_WAIT_TIMEOUT_S (seconds, default 300).  Past it the wait throws GG_ERR_TIMEOUT
// naming what it waited for and the thread's WaitScope (part, stage).
double wait_timeout_s();
void wait_event_(hipEvent_t e, const char* what, const char* fn, int line);
void wait_stream_(hipStream_t s, const char* what, const char* fn, int line);
#define GG_WAIT_EVENT(e) ::gg::wait_event_((e), #e, __func__, __LINE__)
#define GG_WAIT_STREAM(s) ::gg::wait_stream_((s), #s, __func__, __LINE__)
// the calling thread's part of a proof, for timeout messages ("part 3: ratio")
struct WaitScope {
    std::string prev;
    explicit WaitScope(const std::string& label);
    ~WaitScope();
};
// A reusable barrier of n host threads that a failing thread breaks (abort) and
// whose wait gives up at the wait deadline (the Groth16 one-process exchanges).
struct PartBarrier {
    std::mutex mu;
    std::condition_variable cv;
    int n = 1, count = 0;
    uint64_t gen = 0;
    bool broken = false;
    std::string why;  // set when broken by a timeout
    // GG_OK, GG_ERR_INTERNAL (broken by a peer) or GG_ERR_TIMEOUT (this wait or a peer's timed out)
    int wait(const char* what);
    void abort();
    void reset();
};

// ---- host tasks on kept worker threads (round 6).  The provers start a host
// thread per concurrent task (a Groth16 MSM, a PlonK part's slice MSM, the ratio
// slice of a part, ...): std::async made a fresh thread each time, which pays the
// thread's creation and the HIP runtime's per-thread set-up before its first
// launch -- on the critical path of every stage hand-over.  run_task posts the
// task to a process-wide set of workers instead, which grows whenever no worker
// is idle (a task that waits for another task never starves) and keeps its
// threads.  The task runs on the submitting thread's current device.  Task<R>
// keeps std::async's contract: get() rethrows the task's exception, and the
// last copy of a Task waits for the task when it goes away, so a task may refer
// to its caller's locals.  GG_TASK_POOL=0: a fresh thread per task (A/B).
bool pool_enabled();
void pool_post(std::function<void()> fn);
template <class R>
struct TaskState {
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    std::exception_ptr ex;
    std::function<void()> deferred;  // run by the first waiter (deferred tasks)
    typename std::conditional<std::is_void<R>::value, char, R>::type val{};
    void wait() {
        std::function<void()> d;
        {
            std::unique_lock<std::mutex> l(m);
            if (!deferred) {
                cv.wait(l, [&] { return done; });
                return;
            }
            d.swap(deferred);
        }
        d();
    }
    // the last handle goes: wait for a started task, drop a deferred one (as a
    // std::async future does)
    void release() {
        std::unique_lock<std::mutex> l(m);
        if (deferred) {
            deferred = nullptr;
            return;
        }
        cv.wait(l, [&] { return done; });
    }
    template <class Fn>
    void run(Fn& fn) {
        try {
            if constexpr (std::is_void<R>::value) fn();
            else val = fn();
        } catch (...) {
            ex = std::current_exception();
        }
        {
            std::lock_guard<std::mutex> l(m);
            done = true;
        }
        cv.notify_all();
    }
};
template <class R>
class Task {
    struct Guard {
        std::shared_ptr<TaskState<R>> st;
        ~Guard() {
            if (st) st->release();
        }
    };
    std::shared_ptr<Guard> g_;

   public:
    Task() = default;
    explicit Task(std::shared_ptr<TaskState<R>> st) : g_(new Guard{std::move(st)}) {}
    bool valid() const { return (bool)g_; }
    void wait() const { g_->st->wait(); }
    R get() const {
        wait();
        if (g_->st->ex) std::rethrow_exception(g_->st->ex);
        if constexpr (!std::is_void<R>::value) return g_->st->val;
    }
    Task share() const { return *this; }
};
// fn on a kept worker (deferred: on the first get() / wait(), the serial modes)
template <class Fn>
auto run_task(Fn fn, bool deferred = false) -> Task<decltype(fn())> {
    using R = decltype(fn());
    auto st = std::make_shared<TaskState<R>>();
    if (deferred) {
        TaskState<R>* raw = st.get();  // the state outlives its waiters' calls
        st->deferred = [raw, fn]() mutable { raw->run(fn); };
    } else {
        int dev = 0;
        (void)hipGetDevice(&dev);
        auto job = [st, fn, dev]() mutable {
            (void)hipSetDevice(dev);
            st->run(fn);
        };
        pool_post(std::function<void()>(std::move(job)));
    }
    return Task<R>(st);
}

inline unsigned grid_for(size_t n, unsigned block) {
    size_t g = (n + block - 1) / block;
    return (unsigned)(g ? g : 1);
}

}  // namespace gg
