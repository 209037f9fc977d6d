// Optional kernel timing with HIP events on the launch stream (gg_profile_*).
#pragma once
#include <hip/hip_runtime.h>
#include <string>

namespace gg {
bool prof_on();
// opaque scope: records a start event on `st` at construction and the stop
// event at stop(); the elapsed time is accumulated under `name` lazily (the
// caller must have synchronized `st` before prof_collect()).
struct ProfScope {
    hipEvent_t a = nullptr, b = nullptr;
    const char* name = nullptr;
    double units = 0;
    bool active = false;
    ProfScope(const char* n, hipStream_t st, double u = 0);
    void stop(hipStream_t st);
    ~ProfScope();
};
}  // namespace gg
