#include "prof.h"
#include "common.h"
#include <map>
#include <mutex>
#include <vector>
#include <cstring>

namespace gg {
namespace {
struct Acc {
    double ms = 0;
    int64_t n = 0;
    double units = 0;
};
std::mutex g_mu;
std::map<std::string, Acc> g_acc;
bool g_on = false;
}  // namespace

bool prof_on() { return g_on; }

ProfScope::ProfScope(const char* n, hipStream_t st, double u) : name(n), units(u) {
    if (!g_on) return;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
    (void)hipEventRecord(a, st);
    active = true;
}

void ProfScope::stop(hipStream_t st) {
    if (!active) return;
    (void)hipEventRecord(b, st);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    std::lock_guard<std::mutex> lk(g_mu);
    Acc& x = g_acc[name];
    x.ms += ms;
    x.n += 1;
    x.units += units;
    active = false;
}

ProfScope::~ProfScope() {
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
}
}  // namespace gg

extern "C" int gg_profile_enable(int on) {
    std::lock_guard<std::mutex> lk(gg::g_mu);
    gg::g_acc.clear();
    gg::g_on = on != 0;
    return GG_OK;
}

extern "C" int gg_profile_get(const char* name, double* total_ms, int64_t* launches, double* units) {
    std::lock_guard<std::mutex> lk(gg::g_mu);
    auto it = gg::g_acc.find(name ? name : "");
    double ms = 0, u = 0;
    int64_t n = 0;
    if (it != gg::g_acc.end()) { ms = it->second.ms; n = it->second.n; u = it->second.units; }
    if (total_ms) *total_ms = ms;
    if (launches) *launches = n;
    if (units) *units = u;
    return GG_OK;
}
