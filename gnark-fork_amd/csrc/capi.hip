// C-ABI runtime entry points: errors, devices, memory, host-side point helpers.
#include "common.h"
#include "curve.cuh"
#include <cstring>
#include <map>
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
std::map<int, int> g_tq_used;                // device -> dedicated task queues in use
std::map<hipStream_t, int> g_tq_streams;     // dedicated stream -> its device
}  // namespace

void gg::create_task_stream(hipStream_t* s, int device) {
    int cap = 8;
    if (const char* e = getenv("GG_TASK_QUEUES")) cap = std::max(0, atoi(e));
    std::lock_guard<std::mutex> g(g_tq_mu);
    if (g_tq_used[device] < cap) {
        int cus = 0;
        GG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
        for (int c = 0; c < cus; c++) mask[(size_t)c / 32] |= 1u << (c % 32);
        if (hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data()) == hipSuccess) {
            g_tq_used[device]++;
            g_tq_streams[*s] = device;
            return;
        }
        (void)hipGetLastError();
    }
    GG_HIP(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
}

void gg::destroy_task_stream(hipStream_t s) {
    if (!s) return;
    {
        std::lock_guard<std::mutex> g(g_tq_mu);
        auto it = g_tq_streams.find(s);
        if (it != g_tq_streams.end()) {
            g_tq_used[it->second]--;
            g_tq_streams.erase(it);
        }
    }
    (void)hipStreamDestroy(s);
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
