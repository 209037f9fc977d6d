// Witness / fr vector binary format (backend/witness/witness.go:15-36): field
// elements travel as 32-byte big-endian canonical integers
// ([u32 nbPublic | u32 nbSecret | u32 len | len x 32 B]); the prover works on
// gnark-crypto's in-memory layout (Montgomery, little-endian limbs).  These
// elementwise kernels convert between the two on the device (HBM-bound: 64 B of
// traffic per element), with fr.Vector.ReadFrom's range check (value < r).
#include "common.h"
#include "field.cuh"

namespace gg {

template <class C>
__global__ void k_fr_from_be(const uint8_t* in, Fe<C>* out, size_t n, unsigned long long* bad) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* q = reinterpret_cast<const uint4*>(in + 32 * i);
    uint4 a = q[0], b = q[1];
    uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    Fe<C> x;
#pragma unroll
    for (int k = 0; k < 8; k++) x.v[k] = __builtin_bswap32(w[7 - k]);  // big-endian bytes -> LE limbs
    // canonical check: x < modulus
    uint32_t br = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) (void)__builtin_subc(x.v[k], C::P[k], br, &br);
    if (!br) {
        atomicAdd(bad, 1ull);
        x = Fe<C>::zero();
    }
    x = x * Fe<C>::r2();  // to Montgomery
    uint4* o = reinterpret_cast<uint4*>(out + i);
    o[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
    o[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
}

template <class C>
__global__ void k_fr_to_be(const Fe<C>* in, uint8_t* out, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* q = reinterpret_cast<const uint4*>(in + i);
    uint4 a = q[0], b = q[1];
    Fe<C> x;
    x.v[0] = a.x; x.v[1] = a.y; x.v[2] = a.z; x.v[3] = a.w;
    x.v[4] = b.x; x.v[5] = b.y; x.v[6] = b.z; x.v[7] = b.w;
    Fe<C> one = Fe<C>::zero();
    one.v[0] = 1;
    x = x * one;  // from Montgomery
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = __builtin_bswap32(x.v[7 - k]);
    uint4* o = reinterpret_cast<uint4*>(out + 32 * i);
    o[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

}  // namespace gg

using namespace gg;

extern "C" int gg_fr_from_canonical_be(int curve, const void* in_dev, void* out_dev, size_t n,
                                       uint64_t* n_invalid, void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(in_dev && out_dev, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "bad curve");
    // the kernels move 16-B vectors (a raw witness blob + 12 header bytes is not aligned)
    GG_CHECK(((uintptr_t)in_dev & 15) == 0 && ((uintptr_t)out_dev & 15) == 0, GG_ERR_INVALID_ARG,
             "in_dev / out_dev must be 16-byte aligned");
    if (n_invalid) *n_invalid = 0;
    if (n == 0) return GG_OK;
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : hipStreamPerThread;
    DevBuf bad(8);
    GG_HIP(hipMemsetAsync(bad.p, 0, 8, st));
    if (curve == GG_CURVE_BN254)
        hipLaunchKernelGGL(k_fr_from_be<FrCfg>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                           (const uint8_t*)in_dev, (Fr*)out_dev, n, (unsigned long long*)bad.p);
    else
        hipLaunchKernelGGL(k_fr_from_be<FrBlsCfg>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                           (const uint8_t*)in_dev, (FrBls*)out_dev, n, (unsigned long long*)bad.p);
    GG_HIP(hipGetLastError());
    uint64_t nb = 0;
    GG_HIP(hipMemcpyAsync(&nb, bad.p, 8, hipMemcpyDeviceToHost, st));
    GG_WAIT_STREAM(st);
    if (n_invalid) *n_invalid = nb;
    GG_CHECK(nb == 0, GG_ERR_INVALID_ARG, "non-canonical field element (>= modulus) in the vector");
    GG_CAPI_END
}

extern "C" int gg_fr_to_canonical_be(int curve, const void* in_dev, void* out_dev, size_t n,
                                     void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(in_dev && out_dev, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "bad curve");
    GG_CHECK(((uintptr_t)in_dev & 15) == 0 && ((uintptr_t)out_dev & 15) == 0, GG_ERR_INVALID_ARG,
             "in_dev / out_dev must be 16-byte aligned");
    if (n == 0) return GG_OK;
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : hipStreamPerThread;
    if (curve == GG_CURVE_BN254)
        hipLaunchKernelGGL(k_fr_to_be<FrCfg>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                           (const Fr*)in_dev, (uint8_t*)out_dev, n);
    else
        hipLaunchKernelGGL(k_fr_to_be<FrBlsCfg>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                           (const FrBls*)in_dev, (uint8_t*)out_dev, n);
    GG_HIP(hipGetLastError());
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}
