// Fixed-base batch scalar multiplication out[i] = k_i * B on the GPU:
// replaces curve.BatchScalarMultiplicationG1/G2 used by Setup
// (setup.go:240-251, 306-318) and by the prover for [r,s,kr]*delta (prove.go:192).
//
// 8-bit fixed-base comb: T[w][j] = j * 2^(8w) * B (32 x 256 affine points, built
// on the host once per call), every scalar is 32 table lookups + 31 mixed XYZZ
// additions; the XYZZ results are batch-normalised to affine on the device.
#include "common.h"
#include "curve.cuh"
#include "msm_impl.cuh"
#include <vector>
#include <cstring>

namespace gg {

template <class F, class SC>
__global__ void __launch_bounds__(256) k_comb(const Affine<F>* table, const Fe<SC>* scalars, size_t n,
                                              Xyzz<F>* out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fe<SC> k = from_mont(ld(scalars + i));
    Xyzz<F> acc = Xyzz<F>::inf();
    for (int w = 0; w < 32; w++) {
        uint32_t j = (k.v[w >> 2] >> ((w & 3) * 8)) & 0xffu;
        if (j) acc = xyzz_madd(acc, ld(table + w * 256 + j));
    }
    st(out + i, acc);
}

// batch-normalise with infinity support (k = 0 -> all-zero affine)
template <class F>
__global__ void __launch_bounds__(256) k_normalize_inf(const Xyzz<F>* cur, size_t n, size_t T,
                                                       F* prefix, Affine<F>* out) {
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T || t >= n) return;
    F acc = F::one();
    for (size_t i = t; i < n; i += T) {
        st(prefix + i, acc);
        Xyzz<F> p = ld(cur + i);
        if (!p.is_inf()) acc = acc * p.zzz;
    }
    F inv = inverse(acc);
    size_t last = t + ((n - 1 - t) / T) * T;
    for (size_t i = last;; i -= T) {
        Xyzz<F> p = ld(cur + i);
        if (p.is_inf()) {
            st(out + i, Affine<F>::inf());
        } else {
            F izzz = inv * ld(prefix + i);
            inv = inv * p.zzz;
            F izz = sqr(izzz) * sqr(p.zz);
            st(out + i, Affine<F>{p.x * izz, p.y * izzz});
        }
        if (i < T) break;
    }
}

// host: T[w][j] = j * 2^(8w) * B, affine (batch inversion on the host)
template <class F>
static std::vector<Affine<F>> build_comb_table(const Affine<F>& base) {
    std::vector<Jac<F>> J(32 * 256);
    Jac<F> bw = Jac<F>::from_affine(base);
    for (int w = 0; w < 32; w++) {
        J[w * 256] = Jac<F>::inf();
        for (int j = 1; j < 256; j++) J[w * 256 + j] = jac_add(J[w * 256 + j - 1], bw);
        for (int s = 0; s < 8; s++) bw = jac_dbl(bw);
    }
    // Montgomery batch inversion of the Z coordinates
    std::vector<F> pre(J.size());
    F acc = F::one();
    for (size_t i = 0; i < J.size(); i++) {
        pre[i] = acc;
        if (!J[i].is_inf()) acc = acc * J[i].z;
    }
    F inv = inverse(acc);
    std::vector<Affine<F>> T(J.size());
    for (size_t i = J.size(); i-- > 0;) {
        if (J[i].is_inf()) { T[i] = Affine<F>::inf(); continue; }
        F zi = inv * pre[i];
        inv = inv * J[i].z;
        F zi2 = sqr(zi);
        T[i] = Affine<F>{J[i].x * zi2, J[i].y * zi2 * zi};
    }
    return T;
}

template <class F, class SC>
static void batch_mul(const void* base_aff, const void* scalars, size_t n, int scalars_on_device,
                      void* out, int out_on_device) {
    Affine<F> base;
    memcpy(&base, base_aff, sizeof(base));
    hipStream_t st = hipStreamPerThread;
    auto table = build_comb_table<F>(base);
    DevBuf dtab(table.size() * sizeof(Affine<F>));
    GG_HIP(hipMemcpyAsync(dtab.p, table.data(), dtab.bytes, hipMemcpyHostToDevice, st));
    DevBuf dsc;
    const Fe<SC>* sdev = (const Fe<SC>*)scalars;
    if (!scalars_on_device) {
        dsc.alloc(n * 32);
        GG_HIP(hipMemcpyAsync(dsc.p, scalars, n * 32, hipMemcpyHostToDevice, st));
        sdev = dsc.as<Fe<SC>>();
    }
    DevBuf cur(n * sizeof(Xyzz<F>)), prefix(n * sizeof(F));
    DevBuf dout;
    Affine<F>* o = (Affine<F>*)out;
    if (!out_on_device) {
        dout.alloc(n * sizeof(Affine<F>));
        o = dout.as<Affine<F>>();
    }
    hipLaunchKernelGGL((k_comb<F, SC>), dim3(grid_for(n, 256)), dim3(256), 0, st,
                       (const Affine<F>*)dtab.p, sdev, n, cur.as<Xyzz<F>>());
    GG_HIP(hipGetLastError());
    const size_t T = std::min<size_t>(n, std::max<size_t>(16384, n / 64));
    hipLaunchKernelGGL(k_normalize_inf<F>, dim3(grid_for(T, 256)), dim3(256), 0, st,
                       (const Xyzz<F>*)cur.p, n, T, prefix.as<F>(), o);
    GG_HIP(hipGetLastError());
    if (!out_on_device)
        GG_HIP(hipMemcpyAsync(out, o, n * sizeof(Affine<F>), hipMemcpyDeviceToHost, st));
    GG_WAIT_STREAM(st);
}

}  // namespace gg

using namespace gg;

extern "C" int gg_batch_scalar_mul(int group, const void* base_aff, const void* scalars, size_t n,
                                   int scalars_on_device, void* out_aff, int out_on_device) {
    GG_CAPI_BEGIN
    GG_CHECK(base_aff && out_aff, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(group == GG_G1 || group == GG_G2 || group == GG_BLS12_381_G1 || group == GG_BLS12_381_G2,
             GG_ERR_INVALID_ARG, "bad group");
    if (n == 0) return GG_OK;
    GG_CHECK(scalars, GG_ERR_INVALID_ARG, "null scalars");
    if (group == GG_G1) batch_mul<Fp, FrCfg>(base_aff, scalars, n, scalars_on_device, out_aff, out_on_device);
    else if (group == GG_G2) batch_mul<Fp2, FrCfg>(base_aff, scalars, n, scalars_on_device, out_aff, out_on_device);
    else if (group == GG_BLS12_381_G1) batch_mul<FpBls, FrBlsCfg>(base_aff, scalars, n, scalars_on_device, out_aff, out_on_device);
    else batch_mul<Fp2Bls, FrBlsCfg>(base_aff, scalars, n, scalars_on_device, out_aff, out_on_device);
    GG_CAPI_END
}
