// PlonK BLS12-381 quotient-path kernels, BLS12-381 fr
// (32 B Montgomery, R = 2^256) in gnark-crypto's memory layout.
//
//   gg_plonk_numerator_coset  allConstraints of computeNumerator on one coset of
//                             the big domain + the bit-reversed scatter into cres
//                             (backend/plonk/bls12-381/prove.go:850-935, 1030-1041)
//   gg_plonk_divide_by_xn_minus_one
//                             r[i] *= (x^n - 1)^-1 on the big coset, then the big
//                             coset iFFT (DIT: bit-reversed in, canonical regular
//                             out) -- divideByXMinusOne, prove.go:1223-1276
//   gg_bls12_381_fr_batch_invert
//                             fr.BatchInvert (prove.go:1273): zeros stay zero
#include "plonk_ops.h"
#include "prof.h"
#include <vector>
#include <cstring>
#include <type_traits>

namespace gg {
void any_ntt_inplace(gg_domain* d, void* data, int inverse, int dit, int coset, hipStream_t st);
size_t domain_size(gg_domain* d, int* curve);
void xn_minus_one_inv(gg_domain* big, size_t n_small, void* out);
}  // namespace gg

namespace gg {
namespace plk {

template <class F>
__device__ __forceinline__ F ldf(const F* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    F r;
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    return r;
}
template <class F>
__device__ __forceinline__ void stf(F* p, const F& r) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(r.v[0], r.v[1], r.v[2], r.v[3]);
    q[1] = make_uint4(r.v[4], r.v[5], r.v[6], r.v[7]);
}

// sum c[k] x^k: nc - 1 products (the leading coefficient starts the chain)
template <class F>
__device__ __forceinline__ F horner_d(const F* c, int nc, const F& x) {
    if (nc <= 0) return F::zero();
    F r = c[nc - 1];
    for (int k = nc - 2; k >= 0; k--) r = r * x + c[k];
    return r;
}

// allConstraints at point j of the coset (prove.go:928-954)
template <class F>
__device__ __forceinline__ F numerator_at(const NumParamsT<F>& P, uint32_t j) {
    const F one = F::one();
    F L = ldf(P.x[ID_L] + j), R = ldf(P.x[ID_R] + j), O = ldf(P.x[ID_O] + j);
    F Z = ldf(P.x[ID_Z] + j);
    const uint32_t j1 = j + 1 == P.n ? 0 : j + 1;
    F ZS = P.x[ID_ZS] ? ldf(P.x[ID_ZS] + (P.zs_shift ? j1 : j)) : ldf(P.x[ID_Z] + j1);
    F S1 = ldf(P.x[ID_S1] + j) * P.beta, S2 = ldf(P.x[ID_S2] + j) * P.beta,
        S3 = ldf(P.x[ID_S3] + j) * P.beta;
    // blinding: bl/br/bo/bz evaluated at twiddles0[j], bz at twiddles0[(j+1) % n] for ZS
    const F t0 = ldf(P.tw0 + j), t1 = P.tw1 ? ldf(P.tw1 + j) : ldf(P.tw0 + j1);
    L = L + horner_d(P.bcoef[0], P.bdeg[0], t0);
    R = R + horner_d(P.bcoef[1], P.bdeg[1], t0);
    O = O + horner_d(P.bcoef[2], P.bdeg[2], t0);
    Z = Z + horner_d(P.bcoef[3], P.bdeg[3], t0);
    ZS = ZS + horner_d(P.bcoef[3], P.bdeg[3], t1);
    // gateConstraint
    // ql L + qm L R = L (ql + qm R): four products instead of five
    F ic = L * (ldf(P.x[ID_QL] + j) + ldf(P.x[ID_QM] + j) * R) + ldf(P.x[ID_QR] + j) * R;
    ic = ic + ldf(P.x[ID_QO] + j) * O + ldf(P.x[ID_QK] + j);
    for (int q = ID_QCI; q + 1 < P.nx; q += 2) ic = ic + ldf(P.x[q] + j) * ldf(P.x[q + 1] + j);
    // orderingConstraint
    const F id = ldf(P.x[ID_ID] + j);
    F a = P.gamma + L + id * P.ka, b = id * P.kb + R + P.gamma, c = id * P.kc + O + P.gamma;
    F r = a * b * c * Z;
    a = S1 + L + P.gamma;
    b = S2 + R + P.gamma;
    c = S3 + O + P.gamma;
    F l = a * b * c * ZS - r;
    // ratioLocalConstraint
    F rl = (Z - one) * ldf(P.x[ID_LONE] + j);
    const F res = (rl * P.alpha + l) * P.alpha + ic;
    return P.has_out_scale ? res * P.out_scale : res;
}

// small domains: one point per thread, cres[bitrev(rho*j + coset)] (prove.go:1036-1038)
template <class F>
__global__ void __launch_bounds__(256) k_numerator_coset(NumParamsT<F> P) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= P.n) return;
    const F res = numerator_at(P, j);
    uint32_t pos = P.log_big ? __brev(P.rho * j + P.coset) >> (32 - P.log_big) : 0u;
    if (P.local_block) pos &= P.n - 1;
    stf(P.cres + pos, res);
}

// n >= 256: 16 x 16 tiles.  Thread t of block m computes j = h 2^(L-4) + 16 m + l
// (h = t >> 4, l = t & 15): rows of 16 consecutive j, coalesced loads.  With
// rho = 2^r the cres slot is
//   bitrev_{L+r}(rho j + coset) = brev_r(coset) << L | brev4(l) << (L-4)
//                                 | brev_{L-8}(m) << 4 | brev4(h),
// so for each l the 16 values of h fill 16 consecutive slots: the results are
// transposed through LDS and stored as 16 runs of 512 B (not 256 scattered 32-B
// writes).
template <class F>
__global__ void __launch_bounds__(256) k_numerator_coset_tiled(NumParamsT<F> P, uint32_t log_n) {
    __shared__ uint32_t tile[8][256 + 8];  // limb-major, padded
    const uint32_t t = threadIdx.x, h = t >> 4, l = t & 15, m = blockIdx.x;
    const uint32_t j = (h << (log_n - 4)) | (m << 4) | l;
    const F res = numerator_at(P, j);
    const uint32_t slot = l * 16 + (__brev(h) >> 28);
#pragma unroll
    for (int k = 0; k < 8; k++) tile[k][slot + (slot >> 5)] = res.v[k];
    __syncthreads();
    const uint32_t r = P.log_big - log_n;
    const uint32_t l2 = t >> 4, col = t & 15;
    const uint32_t pos = (r && !P.local_block ? (__brev(P.coset) >> (32 - r)) << log_n : 0u) |
                         ((__brev(l2) >> 28) << (log_n - 4)) |
                         (log_n > 8 ? (__brev(m) >> (40 - log_n)) << 4 : 0u) | col;
    F o;
#pragma unroll
    for (int k = 0; k < 8; k++) o.v[k] = tile[k][t + (t >> 5)];
    stf(P.cres + pos, o);
}

template <class F>
struct PeriodicTab {
    F f[8];
};
template <class F>
__global__ void k_mul_periodic_bitrev(F* r, size_t n, int log_n, PeriodicTab<F> t, uint32_t rho) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t irev = log_n ? (__brev((uint32_t)i) >> (32 - log_n)) : 0u;
    stf(r + i, ldf(r + i) * t.f[irev % rho]);
}

// Montgomery batch inversion: thread t owns elements t, t+T, ... (zeros skipped)
template <class F>
__global__ void __launch_bounds__(256) k_batch_invert(F* a, size_t n, size_t T, F* prefix) {
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T || t >= n) return;
    F acc = F::one();
    for (size_t i = t; i < n; i += T) {
        stf(prefix + i, acc);
        F x = ldf(a + i);
        if (!x.is_zero()) acc = acc * x;
    }
    F inv = inverse(acc);
    size_t last = t + ((n - 1 - t) / T) * T;
    for (size_t i = last;; i -= T) {
        F x = ldf(a + i);
        if (!x.is_zero()) {
            F xi = inv * ldf(prefix + i);
            inv = inv * x;
            stf(a + i, xi);
        }
        if (i < T) break;
    }
}

size_t batch_invert_arena_bytes(size_t n) { return ((n * 32 + 255) & ~(size_t)255) + 256; }

// fr.BatchInvert on device memory (zeros stay zero)
template <class F>
void batch_invert(F* a, size_t n, hipStream_t st, Arena& ar) {
    if (n == 0) return;
    const size_t T = std::min<size_t>(n, std::max<size_t>(16384, n / 64));
    F* prefix = ar.get<F>(n);
    hipLaunchKernelGGL(k_batch_invert<F>, dim3(grid_for(T, 256)), dim3(256), 0, st, a, n, T, prefix);
    GG_HIP(hipGetLastError());
}

template <class F>
__global__ void __launch_bounds__(256) k_fold_brev(const F* in, size_t m, int S, int logS, F kappa, F* out) {
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    // coefficient m' + t m (m' = bitrev_m(k)) sits at S k + bitrev_S(t) of the bit-reversed input
    F acc = F::zero();
    for (int t = S - 1; t >= 0; t--) {
        const uint32_t bt = logS ? (__brev((uint32_t)t) >> (32 - logS)) : 0u;
        acc = acc * kappa + ldf(in + (size_t)S * k + bt);
    }
    stf(out + k, acc);
}

template <class F>
void fold_brev(const F* in, size_t n, int S, const F& kappa, F* out, hipStream_t st) {
    int logS = 0;
    while ((1 << logS) < S) logS++;
    GG_CHECK((1 << logS) == S && n % S == 0, GG_ERR_INTERNAL, "fold: S must be a power of two dividing n");
    const size_t m = n / S;
    hipLaunchKernelGGL(k_fold_brev<F>, dim3(grid_for(m, 256)), dim3(256), 0, st, in, m, S, logS, kappa, out);
    GG_HIP(hipGetLastError());
}

template <class F>
__global__ void k_gather_strided(const F* in, size_t n, int S, int s, F* out) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n / S) return;
    stf(out + j, ldf(in + ((size_t)s + (size_t)S * j) % n));
}

template <class F>
void gather_strided(const F* in, size_t n, int S, int s, F* out, hipStream_t st) {
    hipLaunchKernelGGL(k_gather_strided<F>, dim3(grid_for(n / S, 256)), dim3(256), 0, st, in, n, S, s, out);
    GG_HIP(hipGetLastError());
}

template <class F>
void numerator(const NumParamsT<F>& P, hipStream_t st) {
    ProfScope prof("plonk_numerator", st, (double)P.n);
    uint32_t log_n = 0;
    while ((1u << log_n) < P.n) log_n++;
    if (log_n >= 8)
        hipLaunchKernelGGL(k_numerator_coset_tiled<F>, dim3(P.n >> 8), dim3(256), 0, st, P, log_n);
    else
        hipLaunchKernelGGL(k_numerator_coset<F>, dim3(grid_for(P.n, 256)), dim3(256), 0, st, P);
    GG_HIP(hipGetLastError());
    prof.stop(st);
}

template <class F>
void divide_by_xn_minus_one(gg_domain* big, size_t n_small, F* data, hipStream_t st) {
    int curve = -1;
    const size_t m = domain_size(big, &curve);
    GG_CHECK(curve == (std::is_same<F, FrBls>::value ? GG_CURVE_BLS12_381 : GG_CURVE_BN254), GG_ERR_INVALID_ARG,
             "the big domain belongs to another scalar field");
    GG_CHECK(n_small >= 1 && m % n_small == 0, GG_ERR_INVALID_ARG, "big domain must be a multiple of n");
    const uint32_t rho = (uint32_t)(m / n_small);
    GG_CHECK(rho <= 8, GG_ERR_INVALID_ARG, "|big domain| / n > 8");
    // (x^n - 1)^-1 on the big coset has rho distinct values (prove.go:1253-1276)
    PeriodicTab<F> t{};
    xn_minus_one_inv(big, n_small, t.f);
    int lm = 0;
    while (((size_t)1 << lm) < m) lm++;
    hipLaunchKernelGGL(k_mul_periodic_bitrev<F>, dim3(grid_for(m, 256)), dim3(256), 0, st, data, m, lm, t, rho);
    GG_HIP(hipGetLastError());
    // LagrangeCoset/BitReverse -> Canonical/Regular: FFTInverse(DIT, OnCoset)
    any_ntt_inplace(big, data, 1, 1, 1, st);
}

void ntt(gg_domain* d, void* data, int inverse, int dit, int coset, hipStream_t st) {
    any_ntt_inplace(d, data, inverse, dit, coset, st);
}

#define GG_PLK_INST(F)                                                                                         \
    template void batch_invert<F>(F*, size_t, hipStream_t, Arena&);                                            \
    template void numerator<F>(const NumParamsT<F>&, hipStream_t);                                             \
    template void divide_by_xn_minus_one<F>(gg_domain*, size_t, F*, hipStream_t);                             \
    template void fold_brev<F>(const F*, size_t, int, const F&, F*, hipStream_t);                              \
    template void gather_strided<F>(const F*, size_t, int, int, F*, hipStream_t);
GG_PLK_INST(FrBls)
GG_PLK_INST(Fr)
#undef GG_PLK_INST

}  // namespace plk
}  // namespace gg

using namespace gg;

using plk::FrB;
using plk::NumParams;

extern "C" int gg_plonk_numerator_coset(const void* const* x_dev, int nx, const void* bcoef,
                                        const int* bdeg, const void* twiddles0_dev,
                                        const void* beta, const void* gamma, const void* alpha,
                                        const void* coset_gen, size_t n, int rho, int coset,
                                        void* cres_dev, void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(x_dev && bcoef && bdeg && twiddles0_dev && beta && gamma && alpha && coset_gen && cres_dev,
             GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(nx >= plk::ID_QCI && nx <= plk::MAX_X && (nx - plk::ID_QCI) % 2 == 0, GG_ERR_INVALID_ARG,
             "nx must be 15 + 2 * (number of BSB22 commitments), <= 8 commitments");
    GG_CHECK(n >= 1 && (n & (n - 1)) == 0 && n <= (1u << 30), GG_ERR_INVALID_ARG, "n must be a power of 2");
    GG_CHECK(rho >= 1 && (rho & (rho - 1)) == 0 && coset >= 0 && coset < rho, GG_ERR_INVALID_ARG, "bad rho/coset");
    NumParams P{};
    for (int q = 0; q < nx; q++) {
        GG_CHECK(x_dev[q], GG_ERR_INVALID_ARG, "null polynomial");
        P.x[q] = (const FrB*)x_dev[q];
    }
    P.nx = nx;
    const uint8_t* bc = (const uint8_t*)bcoef;
    for (int q = 0; q < 4; q++) {
        GG_CHECK(bdeg[q] >= 0 && bdeg[q] <= plk::MAX_BCOEF, GG_ERR_INVALID_ARG, "blinding order too large");
        P.bdeg[q] = bdeg[q];
        for (int k = 0; k < bdeg[q]; k++) memcpy(P.bcoef[q][k].v, bc + (q * plk::MAX_BCOEF + k) * 32, 32);
    }
    P.tw0 = (const FrB*)twiddles0_dev;
    memcpy(P.beta.v, beta, 32);
    memcpy(P.gamma.v, gamma, 32);
    memcpy(P.alpha.v, alpha, 32);
    memcpy(P.cs.v, coset_gen, 32);
    P.css = P.cs * P.cs;
    P.ka = FrB::one();  // x[ID_ID] = beta X (C ABI contract)
    P.kb = P.cs;
    P.kc = P.css;
    P.n = (uint32_t)n;
    P.rho = (uint32_t)rho;
    P.coset = (uint32_t)coset;
    int lb = 0;
    while (((size_t)1 << lb) < n * (size_t)rho) lb++;
    P.log_big = (uint32_t)lb;
    P.cres = (FrB*)cres_dev;
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : hipStreamPerThread;
    plk::numerator(P, st);
    GG_CAPI_END
}

extern "C" int gg_plonk_divide_by_xn_minus_one(gg_domain_t big, size_t n_small, void* data_dev,
                                               void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(big && data_dev, GG_ERR_INVALID_ARG, "null argument");
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : hipStreamPerThread;
    plk::divide_by_xn_minus_one(big, n_small, (FrB*)data_dev, st);
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}

extern "C" int gg_bls12_381_fr_batch_invert(void* data_dev, size_t n, void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(data_dev || n == 0, GG_ERR_INVALID_ARG, "null argument");
    if (n == 0) return GG_OK;
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : hipStreamPerThread;
    Arena ar;
    ar.reserve(plk::batch_invert_arena_bytes(n));
    plk::batch_invert((FrB*)data_dev, n, st, ar);
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}
