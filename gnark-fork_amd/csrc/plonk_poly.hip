// PlonK BLS12-381 polynomial kernels of SURVEY 8a row a21 (fr, 32 B Montgomery):
//
//   gg_plonk_ratio_copy_constraint  iop.BuildRatioCopyConstraint (prove.go:600-621):
//        Z[0] = 1, Z[i+1] = Z[i] * prod_j (f_j[i] + b*ID(j n + i) + g)
//                                / prod_j (f_j[i] + b*ID(S[j n + i]) + g)
//        with the permutation support ID(s) = u^(s div n) w^(s mod n)
//        (getSupportPermutation, setup.go:391-407; u = FrMultiplicativeGen)
//   gg_bls12_381_fr_prefix_product  inclusive running product (the Z recurrence)
//   gg_bls12_381_fr_horner          Polynomial.Evaluate (Horner) and the KZG
//        opening quotient (f - f(a)) / (X - a) (kzg.Open, prove.go:646, 823-830)
//   gg_plonk_fold_h                 foldH (prove.go:670-705)
//   gg_plonk_linearized             computeLinearizedPolynomial (prove.go:1289-1389)
//
// The two recurrences (running product; x_k = y_k + u x_(k-1)) are scans:
// 8 elements per thread in registers, a Hillis-Steele scan of the 256 thread
// aggregates in LDS, block aggregates scanned recursively (2048 per level),
// then one fix-up pass.  Horner runs the affine scan over the reversed vector.
#include "plonk_ops.h"
#include "prof.h"
#include <vector>
#include <algorithm>
#include <cstring>

namespace gg {
namespace plk {

namespace {
template <class F>
__device__ __forceinline__ F ldb(const F* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    F r;
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    return r;
}
template <class F>
__device__ __forceinline__ void stb(F* p, const F& r) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(r.v[0], r.v[1], r.v[2], r.v[3]);
    q[1] = make_uint4(r.v[4], r.v[5], r.v[6], r.v[7]);
}
}  // namespace

constexpr int SCAN_PER = 8;                    // elements per thread
constexpr int SCAN_BLK = 256 * SCAN_PER;       // elements per block
enum { SCAN_PROD = 0, SCAN_AFFINE = 1 };

// powers of the affine multiplier u of one scan level
template <class F>
struct ScanPow {
    F p[SCAN_PER + 1];  // u^0 .. u^8
    F step[8];          // u^(8 * 2^d): block-scan combine at offset 2^d threads
    const F* lo;        // u^i, i < 64
    const F* hi;        // u^(64 j), j <= 32
};

// In place: inclusive scan of each 2048-element block; aux[b] = block aggregate.
template <class F, int MODE>
__global__ void __launch_bounds__(256) k_scan_local(F* x, size_t m, ScanPow<F> P, F* aux) {
    __shared__ uint32_t sh[256 * 8];
    const size_t base = (size_t)blockIdx.x * SCAN_BLK + (size_t)threadIdx.x * SCAN_PER;
    F v[SCAN_PER];
    const F id = MODE == SCAN_PROD ? F::one() : F::zero();
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) v[k] = base + k < m ? ldb(x + base + k) : id;
#pragma unroll
    for (int k = 1; k < SCAN_PER; k++) v[k] = MODE == SCAN_PROD ? v[k] * v[k - 1] : v[k] + P.p[1] * v[k - 1];
    F agg = v[SCAN_PER - 1];
    // Hillis-Steele over the 256 thread aggregates (LDS, limb-major: no bank conflicts)
    auto put = [&](const F& a) {
#pragma unroll
        for (int l = 0; l < 8; l++) sh[l * 256 + threadIdx.x] = a.v[l];
    };
    auto get = [&](int t) {
        F a;
#pragma unroll
        for (int l = 0; l < 8; l++) a.v[l] = sh[l * 256 + t];
        return a;
    };
    put(agg);
    __syncthreads();
#pragma unroll 1
    for (int d = 0; d < 8; d++) {
        const int off = 1 << d;
        F o = id;
        const bool has = (int)threadIdx.x >= off;
        if (has) o = get(threadIdx.x - off);
        __syncthreads();
        if (has) agg = MODE == SCAN_PROD ? agg * o : agg + P.step[d] * o;
        put(agg);
        __syncthreads();
    }
    // carry-in = inclusive aggregate of the previous thread
    if (threadIdx.x > 0) {
        const F c = get(threadIdx.x - 1);
#pragma unroll
        for (int k = 0; k < SCAN_PER; k++) v[k] = MODE == SCAN_PROD ? v[k] * c : v[k] + P.p[k + 1] * c;
    }
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++)
        if (base + k < m) stb(x + base + k, v[k]);
    if (threadIdx.x == 255 && aux) stb(aux + blockIdx.x, agg);
}

// x[e] (block b > 0) combined with the inclusive aggregate of blocks < b
template <class F, int MODE>
__global__ void __launch_bounds__(256) k_scan_fix(F* x, size_t m, ScanPow<F> P, const F* aux) {
    const size_t b = blockIdx.x + 1;
    const F c = ldb(aux + b - 1);
    const uint32_t o0 = threadIdx.x * SCAN_PER;
    const size_t base = b * SCAN_BLK + o0;
    F f;
    if (MODE == SCAN_AFFINE) {
        const uint32_t e = o0 + 1;  // u^(offset + 1)
        f = ldb(P.hi + (e >> 6)) * ldb(P.lo + (e & 63)) * c;
    }
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        if (base + k >= m) break;
        F v = ldb(x + base + k);
        if (MODE == SCAN_PROD) v = v * c;
        else {
            v = v + f;
            f = f * P.p[1];
        }
        stb(x + base + k, v);
    }
}

// powers of u for one level (host, small) and the 97-entry u^i / u^(64 j)
// table of the affine fix-up (device, one thread: no host buffer in flight)
template <class F>
static void scan_pow_host(const F& u, ScanPow<F>& P) {
    P.p[0] = F::one();
    for (int k = 1; k <= SCAN_PER; k++) P.p[k] = P.p[k - 1] * u;
    F s = P.p[SCAN_PER];
    for (int d = 0; d < 8; d++) {
        P.step[d] = s;
        s = s * s;
    }
}
// thread i < 64 writes u^i, thread 64 + j (j <= 32) writes u^(64 j), each by
// square-and-multiply (<= 12 dependent products instead of a 97-long chain on
// one lane: this table heads every affine scan level)
template <class F>
__device__ __forceinline__ F pow_small(F base, uint32_t e) {
    F r = F::one();
    bool any = false;
    for (int b = 5; b >= 0; b--) {
        if (any) r = r * r;
        if ((e >> b) & 1u) {
            r = any ? r * base : base;
            any = true;
        }
    }
    return r;
}
template <class F>
__global__ void k_pow_tab(F u, F* tab) {
    const uint32_t t = threadIdx.x;
    if (blockIdx.x || t >= 97) return;
    if (t < 64) {
        stb(tab + t, pow_small(u, t));
        return;
    }
    F u64 = u;
#pragma unroll
    for (int k = 0; k < 6; k++) u64 = u64 * u64;
    stb(tab + t, pow_small(u64, t - 64));  // j = t - 64 <= 32
}

size_t scan_arena_bytes(size_t m) {
    size_t b = 0;
    for (;;) {  // one level per recursion of scan_rec: table + block aggregates
        const size_t nblk = (m + SCAN_BLK - 1) / SCAN_BLK;
        b += 256 + ((97 * 32 + 255) & ~(size_t)255) + ((nblk * 32 + 255) & ~(size_t)255);
        if (nblk <= 1) break;
        m = nblk;
    }
    return b + 512;
}

// recursive in-place scan of x[0..m); u: multiplier of this level (affine)
template <class F, int MODE>
static void scan_rec(F* x, size_t m, const F& u, hipStream_t st, Arena& ar) {
    ScanPow<F> P{};
    scan_pow_host(u, P);
    if (MODE == SCAN_AFFINE) {
        F* tab = ar.get<F>(97);
        hipLaunchKernelGGL(k_pow_tab<F>, dim3(1), dim3(128), 0, st, u, tab);
        GG_HIP(hipGetLastError());
        P.lo = tab;
        P.hi = tab + 64;
    }
    const size_t nblk = (m + SCAN_BLK - 1) / SCAN_BLK;
    F* aux = nblk > 1 ? ar.get<F>(nblk) : nullptr;
    hipLaunchKernelGGL((k_scan_local<F, MODE>), dim3((unsigned)nblk), dim3(256), 0, st, x, m, P, aux);
    GG_HIP(hipGetLastError());
    if (nblk <= 1) return;
    // the next level's elements each stand for SCAN_BLK of this level: u^2048
    F un = u;
    for (int i = 0; i < 11; i++) un = un * un;
    scan_rec<F, MODE>(aux, nblk, un, st, ar);
    hipLaunchKernelGGL((k_scan_fix<F, MODE>), dim3((unsigned)(nblk - 1)), dim3(256), 0, st, x, m, P, aux);
    GG_HIP(hipGetLastError());
}

template <class F>
void scan_prod(F* x, size_t m, hipStream_t st, Arena& ar) {
    if (m) scan_rec<F, SCAN_PROD>(x, m, F::one(), st, ar);
}

template <class F>
__global__ void k_reverse_copy(F* dst, const F* src, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) stb(dst + i, ldb(src + n - 1 - i));
}

// q[j] = g[n-2-j] for j < n-1 where g is the reversed affine scan
template <class F>
__global__ void k_quotient_out(F* q, const F* g, size_t n) {
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j + 1 < n) stb(q + j, ldb(g + n - 2 - j));
}

// ---------------------------------------------------------------- ratio
template <class F>
struct PowSplit {  // x^e = hi[e >> S] * lo[e & (2^S - 1)]
    const F *hi, *lo;
    int S;
    __device__ __forceinline__ F at(uint32_t e) const {
        return ldb(hi + (e >> S)) * ldb(lo + (e & ((1u << S) - 1)));
    }
};

template <class F>
__global__ void __launch_bounds__(256) k_ratio_numden(const F* L, const F* R, const F* O,
                                                      const int64_t* perm, uint32_t n, int log_n,
                                                      F beta, F gamma, F u, F uu, PowSplit<F> w,
                                                      F* num, F* den) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i == 0) {
        stb(num, F::one());
        stb(den, F::one());
    }
    if (i + 1 >= n) return;
    const F* f[3] = {L, R, O};
    const F wi = w.at(i);
    F b = F::one(), d = F::one();
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const F fv = ldb(f[j] + i);
        F id = j == 0 ? wi : (j == 1 ? wi * u : wi * uu);
        b = b * (fv + beta * id + gamma);
        const uint64_t s = (uint64_t)perm[(size_t)j * n + i];
        const uint32_t blk = (uint32_t)(s >> log_n), off = (uint32_t)(s & (n - 1));
        F sg = w.at(off);
        if (blk == 1) sg = sg * u;
        else if (blk == 2) sg = sg * uu;
        d = d * (fv + beta * sg + gamma);
    }
    stb(num + i + 1, b);
    stb(den + i + 1, d);
}

template <class F>
__global__ void k_mul_inplace(F* a, const F* b, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) stb(a + i, ldb(a + i) * ldb(b + i));
}

// ---------------------------------------------------------------- foldH / linearized
template <class F>
__global__ void k_fold_h(const F* h, size_t np2, F z, F* out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np2) return;
    F t = ldb(h + 2 * np2 + i) * z + ldb(h + np2 + i);
    stb(out + i, t * z + ldb(h + i));
}

// prove.go:1347-1386, term by term
template <class F>
__global__ void __launch_bounds__(256) k_linearized(LinParamsT<F> P) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.nz) return;
    const F zi = ldb(P.z + i);
    F t = zi * P.s2;
    if (i < P.ns3) t = t + ldb(P.s3 + i) * P.s1;
    t = t * P.alpha;
    if (i < P.nq) {
        F t0 = ldb(P.ql + i) * P.l + ldb(P.qm + i) * P.rl;
        t = t + t0;
        t = t + ldb(P.qr + i) * P.r;
        t = t + (ldb(P.qo + i) * P.o + ldb(P.qk + i));
        for (int j = 0; j < P.ncmt; j++) t = t + ldb(P.pi2[j] + i) * P.qcp[j];
    }
    stb(P.z + i, t + zi * P.lag);
}

// out[bitrev(i)] = in[i] (out-of-place; fft.BitReverse / iop ToRegular)
template <class F>
__global__ void k_bit_reverse(F* out, const F* in, size_t n, int log_n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t r = log_n ? (__brev((uint32_t)i) >> (32 - log_n)) : 0u;
    stb(out + r, ldb(in + i));
}

// y[i] += a * x[i]
template <class F>
__global__ void k_axpy(F* y, const F* x, size_t n, F a) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) stb(y + i, ldb(y + i) + a * ldb(x + i));
}

template <class F>
__global__ void k_scale(F* y, size_t n, F a) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) stb(y + i, ldb(y + i) * a);
}
template <class F>
__global__ void k_shift_copy(const F* in, F* out, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) stb(out + i, ldb(in + (i + 1 == n ? 0 : i + 1)));
}

size_t horner_arena_bytes(size_t n) { return ((n * 32 + 255) & ~(size_t)255) + scan_arena_bytes(n); }

template <class F>
void horner(const F* f, size_t n, const F& a, F* q, F* value_dev, hipStream_t st, Arena& ar) {
    if (n == 0) {
        GG_HIP(hipMemsetAsync(value_dev, 0, 32, st));
        return;
    }
    F* g = ar.get<F>(n);
    hipLaunchKernelGGL(k_reverse_copy<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, g, f, n);
    GG_HIP(hipGetLastError());
    // x_k = y_k + a x_(k-1) over y = reversed f: x_(n-1) = f(a), x_k = sum_(i >= n-1-k) f_i a^(i-(n-1-k))
    scan_rec<F, SCAN_AFFINE>(g, n, a, st, ar);
    if (q && n > 1) {
        hipLaunchKernelGGL(k_quotient_out<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, q, (const F*)g, n);
        GG_HIP(hipGetLastError());
    }
    GG_HIP(hipMemcpyAsync(value_dev, g + n - 1, 32, hipMemcpyDeviceToDevice, st));
}

// x^e tables for e < n split as hi[e >> S] * lo[e & (2^S - 1)]: thread t
// computes lo[t] = w^t and hi[t] = w^(t 2^S) by square-and-multiply (no host
// buffer in flight)
template <class F>
__global__ void k_pow_split(F w, F step, F* lo, uint32_t nlo, F* hi, uint32_t nhi) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    auto pw = [](F b, uint32_t e) {
        F r = F::one();
        while (e) {
            if (e & 1) r = r * b;
            b = b * b;
            e >>= 1;
        }
        return r;
    };
    if (t < nlo) stb(lo + t, pw(w, t));
    if (t < nhi) stb(hi + t, pw(step, t));
}

static int log2_ceil(size_t n) {
    int L = 0;
    while (((size_t)1 << L) < n) L++;
    return L;
}

size_t ratio_arena_bytes(size_t n) {
    const int L = log2_ceil(n), S = (L + 1) / 2;
    const size_t tabs = (((size_t)1 << S) + ((size_t)1 << (L - S))) * 32 + 512;
    return tabs + ((n * 32 + 255) & ~(size_t)255) + batch_invert_arena_bytes(n) + scan_arena_bytes(n) + 1024;
}

template <class F>
void ratio(const F* l, const F* r, const F* o, const int64_t* perm, size_t n, const F& beta, const F& gamma,
           const F& w, const F& u, F* z, hipStream_t st, Arena& ar) {
    const int L = log2_ceil(n);
    const int S = (L + 1) / 2;
    const uint32_t nlo = 1u << S, nhi = 1u << (L - S);
    F* lo = ar.get<F>(nlo);
    F* hi = ar.get<F>(nhi);
    F step = w;
    for (int i = 0; i < S; i++) step = step * step;  // w^(2^S)
    hipLaunchKernelGGL(k_pow_split<F>, dim3(grid_for(std::max(nlo, nhi), 256)), dim3(256), 0, st, w, step, lo, nlo,
                       hi, nhi);
    GG_HIP(hipGetLastError());
    PowSplit<F> ps{hi, lo, S};
    F* den = ar.get<F>(n);
    hipLaunchKernelGGL(k_ratio_numden<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, l, r, o, perm, (uint32_t)n, L,
                       beta, gamma, u, u * u, ps, z, den);
    GG_HIP(hipGetLastError());
    batch_invert(den, n, st, ar);  // t = fr.BatchInvert(t)
    hipLaunchKernelGGL(k_mul_inplace<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, z, (const F*)den, n);
    GG_HIP(hipGetLastError());
    scan_prod(z, n, st, ar);  // Z[i] = Z[i-1] * num_i / den_i
}

// ---------------------------------------------------------------- batched evaluation
template <class F>
struct EvalJob {
    const F* f[EVAL_MAX];
    uint32_t len[EVAL_MAX];
    int count;
};
constexpr int EVAL_BLOCKS = 1024;  // x 256 threads: G = 2^18 lanes, 16 coefficients each at 2^22

// thread g of G: acc_k = sum_j f_k[g + j G] (a^G)^j by Horner over j, times
// a^g; block sums per polynomial into part[k * gridDim.x + block]
template <class F>
__global__ void __launch_bounds__(256) k_eval_many(EvalJob<F> J, PowSplit<F> ap, F aG, F* part) {
    __shared__ uint32_t sh[256 * 8];
    const uint32_t G = gridDim.x * blockDim.x;
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const F ag = ap.at(g);
    for (int k = 0; k < J.count; k++) {
        const uint32_t len = J.len[k];
        F acc = F::zero();
        if (g < len) {
            const uint32_t jn = (len - 1 - g) / G;  // last j with g + j G < len
            const F* f = J.f[k];
            acc = ldb(f + g + (size_t)jn * G);
            for (uint32_t j = jn; j-- > 0;) acc = acc * aG + ldb(f + g + (size_t)j * G);
            acc = acc * ag;
        }
        // block sum (LDS, limb-major)
#pragma unroll
        for (int l = 0; l < 8; l++) sh[l * 256 + threadIdx.x] = acc.v[l];
        __syncthreads();
        for (int s = 128; s > 0; s >>= 1) {
            if ((int)threadIdx.x < s) {
                F o;
#pragma unroll
                for (int l = 0; l < 8; l++) o.v[l] = sh[l * 256 + threadIdx.x + s];
                acc = acc + o;
#pragma unroll
                for (int l = 0; l < 8; l++) sh[l * 256 + threadIdx.x] = acc.v[l];
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) stb(part + (size_t)k * gridDim.x + blockIdx.x, acc);
        __syncthreads();
    }
}

// out[k] = sum_b part[k * nb + b]: one block per polynomial
template <class F>
__global__ void __launch_bounds__(256) k_eval_sum(const F* part, uint32_t nb, F* out) {
    __shared__ uint32_t sh[256 * 8];
    const int k = blockIdx.x;
    F acc = F::zero();
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) acc = acc + ldb(part + (size_t)k * nb + b);
#pragma unroll
    for (int l = 0; l < 8; l++) sh[l * 256 + threadIdx.x] = acc.v[l];
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            F o;
#pragma unroll
            for (int l = 0; l < 8; l++) o.v[l] = sh[l * 256 + threadIdx.x + s];
            acc = acc + o;
#pragma unroll
            for (int l = 0; l < 8; l++) sh[l * 256 + threadIdx.x] = acc.v[l];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) stb(out + k, acc);
}

size_t eval_many_arena_bytes(size_t max_len, int count) {
    (void)max_len;
    const uint32_t G = EVAL_BLOCKS * 256;
    int L = 0;
    while ((1u << L) < G) L++;
    const int S = (L + 1) / 2;
    return (((size_t)1 << S) + ((size_t)1 << (L - S))) * 32 + 512 + (size_t)count * EVAL_BLOCKS * 32 + 512;
}

template <class F>
void eval_many(const F* const* f, const size_t* len, int count, const F& a, F* out_dev, hipStream_t st,
               Arena& ar) {
    GG_CHECK(count >= 1 && count <= EVAL_MAX, GG_ERR_INVALID_ARG, "eval_many: 1..16 polynomials");
    EvalJob<F> J{};
    J.count = count;
    for (int k = 0; k < count; k++) {
        GG_CHECK(len[k] < ((size_t)1 << 31), GG_ERR_INVALID_ARG, "eval_many: polynomial too long");
        J.f[k] = f[k];
        J.len[k] = (uint32_t)len[k];
    }
    const uint32_t G = EVAL_BLOCKS * 256;
    int L = 0;
    while ((1u << L) < G) L++;
    const int S = (L + 1) / 2;
    const uint32_t nlo = 1u << S, nhi = 1u << (L - S);
    F* lo = ar.get<F>(nlo);
    F* hi = ar.get<F>(nhi);
    F step = a;
    for (int i = 0; i < S; i++) step = step * step;  // a^(2^S)
    hipLaunchKernelGGL(k_pow_split<F>, dim3(grid_for(std::max(nlo, nhi), 256)), dim3(256), 0, st, a, step, lo, nlo,
                       hi, nhi);
    GG_HIP(hipGetLastError());
    F aG = a;
    for (int i = 0; i < L; i++) aG = aG * aG;  // a^G, G = 2^L
    F* part = ar.get<F>((size_t)count * EVAL_BLOCKS);
    hipLaunchKernelGGL(k_eval_many<F>, dim3(EVAL_BLOCKS), dim3(256), 0, st, J, PowSplit<F>{hi, lo, S}, aG, part);
    GG_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_eval_sum<F>, dim3(count), dim3(256), 0, st, (const F*)part, (uint32_t)EVAL_BLOCKS, out_dev);
    GG_HIP(hipGetLastError());
}

template <class F>
struct LinComb {
    const F* f[EVAL_MAX];
    uint32_t len[EVAL_MAX];
    F c[EVAL_MAX];
    int count;
};
template <class F>
__global__ void __launch_bounds__(256) k_lincomb(F* out, size_t n_out, LinComb<F> L) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_out) return;
    F acc = F::zero();
    for (int k = 0; k < L.count; k++)
        if (j < L.len[k]) acc = acc + L.c[k] * ldb(L.f[k] + j);
    stb(out + j, acc);
}

template <class F>
void lincomb(F* out, size_t n_out, const F* const* f, const size_t* len, const F* c, int count, hipStream_t st) {
    GG_CHECK(count >= 1 && count <= EVAL_MAX, GG_ERR_INVALID_ARG, "lincomb: 1..16 polynomials");
    LinComb<F> L{};
    L.count = count;
    for (int k = 0; k < count; k++) {
        L.f[k] = f[k];
        L.len[k] = (uint32_t)std::min(len[k], n_out);
        L.c[k] = c[k];
    }
    hipLaunchKernelGGL(k_lincomb<F>, dim3(grid_for(n_out, 256)), dim3(256), 0, st, out, n_out, L);
    GG_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- ratio over a slice
template <class F>
__global__ void __launch_bounds__(256) k_ratio_factors(const F* L, const F* R, const F* O, const int64_t* p0,
                                                       const int64_t* p1, const int64_t* p2, uint32_t lo, uint32_t cnt,
                                                       int log_n, F beta, F gamma, F u, F uu, PowSplit<F> w, F* num,
                                                       F* den) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const uint32_t i = lo + t, nmask = (1u << log_n) - 1;
    const F* f[3] = {L, R, O};
    const int64_t* pm[3] = {p0, p1, p2};
    const F wi = w.at(i);
    F b = F::one(), d = F::one();
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const F fv = ldb(f[j] + t);
        F id = j == 0 ? wi : (j == 1 ? wi * u : wi * uu);
        b = b * (fv + beta * id + gamma);
        const uint64_t s = (uint64_t)pm[j][t];
        const uint32_t blk = (uint32_t)(s >> log_n), off = (uint32_t)(s & nmask);
        F sg = w.at(off);
        if (blk == 1) sg = sg * u;
        else if (blk == 2) sg = sg * uu;
        d = d * (fv + beta * sg + gamma);
    }
    stb(num + t, b);
    stb(den + t, d);
}

template <class F>
__global__ void k_ratio_fixup(const F* P, size_t cnt, F prefix, F* z) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    stb(z + t, t ? prefix * ldb(P + t - 1) : prefix);
}

size_t ratio_range_arena_bytes(size_t n, size_t cnt) {
    const int L = log2_ceil(n), S = (L + 1) / 2;
    const size_t tabs = (((size_t)1 << S) + ((size_t)1 << (L - S))) * 32 + 512;
    return tabs + ((cnt * 32 + 255) & ~(size_t)255) + batch_invert_arena_bytes(cnt) + scan_arena_bytes(cnt) + 1024;
}

template <class F>
void ratio_range(const F* l, const F* r, const F* o, const int64_t* perm0, const int64_t* perm1,
                 const int64_t* perm2, size_t lo, size_t cnt, size_t n, const F& beta, const F& gamma,
                 const F& w, const F& u, F* P, hipStream_t st, Arena& ar) {
    if (!cnt) return;
    const int L = log2_ceil(n);
    const int S = (L + 1) / 2;
    const uint32_t nlo = 1u << S, nhi = 1u << (L - S);
    F* tlo = ar.get<F>(nlo);
    F* thi = ar.get<F>(nhi);
    F step = w;
    for (int i = 0; i < S; i++) step = step * step;  // w^(2^S)
    hipLaunchKernelGGL(k_pow_split<F>, dim3(grid_for(std::max(nlo, nhi), 256)), dim3(256), 0, st, w, step, tlo, nlo,
                       thi, nhi);
    GG_HIP(hipGetLastError());
    F* den = ar.get<F>(cnt);
    hipLaunchKernelGGL(k_ratio_factors<F>, dim3(grid_for(cnt, 256)), dim3(256), 0, st, l, r, o, perm0, perm1, perm2,
                       (uint32_t)lo, (uint32_t)cnt, L, beta, gamma, u, u * u, PowSplit<F>{thi, tlo, S}, P, den);
    GG_HIP(hipGetLastError());
    batch_invert(den, cnt, st, ar);
    hipLaunchKernelGGL(k_mul_inplace<F>, dim3(grid_for(cnt, 256)), dim3(256), 0, st, P, (const F*)den, cnt);
    GG_HIP(hipGetLastError());
    scan_prod(P, cnt, st, ar);
}

template <class F>
void ratio_fixup(const F* P, size_t cnt, const F& prefix, F* z, hipStream_t st) {
    if (!cnt) return;
    hipLaunchKernelGGL(k_ratio_fixup<F>, dim3(grid_for(cnt, 256)), dim3(256), 0, st, P, cnt, prefix, z);
    GG_HIP(hipGetLastError());
}

template <class F>
void fold_h(const F* h, size_t n_small, const F& zz, F* out, hipStream_t st) {
    const size_t np2 = n_small + 2;
    hipLaunchKernelGGL(k_fold_h<F>, dim3(grid_for(np2, 256)), dim3(256), 0, st, h, np2, zz, out);
    GG_HIP(hipGetLastError());
}

template <class F>
void linearized(const LinParamsT<F>& P, hipStream_t st) {
    hipLaunchKernelGGL(k_linearized<F>, dim3(grid_for(P.nz, 256)), dim3(256), 0, st, P);
    GG_HIP(hipGetLastError());
}

template <class F>
void bit_reverse(const F* in, F* out, size_t n, hipStream_t st) {
    int L = 0;
    while (((size_t)1 << L) < n) L++;
    hipLaunchKernelGGL(k_bit_reverse<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, out, in, n, L);
    GG_HIP(hipGetLastError());
}

template <class F>
void axpy(F* y, const F* x, size_t n, const F& a, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_axpy<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, y, x, n, a);
    GG_HIP(hipGetLastError());
}

template <class F>
void scale(F* y, size_t n, const F& a, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_scale<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, y, n, a);
    GG_HIP(hipGetLastError());
}

template <class F>
void shift_copy(const F* in, F* out, size_t n, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_shift_copy<F>, dim3(grid_for(n, 256)), dim3(256), 0, st, in, out, n);
    GG_HIP(hipGetLastError());
}

// the two scalar fields of the PlonK provers
#define GG_PLK_INST(F)                                                                                          \
    template void scan_prod<F>(F*, size_t, hipStream_t, Arena&);                                                \
    template void horner<F>(const F*, size_t, const F&, F*, F*, hipStream_t, Arena&);                          \
    template void eval_many<F>(const F* const*, const size_t*, int, const F&, F*, hipStream_t, Arena&);          \
    template void lincomb<F>(F*, size_t, const F* const*, const size_t*, const F*, int, hipStream_t);           \
    template void ratio_range<F>(const F*, const F*, const F*, const int64_t*, const int64_t*, const int64_t*,    \
                                 size_t, size_t, size_t, const F&, const F&, const F&, const F&, F*, hipStream_t,  \
                                 Arena&);                                                                          \
    template void ratio_fixup<F>(const F*, size_t, const F&, F*, hipStream_t);                                  \
    template void ratio<F>(const F*, const F*, const F*, const int64_t*, size_t, const F&, const F&, const F&, \
                           const F&, F*, hipStream_t, Arena&);                                                  \
    template void fold_h<F>(const F*, size_t, const F&, F*, hipStream_t);                                       \
    template void linearized<F>(const LinParamsT<F>&, hipStream_t);                                             \
    template void bit_reverse<F>(const F*, F*, size_t, hipStream_t);                                            \
    template void axpy<F>(F*, const F*, size_t, const F&, hipStream_t);                                         \
    template void scale<F>(F*, size_t, const F&, hipStream_t);                                                  \
    template void shift_copy<F>(const F*, F*, size_t, hipStream_t);
GG_PLK_INST(FrBls)
GG_PLK_INST(Fr)
#undef GG_PLK_INST

}  // namespace plk

static plk::FrB frb(const void* p) {
    plk::FrB x;
    memcpy(x.v, p, 32);
    return x;
}
static hipStream_t pick(void* s) { return s ? (hipStream_t)s : hipStreamPerThread; }

}  // namespace gg

using namespace gg;
using plk::FrB;

// ---- C ABI: synchronous wrappers (scratch lives for the call)
extern "C" int gg_bls12_381_fr_prefix_product(void* data_dev, size_t n, void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(data_dev || n == 0, GG_ERR_INVALID_ARG, "null argument");
    hipStream_t st = pick(hip_stream);
    Arena ar;
    ar.reserve(plk::scan_arena_bytes(n));
    plk::scan_prod((FrB*)data_dev, n, st, ar);
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}

extern "C" int gg_bls12_381_fr_horner(const void* f_dev, size_t n, const void* a_mont, void* q_dev,
                                      void* value_out, void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(f_dev && a_mont && value_out, GG_ERR_INVALID_ARG, "null argument");
    if (n == 0) {
        memset(value_out, 0, 32);
        return GG_OK;
    }
    hipStream_t st = pick(hip_stream);
    Arena ar;
    ar.reserve(plk::horner_arena_bytes(n) + 256);
    FrB* v = ar.get<FrB>(1);
    plk::horner((const FrB*)f_dev, n, frb(a_mont), (FrB*)q_dev, v, st, ar);
    GG_HIP(hipMemcpyAsync(value_out, v, 32, hipMemcpyDeviceToHost, st));
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}

extern "C" int gg_fr_evaluate_many(int curve, const void* const* polys_dev, const size_t* lens, int count,
                                   const void* point_mont, void* values_out, void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(polys_dev && lens && point_mont && values_out, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "bad curve");
    GG_CHECK(count >= 1 && count <= plk::EVAL_MAX, GG_ERR_INVALID_ARG, "1..16 polynomials");
    size_t mx = 0;
    for (int k = 0; k < count; k++) {
        GG_CHECK(polys_dev[k] || lens[k] == 0, GG_ERR_INVALID_ARG, "null polynomial");
        mx = std::max(mx, lens[k]);
    }
    hipStream_t st = pick(hip_stream);
    Arena ar;
    ar.reserve(plk::eval_many_arena_bytes(mx, count) + 256 + 32 * (size_t)count);
    auto run = [&](auto tag) {
        using F = decltype(tag);
        F a;
        memcpy(a.v, point_mont, 32);
        F* out = ar.get<F>(count);
        plk::eval_many((const F* const*)polys_dev, lens, count, a, out, st, ar);
        GG_HIP(hipMemcpyAsync(values_out, out, 32 * (size_t)count, hipMemcpyDeviceToHost, st));
    };
    if (curve == GG_CURVE_BN254) run(Fr{});
    else run(FrB{});
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}

extern "C" int gg_plonk_ratio_copy_constraint(const void* l_dev, const void* r_dev, const void* o_dev,
                                              const int64_t* perm_dev, size_t n, const void* beta,
                                              const void* gamma, const void* omega_mont,
                                              const void* coset_shift_mont, void* z_dev,
                                              void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(l_dev && r_dev && o_dev && perm_dev && beta && gamma && omega_mont && coset_shift_mont && z_dev,
             GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(n >= 1 && (n & (n - 1)) == 0 && n <= ((size_t)1 << 30), GG_ERR_INVALID_ARG,
             "n must be a power of 2");
    const FrB w = frb(omega_mont);
    GG_CHECK(pow_u64(w, n) == FrB::one(), GG_ERR_INVALID_ARG, "omega^n != 1");
    hipStream_t st = pick(hip_stream);
    Arena ar;
    ar.reserve(plk::ratio_arena_bytes(n));
    plk::ratio((const FrB*)l_dev, (const FrB*)r_dev, (const FrB*)o_dev, perm_dev, n, frb(beta), frb(gamma), w,
               frb(coset_shift_mont), (FrB*)z_dev, st, ar);
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}

extern "C" int gg_plonk_fold_h(const void* h_dev, size_t n_small, const void* zeta_pow_np2,
                               void* out_dev, void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(h_dev && zeta_pow_np2 && out_dev, GG_ERR_INVALID_ARG, "null argument");
    hipStream_t st = pick(hip_stream);
    plk::fold_h((const FrB*)h_dev, n_small, frb(zeta_pow_np2), (FrB*)out_dev, st);
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}

extern "C" int gg_plonk_linearized(void* blinded_z_dev, size_t nz, const void* s3_dev, size_t ns3,
                                   const void* const* q_dev, size_t nq, const void* const* pi2_dev,
                                   const void* qcp_zeta, int n_cmt, const void* scalars8,
                                   void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(blinded_z_dev && (s3_dev || ns3 == 0) && q_dev && scalars8, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(n_cmt >= 0 && n_cmt <= plk::MAX_CMT, GG_ERR_INVALID_ARG, "at most 8 BSB22 commitments");
    GG_CHECK(n_cmt == 0 || (pi2_dev && qcp_zeta), GG_ERR_INVALID_ARG, "null commitment polynomials");
    plk::LinParams P{};
    P.z = (FrB*)blinded_z_dev;
    P.nz = nz;
    P.s3 = (const FrB*)s3_dev;
    P.ns3 = ns3;
    for (int k = 0; k < 5; k++) GG_CHECK(q_dev[k] || nq == 0, GG_ERR_INVALID_ARG, "null selector");
    P.ql = (const FrB*)q_dev[0];
    P.qr = (const FrB*)q_dev[1];
    P.qm = (const FrB*)q_dev[2];
    P.qo = (const FrB*)q_dev[3];
    P.qk = (const FrB*)q_dev[4];
    P.nq = nq;
    P.ncmt = n_cmt;
    for (int j = 0; j < n_cmt; j++) {
        GG_CHECK(pi2_dev[j], GG_ERR_INVALID_ARG, "null pi2 polynomial");
        P.pi2[j] = (const FrB*)pi2_dev[j];
        P.qcp[j] = frb((const uint8_t*)qcp_zeta + 32 * j);
    }
    const uint8_t* s = (const uint8_t*)scalars8;
    FrB* dst[8] = {&P.s1, &P.s2, &P.alpha, &P.l, &P.r, &P.rl, &P.o, &P.lag};
    for (int k = 0; k < 8; k++) *dst[k] = frb(s + 32 * k);
    hipStream_t st = pick(hip_stream);
    plk::linearized(P, st);
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}

extern "C" int gg_bls12_381_fr_bit_reverse(const void* in_dev, void* out_dev, size_t n, void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(in_dev && out_dev && in_dev != out_dev, GG_ERR_INVALID_ARG, "need distinct in / out buffers");
    GG_CHECK(n >= 1 && (n & (n - 1)) == 0 && n <= ((size_t)1 << 31), GG_ERR_INVALID_ARG, "n must be a power of 2");
    hipStream_t st = pick(hip_stream);
    plk::bit_reverse((const FrB*)in_dev, (FrB*)out_dev, n, st);
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}

extern "C" int gg_bls12_381_fr_axpy(void* y_dev, const void* x_dev, size_t n, const void* a_mont,
                                    void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(y_dev && x_dev && a_mont, GG_ERR_INVALID_ARG, "null argument");
    if (n == 0) return GG_OK;
    hipStream_t st = pick(hip_stream);
    plk::axpy((FrB*)y_dev, (const FrB*)x_dev, n, frb(a_mont), st);
    GG_WAIT_STREAM(st);
    GG_CAPI_END
}
