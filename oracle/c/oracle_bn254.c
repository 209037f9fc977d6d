/* ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Multithreaded C restatement of the reference's Groth16/BN254 hot path,
 * used (a) as the large-size parity checker in tests/ and (b) as bench.py's
 * cpu_baseline ("port": our restatement, not gnark itself -- no Go toolchain
 * exists in this image).  Never linked by the product.
 *
 * Follows:
 *   computeH               backend/groth16/bn254/prove.go:353-396
 *   Prove (MSMs, epilogue) backend/groth16/bn254/prove.go:127-320
 *   filtering              prove.go:151-175 (InfinityA/B)
 *   MultiExp / FFT         gnark-crypto [ext] published algorithms
 *                          (signed-digit Pippenger with XYZZ buckets;
 *                           radix-2 DIF/DIT with gnark's ordering conventions).
 * Cross-checked against oracle/bn254_oracle.py in tests/test_oracle_c.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>
#include "field.h"

field_t FP, FR;

static const u64 P_LIMBS[4] = {0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL};
static const u64 R_LIMBS[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL};

static void init_field(field_t *F, const u64 p[4]) {
    memcpy(F->p, p, 32);
    /* inv = -p^{-1} mod 2^64 by Newton iteration */
    u64 x = 1;
    for (int i = 0; i < 7; i++) x *= 2 - p[0] * x;
    F->inv = (u64)0 - x;
    /* one = 2^256 mod p; r2 = 2^512 mod p, by repeated doubling of 1 */
    fe_t t = {{1, 0, 0, 0}};
    for (int i = 0; i < 256; i++) fe_add(F, &t, &t, &t);
    F->one = t;
    for (int i = 0; i < 256; i++) fe_add(F, &t, &t, &t);
    F->r2 = t;
}

static int g_inited = 0;
void oracle_field_init(void) {
    if (g_inited) return;
    init_field(&FP, P_LIMBS);
    init_field(&FR, R_LIMBS);
    g_inited = 1;
}

void fe_pow(const field_t *F, fe_t *r, const fe_t *a, const u64 e[4]) {
    fe_t acc = F->one, b = *a;
    for (int i = 255; i >= 0; i--) {
        fe_mul(F, &acc, &acc, &acc);
        if ((e[i >> 6] >> (i & 63)) & 1) fe_mul(F, &acc, &acc, &b);
    }
    *r = acc;
}

void fe_inv(const field_t *F, fe_t *r, const fe_t *a) {
    u64 e[4];
    memcpy(e, F->p, 32);
    /* p - 2 */
    u128 x = (u128)e[0] - 2;
    e[0] = (u64)x;
    if ((x >> 64) & 1) { for (int i = 1; i < 4; i++) { if (e[i]--) break; } }
    fe_pow(F, r, a, e);
}

void fe_from_u64(const field_t *F, fe_t *r, u64 v) {
    fe_t t = {{v, 0, 0, 0}};
    fe_to_mont(F, r, &t);
}

void fe_batch_inv(const field_t *F, fe_t *a, size_t n) {
    if (!n) return;
    fe_t *pre = (fe_t *)malloc(sizeof(fe_t) * n);
    fe_t acc = F->one;
    for (size_t i = 0; i < n; i++) {
        pre[i] = acc;
        if (!fe_is_zero(&a[i])) fe_mul(F, &acc, &acc, &a[i]);
    }
    fe_t inv;
    fe_inv(F, &inv, &acc);
    for (size_t i = n; i-- > 0;) {
        if (fe_is_zero(&a[i])) continue;
        fe_t t;
        fe_mul(F, &t, &inv, &pre[i]);
        fe_mul(F, &inv, &inv, &a[i]);
        a[i] = t;
    }
    free(pre);
}

void fe2_inv(fe2_t *r, const fe2_t *a) {
    fe_t t0, t1;
    fe_sqr(&FP, &t0, &a->a0);
    fe_sqr(&FP, &t1, &a->a1);
    fe_add(&FP, &t0, &t0, &t1);
    fe_inv(&FP, &t1, &t0);
    fe_mul(&FP, &r->a0, &a->a0, &t1);
    fe_mul(&FP, &t0, &a->a1, &t1);
    fe_neg(&FP, &r->a1, &t0);
}

void fe2_batch_inv(fe2_t *a, size_t n) {
    if (!n) return;
    fe2_t *pre = (fe2_t *)malloc(sizeof(fe2_t) * n);
    fe2_t acc; acc.a0 = FP.one; memset(&acc.a1, 0, 32);
    for (size_t i = 0; i < n; i++) {
        pre[i] = acc;
        if (!fe2_is_zero(&a[i])) fe2_mul(&acc, &acc, &a[i]);
    }
    fe2_t inv;
    fe2_inv(&inv, &acc);
    for (size_t i = n; i-- > 0;) {
        if (fe2_is_zero(&a[i])) continue;
        fe2_t t;
        fe2_mul(&t, &inv, &pre[i]);
        fe2_mul(&inv, &inv, &a[i]);
        a[i] = t;
    }
    free(pre);
}

/* ---------------- G1 instantiation ---------------- */
#define FP_ADD(r, a, b) fe_add(&FP, r, a, b)
#define FP_SUB(r, a, b) fe_sub(&FP, r, a, b)
#define FP_MUL(r, a, b) fe_mul(&FP, r, a, b)
#define FP_SQR(r, a) fe_mul(&FP, r, a, a)
#define FP_DBL(r, a) fe_add(&FP, r, a, a)
#define FP_NEG(r, a) fe_neg(&FP, r, a)
#define FP_BINV(a, n) fe_batch_inv(&FP, a, n)

#define CP g1
#define CF_T fe_t
#define CF_ADD FP_ADD
#define CF_SUB FP_SUB
#define CF_MUL FP_MUL
#define CF_SQR FP_SQR
#define CF_DBL FP_DBL
#define CF_NEG FP_NEG
#define CF_ISZERO fe_is_zero
#define CF_EQ fe_eq
#define CF_BATCH_INV FP_BINV
#define CF_ONE (FP.one)
#include "curve_impl.h"
#undef CP
#undef CF_T
#undef CF_ADD
#undef CF_SUB
#undef CF_MUL
#undef CF_SQR
#undef CF_DBL
#undef CF_NEG
#undef CF_ISZERO
#undef CF_EQ
#undef CF_BATCH_INV
#undef CF_ONE

/* ---------------- G2 instantiation ---------------- */
static fe2_t FP2_ONE;
#define CP g2
#define CF_T fe2_t
#define CF_ADD fe2_add
#define CF_SUB fe2_sub
#define CF_MUL fe2_mul
#define CF_SQR fe2_sqr
#define CF_DBL fe2_dbl
#define CF_NEG fe2_neg
#define CF_ISZERO fe2_is_zero
#define CF_EQ fe2_eq
#define CF_BATCH_INV fe2_batch_inv
#define CF_ONE (FP2_ONE)
#include "curve_impl.h"

static void oc_init_all(void) {
    oracle_field_init();
    FP2_ONE.a0 = FP.one;
    memset(&FP2_ONE.a1, 0, 32);
}

/* ---------------- scalars ---------------- */
static void scalars_canonical(const fe_t *in, u64 (*out)[4], size_t n, int nt) {
#pragma omp parallel for num_threads(nt) schedule(static)
    for (size_t i = 0; i < n; i++) {
        fe_t t;
        fe_from_mont(&FR, &t, &in[i]);
        memcpy(out[i], t.v, 32);
    }
}

static int best_c(size_t n) {
    int best = 2;
    double bcost = 1e300;
    for (int c = 2; c <= 20; c++) {
        int w = (256 + c - 1) / c;
        double cost = (double)w * ((double)n + (double)(1u << c));
        if (cost < bcost) { bcost = cost; best = c; }
    }
    return best;
}

/* signed digits: digits[i*W + w] in [-2^(c-1), 2^(c-1)] */
static void signed_digits(const u64 (*k)[4], size_t n, int c, int W, int32_t *digits, int nt) {
    const u64 mask = (1ULL << c) - 1;
#pragma omp parallel for num_threads(nt) schedule(static)
    for (size_t i = 0; i < n; i++) {
        int carry = 0;
        for (int w = 0; w < W; w++) {
            int bit = w * c;
            u64 v = 0;
            if (bit < 256) {
                int limb = bit >> 6, off = bit & 63;
                v = k[i][limb] >> off;
                if (off + c > 64 && limb < 3) v |= k[i][limb + 1] << (64 - off);
                v &= mask;
            }
            int64_t d = (int64_t)v + carry;
            if (d > (int64_t)(1ULL << (c - 1))) { d -= (int64_t)(1ULL << c); carry = 1; }
            else carry = 0;
            digits[i * W + w] = (int32_t)d;
        }
    }
}

#define MSM_IMPL(G, AFF_T, XYZZ_T, JAC_T)                                                         \
static void G##_msm_impl(JAC_T *out, const AFF_T *pts, const fe_t *scalars, size_t n, int nt) {     \
    G##_jac_set_inf(out);                                                                          \
    if (n == 0) return;                                                                            \
    int c = best_c(n);                                                                             \
    int W = (256 + c - 1) / c;                                                                     \
    u64 (*k)[4] = malloc(sizeof(u64) * 4 * n);                                                     \
    int32_t *dg = malloc(sizeof(int32_t) * n * W);                                                 \
    scalars_canonical(scalars, k, n, nt);                                                          \
    signed_digits((const u64 (*)[4])k, n, c, W, dg, nt);                                           \
    free(k);                                                                                       \
    int chunks = (2 * nt + W - 1) / W;                                                             \
    if ((size_t)chunks > n) chunks = (int)n;                                                       \
    if (chunks < 1) chunks = 1;                                                                    \
    int ntask = W * chunks;                                                                        \
    XYZZ_T *part = malloc(sizeof(XYZZ_T) * ntask);                                                 \
    size_t nb = (size_t)1 << (c - 1);                                                              \
    _Pragma("omp parallel for num_threads(nt) schedule(dynamic)")                                  \
    for (int task = 0; task < ntask; task++) {                                                     \
        int w = task / chunks, ch = task % chunks;                                                 \
        size_t lo = n * ch / chunks, hi = n * (ch + 1) / chunks;                                   \
        XYZZ_T *bk = calloc(nb, sizeof(XYZZ_T));                                                   \
        for (size_t i = lo; i < hi; i++) {                                                         \
            int32_t d = dg[i * W + w];                                                             \
            if (d > 0) G##_xyzz_add_aff(&bk[d - 1], &bk[d - 1], &pts[i], 0);                       \
            else if (d < 0) G##_xyzz_add_aff(&bk[-d - 1], &bk[-d - 1], &pts[i], 1);                \
        }                                                                                          \
        XYZZ_T run, acc;                                                                           \
        G##_xyzz_set_inf(&run); G##_xyzz_set_inf(&acc);                                            \
        for (size_t b = nb; b-- > 0;) {                                                            \
            G##_xyzz_add(&run, &run, &bk[b]);                                                      \
            G##_xyzz_add(&acc, &acc, &run);                                                        \
        }                                                                                          \
        part[task] = acc;                                                                          \
        free(bk);                                                                                  \
    }                                                                                              \
    free(dg);                                                                                      \
    XYZZ_T tot;                                                                                    \
    G##_xyzz_set_inf(&tot);                                                                        \
    for (int w = W - 1; w >= 0; w--) {                                                             \
        for (int i = 0; i < c; i++) G##_xyzz_dbl(&tot, &tot);                                      \
        for (int ch = 0; ch < chunks; ch++) G##_xyzz_add(&tot, &tot, &part[w * chunks + ch]);      \
    }                                                                                              \
    free(part);                                                                                    \
    G##_xyzz_to_jac(out, &tot);                                                                    \
}

MSM_IMPL(g1, g1_aff_t, g1_xyzz_t, g1_jac_t)
MSM_IMPL(g2, g2_aff_t, g2_xyzz_t, g2_jac_t)

/* ---------------- NTT (gnark conventions) ---------------- */
static fe_t *twiddles(const fe_t *w, size_t half, int nt) {
    fe_t *t = malloc(sizeof(fe_t) * (half ? half : 1));
    /* chunked power table */
    int nb = nt * 4;
    if ((size_t)nb > half) nb = half ? (int)half : 1;
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int b = 0; b < nb; b++) {
        size_t lo = half * b / nb, hi = half * (b + 1) / nb;
        if (lo >= hi) continue;
        fe_t x;
        u64 e[4] = {lo, 0, 0, 0};
        fe_pow(&FR, &x, w, e);
        for (size_t i = lo; i < hi; i++) { t[i] = x; fe_mul(&FR, &x, &x, w); }
    }
    return t;
}

static void dif(fe_t *a, size_t n, const fe_t *tw, int nt) {
    for (size_t m = n >> 1; m >= 1; m >>= 1) {
        size_t stride = n / (2 * m);
#pragma omp parallel for num_threads(nt) schedule(static)
        for (size_t b = 0; b < n / 2; b++) {
            size_t blk = b / m, j = b % m;
            size_t i = blk * 2 * m + j;
            fe_t u = a[i], v = a[i + m];
            fe_add(&FR, &a[i], &u, &v);
            fe_t d;
            fe_sub(&FR, &d, &u, &v);
            fe_mul(&FR, &a[i + m], &d, &tw[j * stride]);
        }
    }
}

static void dit(fe_t *a, size_t n, const fe_t *tw, int nt) {
    for (size_t m = 1; m < n; m <<= 1) {
        size_t stride = n / (2 * m);
#pragma omp parallel for num_threads(nt) schedule(static)
        for (size_t b = 0; b < n / 2; b++) {
            size_t blk = b / m, j = b % m;
            size_t i = blk * 2 * m + j;
            fe_t u = a[i], v;
            fe_mul(&FR, &v, &a[i + m], &tw[j * stride]);
            fe_add(&FR, &a[i], &u, &v);
            fe_sub(&FR, &a[i + m], &u, &v);
        }
    }
}

static size_t brev(size_t i, int logn) {
    size_t r = 0;
    for (int b = 0; b < logn; b++) r |= ((i >> b) & 1) << (logn - 1 - b);
    return r;
}

typedef struct {
    int log_n;
    size_t n;
    fe_t w, winv, ninv, g, ginv;
    fe_t *tw, *twinv, *coset, *cosetinv;
} dom_t;

static void dom_init(dom_t *d, int log_n, int nt) {
    d->log_n = log_n;
    d->n = (size_t)1 << log_n;
    fe_t five;
    fe_from_u64(&FR, &five, 5);
    /* omega_n = 5^((r-1)/n) */
    u64 e[4];
    memcpy(e, R_LIMBS, 32);
    e[0] -= 1;
    for (int s = 0; s < log_n; s++) {
        for (int i = 0; i < 3; i++) e[i] = (e[i] >> 1) | (e[i + 1] << 63);
        e[3] >>= 1;
    }
    fe_pow(&FR, &d->w, &five, e);
    fe_inv(&FR, &d->winv, &d->w);
    fe_t nn;
    fe_from_u64(&FR, &nn, d->n);
    fe_inv(&FR, &d->ninv, &nn);
    d->g = five;
    fe_inv(&FR, &d->ginv, &five);
    d->tw = twiddles(&d->w, d->n / 2, nt);
    d->twinv = twiddles(&d->winv, d->n / 2, nt);
    d->coset = twiddles(&d->g, d->n, nt);
    d->cosetinv = twiddles(&d->ginv, d->n, nt);
}

static void dom_free(dom_t *d) { free(d->tw); free(d->twinv); free(d->coset); free(d->cosetinv); }

/* domain.FFT(a, dec, coset) */
static void fft_fwd(dom_t *d, fe_t *a, int is_dif, int coset, int nt) {
    size_t n = d->n;
    if (coset) {
#pragma omp parallel for num_threads(nt) schedule(static)
        for (size_t i = 0; i < n; i++) {
            size_t k = is_dif ? i : brev(i, d->log_n);
            fe_mul(&FR, &a[i], &a[i], &d->coset[k]);
        }
    }
    if (n > 1) { if (is_dif) dif(a, n, d->tw, nt); else dit(a, n, d->tw, nt); }
}

/* domain.FFTInverse(a, dec, coset) */
static void fft_inv(dom_t *d, fe_t *a, int is_dif, int coset, int nt) {
    size_t n = d->n;
    if (n > 1) { if (is_dif) dif(a, n, d->twinv, nt); else dit(a, n, d->twinv, nt); }
#pragma omp parallel for num_threads(nt) schedule(static)
    for (size_t i = 0; i < n; i++) {
        if (coset) {
            size_t k = is_dif ? brev(i, d->log_n) : i;
            fe_mul(&FR, &a[i], &a[i], &d->cosetinv[k]);
        }
        fe_mul(&FR, &a[i], &a[i], &d->ninv);
    }
}

static void compute_h(dom_t *d, fe_t *a, fe_t *b, fe_t *c, int nt) {
    size_t n = d->n;
    fft_inv(d, a, 1, 0, nt);
    fft_inv(d, b, 1, 0, nt);
    fft_inv(d, c, 1, 0, nt);
    fft_fwd(d, a, 0, 1, nt);
    fft_fwd(d, b, 0, 1, nt);
    fft_fwd(d, c, 0, 1, nt);
    fe_t den, one = FR.one;
    u64 e[4] = {n, 0, 0, 0};
    fe_pow(&FR, &den, &d->g, e);
    fe_sub(&FR, &den, &den, &one);
    fe_inv(&FR, &den, &den);
#pragma omp parallel for num_threads(nt) schedule(static)
    for (size_t i = 0; i < n; i++) {
        fe_mul(&FR, &a[i], &a[i], &b[i]);
        fe_sub(&FR, &a[i], &a[i], &c[i]);
        fe_mul(&FR, &a[i], &a[i], &den);
    }
    fft_inv(d, a, 1, 1, nt);
}

/* ====================== exported API ====================== */
static int nthreads(int nt) { return nt > 0 ? nt : omp_get_max_threads(); }

int oc_msm_g1(const void *points, const void *scalars, size_t n, int nt, void *out_aff) {
    oc_init_all();
    g1_jac_t r;
    g1_msm_impl(&r, (const g1_aff_t *)points, (const fe_t *)scalars, n, nthreads(nt));
    g1_jac_to_aff((g1_aff_t *)out_aff, &r);
    return 0;
}

int oc_msm_g2(const void *points, const void *scalars, size_t n, int nt, void *out_aff) {
    oc_init_all();
    g2_jac_t r;
    g2_msm_impl(&r, (const g2_aff_t *)points, (const fe_t *)scalars, n, nthreads(nt));
    g2_jac_to_aff((g2_aff_t *)out_aff, &r);
    return 0;
}

/* out[i] = k_i * base (affine), k_i Montgomery fr; used to build test keys */
int oc_g1_batch_mul(const void *base_aff, const void *scalars, size_t n, int nt, void *out_aff) {
    oc_init_all();
    nt = nthreads(nt);
    const g1_aff_t *b = (const g1_aff_t *)base_aff;
    /* 8-bit fixed-base table: T[w][j] = j * 2^(8w) * base */
    g1_jac_t *T = malloc(sizeof(g1_jac_t) * 32 * 256);
    g1_jac_t bw;
    g1_jac_from_aff(&bw, b);
    for (int w = 0; w < 32; w++) {
        g1_jac_set_inf(&T[w * 256]);
        for (int j = 1; j < 256; j++) g1_jac_add(&T[w * 256 + j], &T[w * 256 + j - 1], &bw);
        for (int s = 0; s < 8; s++) g1_jac_dbl(&bw, &bw);
    }
    g1_aff_t *Ta = malloc(sizeof(g1_aff_t) * 32 * 256);
    g1_batch_to_aff(Ta, T, 32 * 256);
    free(T);
    g1_jac_t *acc = malloc(sizeof(g1_jac_t) * (n ? n : 1));
    const fe_t *sc = (const fe_t *)scalars;
#pragma omp parallel for num_threads(nt) schedule(static)
    for (size_t i = 0; i < n; i++) {
        fe_t k;
        fe_from_mont(&FR, &k, &sc[i]);
        g1_jac_t a;
        g1_jac_set_inf(&a);
        for (int w = 0; w < 32; w++) {
            int j = (int)((k.v[w >> 3] >> ((w & 7) * 8)) & 0xff);
            if (j) g1_jac_add_aff(&a, &a, &Ta[w * 256 + j]);
        }
        acc[i] = a;
    }
    free(Ta);
    /* parallel chunked batch-normalize */
    int nb = nt;
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int c = 0; c < nb; c++) {
        size_t lo = n * c / nb, hi = n * (c + 1) / nb;
        if (hi > lo) g1_batch_to_aff((g1_aff_t *)out_aff + lo, acc + lo, hi - lo);
    }
    free(acc);
    return 0;
}

int oc_g2_batch_mul(const void *base_aff, const void *scalars, size_t n, int nt, void *out_aff) {
    oc_init_all();
    nt = nthreads(nt);
    const g2_aff_t *b = (const g2_aff_t *)base_aff;
    g2_jac_t *T = malloc(sizeof(g2_jac_t) * 32 * 256);
    g2_jac_t bw;
    g2_jac_from_aff(&bw, b);
    for (int w = 0; w < 32; w++) {
        g2_jac_set_inf(&T[w * 256]);
        for (int j = 1; j < 256; j++) g2_jac_add(&T[w * 256 + j], &T[w * 256 + j - 1], &bw);
        for (int s = 0; s < 8; s++) g2_jac_dbl(&bw, &bw);
    }
    g2_aff_t *Ta = malloc(sizeof(g2_aff_t) * 32 * 256);
    g2_batch_to_aff(Ta, T, 32 * 256);
    free(T);
    g2_jac_t *acc = malloc(sizeof(g2_jac_t) * (n ? n : 1));
    const fe_t *sc = (const fe_t *)scalars;
#pragma omp parallel for num_threads(nt) schedule(static)
    for (size_t i = 0; i < n; i++) {
        fe_t k;
        fe_from_mont(&FR, &k, &sc[i]);
        g2_jac_t a;
        g2_jac_set_inf(&a);
        for (int w = 0; w < 32; w++) {
            int j = (int)((k.v[w >> 3] >> ((w & 7) * 8)) & 0xff);
            if (j) g2_jac_add_aff(&a, &a, &Ta[w * 256 + j]);
        }
        acc[i] = a;
    }
    free(Ta);
    int nb = nt;
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int c = 0; c < nb; c++) {
        size_t lo = n * c / nb, hi = n * (c + 1) / nb;
        if (hi > lo) g2_batch_to_aff((g2_aff_t *)out_aff + lo, acc + lo, hi - lo);
    }
    free(acc);
    return 0;
}

/* gnark FFT semantics: inverse=0 -> domain.FFT, 1 -> domain.FFTInverse */
int oc_ntt(void *data, int log_n, int inverse, int is_dif, int coset, int nt) {
    oc_init_all();
    nt = nthreads(nt);
    dom_t d;
    dom_init(&d, log_n, nt);
    if (inverse) fft_inv(&d, (fe_t *)data, is_dif, coset, nt);
    else fft_fwd(&d, (fe_t *)data, is_dif, coset, nt);
    dom_free(&d);
    return 0;
}

/* computeH (prove.go:353-396): a,b,c of length len <= 2^log_n (padded) -> h bit-reversed */
int oc_compute_h(const void *a, const void *b, const void *c, size_t len, int log_n, int nt, void *h_out) {
    oc_init_all();
    nt = nthreads(nt);
    dom_t d;
    dom_init(&d, log_n, nt);
    size_t n = d.n;
    if (len > n) { dom_free(&d); return -1; }
    fe_t *A = calloc(n, sizeof(fe_t)), *B = calloc(n, sizeof(fe_t)), *C = calloc(n, sizeof(fe_t));
    memcpy(A, a, len * 32); memcpy(B, b, len * 32); memcpy(C, c, len * 32);
    compute_h(&d, A, B, C, nt);
    memcpy(h_out, A, n * 32);
    free(A); free(B); free(C);
    dom_free(&d);
    return 0;
}

/* Groth16 Prove after Solve (prove.go:127-320), no commitments.
 * All field/point inputs in gnark memory layout (Montgomery, LE limbs). */
int oc_groth16_prove(
    int log_n,
    const void *g1A, size_t nA, const void *g1B, size_t nB,
    const void *g1Z, const void *g1K, size_t nK,
    const void *alpha1, const void *beta1, const void *delta1,
    const void *g2B, const void *beta2, const void *delta2,
    const uint8_t *infA, const uint8_t *infB,
    const void *wires, size_t nWires, size_t nbPublic,
    const void *solA, const void *solB, const void *solC, size_t nCons,
    const void *r_mont, const void *s_mont, int nt,
    void *outAr, void *outBs, void *outKrs, void *h_out) {
    oc_init_all();
    nt = nthreads(nt);
    size_t n = (size_t)1 << log_n;
    if (nCons > n) return -1;
    fe_t *h = malloc(n * 32);
    if (oc_compute_h(solA, solB, solC, nCons, log_n, nt, h)) { free(h); return -1; }
    if (h_out) memcpy(h_out, h, n * 32);
    const fe_t *w = (const fe_t *)wires;
    fe_t *wA = malloc(sizeof(fe_t) * (nA ? nA : 1)), *wB = malloc(sizeof(fe_t) * (nB ? nB : 1));
    size_t ja = 0, jb = 0;
    for (size_t i = 0; i < nWires; i++) {
        if (!infA[i]) { if (ja < nA) wA[ja] = w[i]; ja++; }
        if (!infB[i]) { if (jb < nB) wB[jb] = w[i]; jb++; }
    }
    if (ja != nA || jb != nB || nWires - nbPublic != nK) { free(h); free(wA); free(wB); return -2; }
    fe_t r, s, kr;
    memcpy(&r, r_mont, 32); memcpy(&s, s_mont, 32);
    fe_mul(&FR, &kr, &r, &s);
    fe_neg(&FR, &kr, &kr);
    fe_t rc, sc, krc;
    fe_from_mont(&FR, &rc, &r); fe_from_mont(&FR, &sc, &s); fe_from_mont(&FR, &krc, &kr);
    g1_jac_t dl, dr, ds, dkr;
    g1_jac_from_aff(&dl, (const g1_aff_t *)delta1);
    g1_jac_mul(&dr, &dl, rc.v); g1_jac_mul(&ds, &dl, sc.v); g1_jac_mul(&dkr, &dl, krc.v);

    g1_jac_t ar, bs1, krs, krs2, t;
    g1_msm_impl(&ar, (const g1_aff_t *)g1A, wA, nA, nt);
    g1_jac_add_aff(&ar, &ar, (const g1_aff_t *)alpha1);
    g1_jac_add(&ar, &ar, &dr);
    g1_msm_impl(&bs1, (const g1_aff_t *)g1B, wB, nB, nt);
    g1_jac_add_aff(&bs1, &bs1, (const g1_aff_t *)beta1);
    g1_jac_add(&bs1, &bs1, &ds);
    g1_msm_impl(&krs2, (const g1_aff_t *)g1Z, h, n - 1, nt);
    g1_msm_impl(&krs, (const g1_aff_t *)g1K, w + nbPublic, nK, nt);
    g1_jac_add(&krs, &krs, &dkr);
    g1_jac_add(&krs, &krs, &krs2);
    g1_jac_mul(&t, &ar, sc.v); g1_jac_add(&krs, &krs, &t);
    g1_jac_mul(&t, &bs1, rc.v); g1_jac_add(&krs, &krs, &t);
    g1_jac_to_aff((g1_aff_t *)outAr, &ar);
    g1_jac_to_aff((g1_aff_t *)outKrs, &krs);

    g2_jac_t bs, d2;
    g2_msm_impl(&bs, (const g2_aff_t *)g2B, wB, nB, nt);
    g2_jac_from_aff(&d2, (const g2_aff_t *)delta2);
    g2_jac_mul(&d2, &d2, sc.v);
    g2_jac_add(&bs, &bs, &d2);
    g2_jac_add_aff(&bs, &bs, (const g2_aff_t *)beta2);
    g2_jac_to_aff((g2_aff_t *)outBs, &bs);
    free(h); free(wA); free(wB);
    return 0;
}

/* small helpers for tests */
int oc_g1_add(const void *a, const void *b, void *out) {
    oc_init_all();
    g1_jac_t x;
    g1_jac_from_aff(&x, (const g1_aff_t *)a);
    g1_jac_add_aff(&x, &x, (const g1_aff_t *)b);
    g1_jac_to_aff((g1_aff_t *)out, &x);
    return 0;
}

int oc_max_threads(void) { return omp_get_max_threads(); }
