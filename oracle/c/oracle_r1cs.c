/* ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle/bn254_oracle.py header).
 *
 * O(n) checker for full-size Groth16 proofs (BASELINE config 4, 2^24
 * constraints), multithreaded:
 *   - a synthetic R1CS of independent MiMC x^5 chains (the shape of
 *     std/hash/mimc/encrypt.go pow5: t = x*x, u = t*t, x' = u*x + k per round),
 *     restating oracle/bn254_oracle.py:mimc_chain_r1cs in CSR form;
 *   - its solver (constraint/bn254/solver.go:418-560 for this shape: the unknown
 *     wire of each constraint is the first O term, coefficient 1);
 *   - the solution vectors A, B, C (solver.go:532-560);
 *   - the proving-key discrete logs of Setup with given toxic waste
 *     (setupABC setup.go:352-434: L_j(t) Lagrange values; K, Z setup.go:212-275,
 *     Z bit-reversed setup.go:265);
 *   - the discrete logs of the proof (Ar, Bs, Krs) for injected r, s
 *     (prove.go:177-299), with h(t) Z(t) = A(t) B(t) - C(t): exact for a
 *     satisfied instance, so the GPU's h is checked through Krs without any
 *     FFT on the CPU side (oracle/bn254_oracle.py:expected_proof_scalars is the
 *     big-int version, cross-checked in tests/test_oracle_c.py).
 * Also: evaluation at a point of a bit-reversed coefficient vector and of a
 * Lagrange-basis vector, for the size-independent identity h (X^n - 1) = AB - C.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>
#include "field.h"

typedef struct {
    size_t ncons, nw, nb_public;
    /* CSR per side (0 = L, 1 = R, 2 = O) */
    size_t *off[3];
    uint32_t *wid[3];
    fe_t *coef[3];
} r1cs_t;

static int nthr(int nt) { return nt > 0 ? nt : omp_get_max_threads(); }

/* K chains x R rounds; chain inputs are wires 1..K, the first nb_public_inputs
 * of them public (nb_public = 1 + nb_public_inputs, wire 0 = ONE). */
void *oc_r1cs_create_mimc(size_t nb_chains, size_t rounds, size_t nb_public_inputs) {
    oracle_field_init();
    if (nb_public_inputs > nb_chains) return NULL;
    r1cs_t *r = calloc(1, sizeof(r1cs_t));
    r->ncons = 3 * nb_chains * rounds;
    r->nw = 1 + nb_chains + 3 * nb_chains * rounds;
    r->nb_public = 1 + nb_public_inputs;
    size_t nterms[3] = {r->ncons, r->ncons, r->ncons + nb_chains * rounds};
    for (int s = 0; s < 3; s++) {
        r->off[s] = malloc(sizeof(size_t) * (r->ncons + 1));
        r->wid[s] = malloc(sizeof(uint32_t) * nterms[s]);
        r->coef[s] = malloc(sizeof(fe_t) * nterms[s]);
        r->off[s][0] = 0;
    }
    size_t j = 0, wid = 1 + nb_chains, to = 0;
    fe_t one = FR.one;
    for (size_t ch = 0; ch < nb_chains; ch++) {
        uint32_t x = (uint32_t)(1 + ch);
        for (size_t rd = 0; rd < rounds; rd++) {
            uint32_t t = (uint32_t)wid, u = (uint32_t)(wid + 1), xn = (uint32_t)(wid + 2);
            wid += 3;
            fe_t k, mk;
            fe_from_u64(&FR, &k, (uint64_t)(rd * 7 + 3));
            fe_neg(&FR, &mk, &k);
            /* x * x = t */
            r->wid[0][j] = x; r->coef[0][j] = one;
            r->wid[1][j] = x; r->coef[1][j] = one;
            r->wid[2][to] = t; r->coef[2][to] = one; to++;
            j++; r->off[0][j] = j; r->off[1][j] = j; r->off[2][j] = to;
            /* t * t = u */
            r->wid[0][j] = t; r->coef[0][j] = one;
            r->wid[1][j] = t; r->coef[1][j] = one;
            r->wid[2][to] = u; r->coef[2][to] = one; to++;
            j++; r->off[0][j] = j; r->off[1][j] = j; r->off[2][j] = to;
            /* u * x = xn - k */
            r->wid[0][j] = u; r->coef[0][j] = one;
            r->wid[1][j] = x; r->coef[1][j] = one;
            r->wid[2][to] = xn; r->coef[2][to] = one; to++;
            r->wid[2][to] = 0; r->coef[2][to] = mk; to++;
            j++; r->off[0][j] = j; r->off[1][j] = j; r->off[2][j] = to;
            x = xn;
        }
    }
    return r;
}

void oc_r1cs_free(void *h) {
    r1cs_t *r = h;
    if (!r) return;
    for (int s = 0; s < 3; s++) { free(r->off[s]); free(r->wid[s]); free(r->coef[s]); }
    free(r);
}

void oc_r1cs_info(void *h, size_t *ncons, size_t *nw, size_t *nb_public) {
    r1cs_t *r = h;
    *ncons = r->ncons;
    *nw = r->nw;
    *nb_public = r->nb_public;
}

static inline void lin(const r1cs_t *r, int s, size_t j, const fe_t *w, fe_t *out) {
    fe_t acc, t;
    memset(&acc, 0, 32);
    for (size_t q = r->off[s][j]; q < r->off[s][j + 1]; q++) {
        fe_mul(&FR, &t, &r->coef[s][q], &w[r->wid[s][q]]);
        fe_add(&FR, &acc, &acc, &t);
    }
    *out = acc;
}

/* wires (Montgomery) from the public + secret inputs (wires 1..nb_chains): each
 * constraint's first O term is the unknown, with coefficient 1. */
int oc_r1cs_solve(void *h, const void *inputs, void *wires_out) {
    r1cs_t *r = h;
    fe_t *w = wires_out;
    memset(w, 0, 32 * r->nw);
    w[0] = FR.one;
    memcpy(&w[1], inputs, 32 * (r->nw - 1 - r->ncons));
    for (size_t j = 0; j < r->ncons; j++) {
        fe_t a, b, rest, t;
        lin(r, 0, j, w, &a);
        lin(r, 1, j, w, &b);
        memset(&rest, 0, 32);
        size_t q0 = r->off[2][j];
        for (size_t q = q0 + 1; q < r->off[2][j + 1]; q++) {
            fe_mul(&FR, &t, &r->coef[2][q], &w[r->wid[2][q]]);
            fe_add(&FR, &rest, &rest, &t);
        }
        if (!fe_eq(&r->coef[2][q0], &FR.one)) return -1;
        fe_mul(&FR, &t, &a, &b);
        fe_sub(&FR, &w[r->wid[2][q0]], &t, &rest);
    }
    return 0;
}

/* A, B, C = L.w, R.w, O.w per constraint; returns the number of unsatisfied ones */
long oc_r1cs_abc(void *h, const void *wires, void *A, void *B, void *C, int nt) {
    r1cs_t *r = h;
    const fe_t *w = wires;
    fe_t *a = A, *b = B, *c = C;
    long bad = 0;
    nt = nthr(nt);
#pragma omp parallel for num_threads(nt) schedule(static) reduction(+ : bad)
    for (size_t j = 0; j < r->ncons; j++) {
        lin(r, 0, j, w, &a[j]);
        lin(r, 1, j, w, &b[j]);
        lin(r, 2, j, w, &c[j]);
        fe_t t;
        fe_mul(&FR, &t, &a[j], &b[j]);
        if (!fe_eq(&t, &c[j])) bad++;
    }
    return bad;
}

/* omega_n = 5^((r-1)/n) (pinned: tests/test_oracle_pins.py) */
static void omega(int log_n, fe_t *w) {
    static const u64 R_LIMBS[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
                                   0x30644e72e131a029ULL};
    u64 e[4];
    memcpy(e, R_LIMBS, 32);
    e[0] -= 1;
    for (int s = 0; s < log_n; s++) {
        for (int i = 0; i < 3; i++) e[i] = (e[i] >> 1) | (e[i + 1] << 63);
        e[3] >>= 1;
    }
    fe_t five;
    fe_from_u64(&FR, &five, 5);
    fe_pow(&FR, w, &five, e);
}

static void pow_u64(fe_t *r, const fe_t *a, u64 k) {
    u64 e[4] = {k, 0, 0, 0};
    fe_pow(&FR, r, a, e);
}

/* L[j] = L_j(x) = w^j (x^n - 1) / (n (x - w^j)), j < cnt <= n; x outside the domain */
static void lagrange_at(int log_n, const fe_t *x, fe_t *L, size_t cnt, int nt) {
    size_t n = (size_t)1 << log_n;
    fe_t w, xn, num, nn, ninv;
    omega(log_n, &w);
    pow_u64(&xn, x, n);
    fe_sub(&FR, &num, &xn, &FR.one);
    fe_from_u64(&FR, &nn, n);
    fe_inv(&FR, &ninv, &nn);
    fe_mul(&FR, &num, &num, &ninv);
    int nb = nt * 8;
#pragma omp parallel for num_threads(nt) schedule(dynamic)
    for (int b = 0; b < nb; b++) {
        size_t lo = cnt * b / nb, hi = cnt * (b + 1) / nb;
        if (lo >= hi) continue;
        fe_t wj;
        pow_u64(&wj, &w, lo);
        fe_t *wp = malloc(sizeof(fe_t) * (hi - lo));
        for (size_t j = lo; j < hi; j++) {
            wp[j - lo] = wj;
            fe_sub(&FR, &L[j], x, &wj);
            fe_mul(&FR, &wj, &wj, &w);
        }
        fe_batch_inv(&FR, &L[lo], hi - lo);
        for (size_t j = lo; j < hi; j++) {
            fe_mul(&FR, &L[j], &L[j], &wp[j - lo]);
            fe_mul(&FR, &L[j], &L[j], &num);
        }
        free(wp);
    }
}

/* Per-wire u_i(t), v_i(t), w_i(t) (setupABC, setup.go:352-434) */
static void setup_abc(const r1cs_t *r, int log_n, const fe_t *tau, fe_t *Au, fe_t *Bv, fe_t *Cw, int nt) {
    fe_t *L = malloc(sizeof(fe_t) * (r->ncons ? r->ncons : 1));
    lagrange_at(log_n, tau, L, r->ncons, nt);
    memset(Au, 0, 32 * r->nw);
    memset(Bv, 0, 32 * r->nw);
    memset(Cw, 0, 32 * r->nw);
    fe_t *dst[3] = {Au, Bv, Cw};
    /* scatter: one thread per side (a wire recurs across constraints) */
#pragma omp parallel for num_threads(nt < 3 ? nt : 3) schedule(static)
    for (int s = 0; s < 3; s++) {
        fe_t t;
        for (size_t j = 0; j < r->ncons; j++)
            for (size_t q = r->off[s][j]; q < r->off[s][j + 1]; q++) {
                fe_mul(&FR, &t, &r->coef[s][q], &L[j]);
                fe_add(&FR, &dst[s][r->wid[s][q]], &dst[s][r->wid[s][q]], &t);
            }
    }
    free(L);
}

static size_t brev(size_t i, int logn) {
    size_t r = 0;
    for (int b = 0; b < logn; b++) r |= ((i >> b) & 1) << (logn - 1 - b);
    return r;
}

/* Discrete logs of the proving key, in pk order (setup.go:212-275):
 *   infA/infB[nw]: 1 where u_i(t) / v_i(t) = 0 (setup.go:212-237)
 *   outA[*nA], outB[*nB]: the non-zero u_i(t), v_i(t) in wire order
 *   outK[nw - nb_public]: (beta u_i + alpha v_i + w_i) / delta, private wires
 *   outZ[n - 1]: t^i (t^n - 1) / delta, bit-reversed (setup.go:259-267) */
int oc_groth16_key_scalars(void *h, int log_n, const void *tau, const void *alpha, const void *beta,
                           const void *delta, uint8_t *infA, uint8_t *infB, void *outA, size_t *nA,
                           void *outB, size_t *nB, void *outK, void *outZ, int nt) {
    r1cs_t *r = h;
    nt = nthr(nt);
    size_t n = (size_t)1 << log_n;
    if (r->ncons > n) return -1;
    const fe_t *t = tau, *al = alpha, *be = beta, *de = delta;
    fe_t *Au = malloc(32 * r->nw), *Bv = malloc(32 * r->nw), *Cw = malloc(32 * r->nw);
    setup_abc(r, log_n, t, Au, Bv, Cw, nt);
    fe_t dinv;
    fe_inv(&FR, &dinv, de);
    fe_t *oa = outA, *ob = outB, *ok = outK, *oz = outZ;
    size_t ja = 0, jb = 0;
    for (size_t i = 0; i < r->nw; i++) {
        infA[i] = fe_is_zero(&Au[i]);
        infB[i] = fe_is_zero(&Bv[i]);
        if (!infA[i]) oa[ja++] = Au[i];
        if (!infB[i]) ob[jb++] = Bv[i];
    }
    *nA = ja;
    *nB = jb;
#pragma omp parallel for num_threads(nt) schedule(static)
    for (size_t i = r->nb_public; i < r->nw; i++) {
        fe_t x, y;
        fe_mul(&FR, &x, be, &Au[i]);
        fe_mul(&FR, &y, al, &Bv[i]);
        fe_add(&FR, &x, &x, &y);
        fe_add(&FR, &x, &x, &Cw[i]);
        fe_mul(&FR, &ok[i - r->nb_public], &x, &dinv);
    }
    /* Z[i] = t^i (t^n - 1) / delta, then bitReverse, keep the first n - 1 */
    fe_t zd;
    pow_u64(&zd, t, n);
    fe_sub(&FR, &zd, &zd, &FR.one);
    fe_mul(&FR, &zd, &zd, &dinv);
    int nb = nt * 4;
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int b = 0; b < nb; b++) {
        size_t lo = n * b / nb, hi = n * (b + 1) / nb;
        fe_t x;
        pow_u64(&x, t, lo);
        fe_mul(&FR, &x, &x, &zd);
        for (size_t i = lo; i < hi; i++) {
            size_t p = brev(i, log_n);
            if (p < n - 1) oz[p] = x;
            fe_mul(&FR, &x, &x, t);
        }
    }
    free(Au); free(Bv); free(Cw);
    return 0;
}

/* Discrete logs (a, b, c) of (Ar, Bs, Krs) for wires w and randomness r, s
 * (prove.go:177-299):
 *   a = alpha + sum w_i u_i(t) + r delta,   b = beta + sum w_i v_i(t) + s delta,
 *   c = (sum_priv w_i (beta u_i + alpha v_i + w_i)(t) + A(t) B(t) - C(t)) / delta
 *       + s a + r b - r s delta
 * with A(t) = sum w_i u_i(t) etc. (h(t) Z(t) = A(t)B(t) - C(t) on a satisfied
 * instance).  Returns -2 if the instance is not satisfied. */
int oc_groth16_expected(void *h, int log_n, const void *tau, const void *alpha, const void *beta,
                        const void *delta, const void *wires, const void *r_mont, const void *s_mont,
                        void *out_abc, int nt) {
    r1cs_t *r = h;
    nt = nthr(nt);
    size_t n = (size_t)1 << log_n;
    if (r->ncons > n) return -1;
    const fe_t *w = wires, *al = alpha, *be = beta, *de = delta;
    fe_t *Au = malloc(32 * r->nw), *Bv = malloc(32 * r->nw), *Cw = malloc(32 * r->nw);
    setup_abc(r, log_n, tau, Au, Bv, Cw, nt);
    /* per-thread partial sums */
    fe_t sa[256], sb[256], sc[256], sp[256];
    if (nt > 256) nt = 256;
    for (int k = 0; k < nt; k++) { memset(&sa[k], 0, 32); sb[k] = sa[k]; sc[k] = sa[k]; sp[k] = sa[k]; }
#pragma omp parallel num_threads(nt)
    {
        int k = omp_get_thread_num();
        fe_t x, y;
#pragma omp for schedule(static)
        for (size_t i = 0; i < r->nw; i++) {
            fe_mul(&FR, &x, &w[i], &Au[i]); fe_add(&FR, &sa[k], &sa[k], &x);
            fe_mul(&FR, &y, &w[i], &Bv[i]); fe_add(&FR, &sb[k], &sb[k], &y);
            fe_t z;
            fe_mul(&FR, &z, &w[i], &Cw[i]); fe_add(&FR, &sc[k], &sc[k], &z);
            if (i >= r->nb_public) {
                fe_t q;
                fe_mul(&FR, &q, be, &x);
                fe_add(&FR, &sp[k], &sp[k], &q);
                fe_mul(&FR, &q, al, &y);
                fe_add(&FR, &sp[k], &sp[k], &q);
                fe_add(&FR, &sp[k], &sp[k], &z);
            }
        }
    }
    fe_t A, B, C, P;
    memset(&A, 0, 32); B = A; C = A; P = A;
    for (int k = 0; k < nt; k++) {
        fe_add(&FR, &A, &A, &sa[k]); fe_add(&FR, &B, &B, &sb[k]);
        fe_add(&FR, &C, &C, &sc[k]); fe_add(&FR, &P, &P, &sp[k]);
    }
    free(Au); free(Bv); free(Cw);
    fe_t rr, ss, a, b, c, t, dinv;
    memcpy(&rr, r_mont, 32);
    memcpy(&ss, s_mont, 32);
    fe_mul(&FR, &t, &rr, de); fe_add(&FR, &a, al, &A); fe_add(&FR, &a, &a, &t);
    fe_mul(&FR, &t, &ss, de); fe_add(&FR, &b, be, &B); fe_add(&FR, &b, &b, &t);
    fe_t hz;
    fe_mul(&FR, &hz, &A, &B);
    fe_sub(&FR, &hz, &hz, &C);
    fe_add(&FR, &c, &P, &hz);
    fe_inv(&FR, &dinv, de);
    fe_mul(&FR, &c, &c, &dinv);
    fe_mul(&FR, &t, &ss, &a); fe_add(&FR, &c, &c, &t);
    fe_mul(&FR, &t, &rr, &b); fe_add(&FR, &c, &c, &t);
    fe_mul(&FR, &t, &rr, &ss); fe_mul(&FR, &t, &t, de); fe_sub(&FR, &c, &c, &t);
    fe_t *o = out_abc;
    o[0] = a; o[1] = b; o[2] = c;
    return 0;
}

/* sum_i coeffs[i] x^bitrev(i): a polynomial stored bit-reversed (h, setup.go:265 order) */
int oc_eval_bitrev(const void *coeffs, int log_n, const void *x, void *out, int nt) {
    oracle_field_init();
    nt = nthr(nt);
    size_t n = (size_t)1 << log_n;
    const fe_t *cf = coeffs;
    int nb = nt * 4;
    fe_t part[1024];
    if (nb > 1024) nb = 1024;
    /* Horner over natural-order coefficient blocks [lo, hi), then scaled by x^lo */
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int b = 0; b < nb; b++) {
        size_t lo = n * b / nb, hi = n * (b + 1) / nb;
        fe_t acc;
        memset(&acc, 0, 32);
        for (size_t k = hi; k-- > lo;) {
            fe_mul(&FR, &acc, &acc, (const fe_t *)x);
            fe_add(&FR, &acc, &acc, &cf[brev(k, log_n)]);
        }
        fe_t xl;
        pow_u64(&xl, (const fe_t *)x, lo);
        fe_mul(&FR, &part[b], &acc, &xl);
    }
    fe_t s;
    memset(&s, 0, 32);
    for (int b = 0; b < nb; b++) fe_add(&FR, &s, &s, &part[b]);
    memcpy(out, &s, 32);
    return 0;
}

/* sum_{j < len} vals[j] L_j(x) on the size-2^log_n domain (the polynomial of
 * evaluations padded with zeros, as computeH's iFFT sees it) */
int oc_eval_lagrange(const void *vals, size_t len, int log_n, const void *x, void *out, int nt) {
    oracle_field_init();
    nt = nthr(nt);
    fe_t *L = malloc(sizeof(fe_t) * (len ? len : 1));
    lagrange_at(log_n, x, L, len, nt);
    const fe_t *v = vals;
    fe_t part[256];
    if (nt > 256) nt = 256;
    for (int k = 0; k < nt; k++) memset(&part[k], 0, 32);
#pragma omp parallel num_threads(nt)
    {
        int k = omp_get_thread_num();
        fe_t t;
#pragma omp for schedule(static)
        for (size_t j = 0; j < len; j++) {
            fe_mul(&FR, &t, &v[j], &L[j]);
            fe_add(&FR, &part[k], &part[k], &t);
        }
    }
    fe_t s;
    memset(&s, 0, 32);
    for (int k = 0; k < nt; k++) fe_add(&FR, &s, &s, &part[k]);
    memcpy(out, &s, 32);
    free(L);
    return 0;
}

/* sum_i a[i] b[i] (fr, Montgomery): the trapdoor MSM(k_i G, s_i) = (sum s_i k_i) G */
int oc_fr_dot(const void *a, const void *b, size_t n, void *out, int nt) {
    oracle_field_init();
    nt = nthr(nt);
    if (nt > 256) nt = 256;
    const fe_t *x = a, *y = b;
    fe_t part[256];
    for (int k = 0; k < nt; k++) memset(&part[k], 0, 32);
#pragma omp parallel num_threads(nt)
    {
        int k = omp_get_thread_num();
        fe_t t;
#pragma omp for schedule(static)
        for (size_t i = 0; i < n; i++) {
            fe_mul(&FR, &t, &x[i], &y[i]);
            fe_add(&FR, &part[k], &part[k], &t);
        }
    }
    fe_t s;
    memset(&s, 0, 32);
    for (int k = 0; k < nt; k++) fe_add(&FR, &s, &s, &part[k]);
    memcpy(out, &s, 32);
    return 0;
}
