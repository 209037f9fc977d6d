/* ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle/bn254_oracle.py header).
 *
 * BN254 Fp / Fr Montgomery arithmetic, 4 x u64 little-endian limbs, R = 2^256:
 * the in-memory layout of gnark-crypto fp.Element / fr.Element [ext,
 * gnark-crypto v0.12.2-0.20231117165148-e77308824822, go.mod:8].
 * Moduli: backend/groth16/bn254/solidity.go:41-42.
 */
#ifndef ORACLE_FIELD_H
#define ORACLE_FIELD_H
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;

typedef struct { u64 v[4]; } fe_t;

typedef struct {
    u64 p[4];
    u64 inv;      /* -p^{-1} mod 2^64 */
    fe_t r2;      /* R^2 mod p */
    fe_t one;     /* R mod p */
} field_t;

extern field_t FP, FR;
void oracle_field_init(void);

static inline int fe_is_zero(const fe_t *a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
static inline int fe_eq(const fe_t *a, const fe_t *b) { return memcmp(a, b, 32) == 0; }

static inline int geq_p(const u64 t[4], const u64 p[4]) {
    for (int i = 3; i >= 0; i--) {
        if (t[i] > p[i]) return 1;
        if (t[i] < p[i]) return 0;
    }
    return 1;
}

static inline void sub_p(u64 t[4], const u64 p[4]) {
    u64 b = 0;
    for (int i = 0; i < 4; i++) {
        u128 x = (u128)t[i] - p[i] - b;
        t[i] = (u64)x;
        b = (u64)(x >> 64) & 1;
    }
}

static inline void fe_add(const field_t *F, fe_t *r, const fe_t *a, const fe_t *b) {
    u64 c = 0;
    u64 t[4];
    for (int i = 0; i < 4; i++) {
        u128 x = (u128)a->v[i] + b->v[i] + c;
        t[i] = (u64)x;
        c = (u64)(x >> 64);
    }
    if (c || geq_p(t, F->p)) sub_p(t, F->p);
    memcpy(r->v, t, 32);
}

static inline void fe_sub(const field_t *F, fe_t *r, const fe_t *a, const fe_t *b) {
    u64 bo = 0;
    u64 t[4];
    for (int i = 0; i < 4; i++) {
        u128 x = (u128)a->v[i] - b->v[i] - bo;
        t[i] = (u64)x;
        bo = (u64)(x >> 64) & 1;
    }
    if (bo) {
        u64 c = 0;
        for (int i = 0; i < 4; i++) {
            u128 x = (u128)t[i] + F->p[i] + c;
            t[i] = (u64)x;
            c = (u64)(x >> 64);
        }
    }
    memcpy(r->v, t, 32);
}

static inline void fe_neg(const field_t *F, fe_t *r, const fe_t *a) {
    if (fe_is_zero(a)) { memset(r, 0, 32); return; }
    fe_t z; memset(&z, 0, 32);
    fe_sub(F, r, &z, a);
}

/* CIOS Montgomery multiplication */
static inline void fe_mul(const field_t *F, fe_t *r, const fe_t *a, const fe_t *b) {
    u64 t[6] = {0, 0, 0, 0, 0, 0};
    const u64 *p = F->p;
    for (int i = 0; i < 4; i++) {
        u64 carry = 0;
        for (int j = 0; j < 4; j++) {
            u128 x = (u128)a->v[j] * b->v[i] + t[j] + carry;
            t[j] = (u64)x;
            carry = (u64)(x >> 64);
        }
        u128 x = (u128)t[4] + carry;
        t[4] = (u64)x;
        t[5] = (u64)(x >> 64);
        u64 m = t[0] * F->inv;
        x = (u128)m * p[0] + t[0];
        carry = (u64)(x >> 64);
        for (int j = 1; j < 4; j++) {
            x = (u128)m * p[j] + t[j] + carry;
            t[j - 1] = (u64)x;
            carry = (u64)(x >> 64);
        }
        x = (u128)t[4] + carry;
        t[3] = (u64)x;
        t[4] = t[5] + (u64)(x >> 64);
    }
    if (t[4] || geq_p(t, p)) sub_p(t, p);
    memcpy(r->v, t, 32);
}

static inline void fe_sqr(const field_t *F, fe_t *r, const fe_t *a) { fe_mul(F, r, a, a); }

static inline void fe_dbl(const field_t *F, fe_t *r, const fe_t *a) { fe_add(F, r, a, a); }

/* canonical (non-Montgomery) integer <-> Montgomery */
static inline void fe_to_mont(const field_t *F, fe_t *r, const fe_t *a) { fe_mul(F, r, a, &F->r2); }
static inline void fe_from_mont(const field_t *F, fe_t *r, const fe_t *a) {
    fe_t one = {{1, 0, 0, 0}};
    fe_mul(F, r, a, &one);
}

void fe_pow(const field_t *F, fe_t *r, const fe_t *a, const u64 e[4]);
void fe_inv(const field_t *F, fe_t *r, const fe_t *a);
void fe_from_u64(const field_t *F, fe_t *r, u64 x);
/* batch inversion (Montgomery trick); zeros stay zero */
void fe_batch_inv(const field_t *F, fe_t *a, size_t n);

/* Fp2 = Fp[u]/(u^2+1) */
typedef struct { fe_t a0, a1; } fe2_t;

static inline void fe2_add(fe2_t *r, const fe2_t *a, const fe2_t *b) {
    fe_add(&FP, &r->a0, &a->a0, &b->a0);
    fe_add(&FP, &r->a1, &a->a1, &b->a1);
}
static inline void fe2_sub(fe2_t *r, const fe2_t *a, const fe2_t *b) {
    fe_sub(&FP, &r->a0, &a->a0, &b->a0);
    fe_sub(&FP, &r->a1, &a->a1, &b->a1);
}
static inline void fe2_neg(fe2_t *r, const fe2_t *a) {
    fe_neg(&FP, &r->a0, &a->a0);
    fe_neg(&FP, &r->a1, &a->a1);
}
static inline void fe2_mul(fe2_t *r, const fe2_t *a, const fe2_t *b) {
    fe_t t0, t1, t2, t3;
    fe_mul(&FP, &t0, &a->a0, &b->a0);
    fe_mul(&FP, &t1, &a->a1, &b->a1);
    fe_add(&FP, &t2, &a->a0, &a->a1);
    fe_add(&FP, &t3, &b->a0, &b->a1);
    fe_mul(&FP, &t2, &t2, &t3);
    fe_sub(&FP, &t2, &t2, &t0);
    fe_sub(&FP, &r->a1, &t2, &t1);
    fe_sub(&FP, &r->a0, &t0, &t1);
}
static inline void fe2_sqr(fe2_t *r, const fe2_t *a) { fe2_mul(r, a, a); }
static inline void fe2_dbl(fe2_t *r, const fe2_t *a) { fe2_add(r, a, a); }
static inline int fe2_is_zero(const fe2_t *a) { return fe_is_zero(&a->a0) && fe_is_zero(&a->a1); }
static inline int fe2_eq(const fe2_t *a, const fe2_t *b) { return memcmp(a, b, 64) == 0; }
void fe2_inv(fe2_t *r, const fe2_t *a);
void fe2_batch_inv(fe2_t *a, size_t n);

#endif
