/* ORACLE -- TEST INFRASTRUCTURE ONLY.
 * Generic short-Weierstrass (a = 0) arithmetic, instantiated for G1 (Fp) and
 * G2 (Fp2) by oracle_bn254.c.  Restates gnark-crypto G1Jac/G2Jac and the
 * extended-Jacobian (XYZZ) bucket points used by its MultiExp [ext].
 * Required macros: CP (prefix), CF_T, CF_ADD, CF_SUB, CF_MUL, CF_SQR, CF_DBL,
 * CF_NEG, CF_ISZERO, CF_EQ, CF_BATCH_INV, CF_ONE.
 */
#define OC_CAT2(a, b) a##b
#define OC_CAT(a, b) OC_CAT2(a, b)
#define FN(name) OC_CAT(CP, name)

typedef struct { CF_T x, y; } FN(_aff_t);
typedef struct { CF_T x, y, z; } FN(_jac_t);
typedef struct { CF_T x, y, zz, zzz; } FN(_xyzz_t);

static inline int FN(_aff_is_inf)(const FN(_aff_t) *p) { return CF_ISZERO(&p->x) && CF_ISZERO(&p->y); }

static inline void FN(_jac_set_inf)(FN(_jac_t) *p) {
    p->x = CF_ONE; p->y = CF_ONE; memset(&p->z, 0, sizeof(CF_T));
}
static inline int FN(_jac_is_inf)(const FN(_jac_t) *p) { return CF_ISZERO(&p->z); }

static inline void FN(_jac_from_aff)(FN(_jac_t) *r, const FN(_aff_t) *a) {
    if (FN(_aff_is_inf)(a)) { FN(_jac_set_inf)(r); return; }
    r->x = a->x; r->y = a->y; r->z = CF_ONE;
}

/* dbl-2009-l */
static void FN(_jac_dbl)(FN(_jac_t) *r, const FN(_jac_t) *p) {
    if (FN(_jac_is_inf)(p)) { *r = *p; return; }
    CF_T A, B, C, D, E, F, t;
    CF_SQR(&A, &p->x);
    CF_SQR(&B, &p->y);
    CF_SQR(&C, &B);
    CF_ADD(&t, &p->x, &B);
    CF_SQR(&t, &t);
    CF_SUB(&t, &t, &A);
    CF_SUB(&t, &t, &C);
    CF_DBL(&D, &t);
    CF_DBL(&E, &A);
    CF_ADD(&E, &E, &A);
    CF_SQR(&F, &E);
    CF_T Z3;
    CF_MUL(&Z3, &p->y, &p->z);
    CF_DBL(&Z3, &Z3);
    CF_T X3;
    CF_DBL(&t, &D);
    CF_SUB(&X3, &F, &t);
    CF_T Y3;
    CF_SUB(&t, &D, &X3);
    CF_MUL(&Y3, &E, &t);
    CF_DBL(&C, &C); CF_DBL(&C, &C); CF_DBL(&C, &C);
    CF_SUB(&Y3, &Y3, &C);
    r->x = X3; r->y = Y3; r->z = Z3;
}

/* add-2007-bl with doubling fallback */
static void FN(_jac_add)(FN(_jac_t) *r, const FN(_jac_t) *p, const FN(_jac_t) *q) {
    if (FN(_jac_is_inf)(p)) { *r = *q; return; }
    if (FN(_jac_is_inf)(q)) { *r = *p; return; }
    CF_T Z1Z1, Z2Z2, U1, U2, S1, S2, t;
    CF_SQR(&Z1Z1, &p->z);
    CF_SQR(&Z2Z2, &q->z);
    CF_MUL(&U1, &p->x, &Z2Z2);
    CF_MUL(&U2, &q->x, &Z1Z1);
    CF_MUL(&S1, &p->y, &q->z); CF_MUL(&S1, &S1, &Z2Z2);
    CF_MUL(&S2, &q->y, &p->z); CF_MUL(&S2, &S2, &Z1Z1);
    if (CF_EQ(&U1, &U2)) {
        if (CF_EQ(&S1, &S2)) { FN(_jac_dbl)(r, p); return; }
        FN(_jac_set_inf)(r); return;
    }
    CF_T H, I, J, rr, V;
    CF_SUB(&H, &U2, &U1);
    CF_DBL(&I, &H); CF_SQR(&I, &I);
    CF_MUL(&J, &H, &I);
    CF_SUB(&rr, &S2, &S1); CF_DBL(&rr, &rr);
    CF_MUL(&V, &U1, &I);
    CF_T X3, Y3, Z3;
    CF_SQR(&X3, &rr); CF_SUB(&X3, &X3, &J); CF_DBL(&t, &V); CF_SUB(&X3, &X3, &t);
    CF_SUB(&t, &V, &X3); CF_MUL(&Y3, &rr, &t);
    CF_MUL(&t, &S1, &J); CF_DBL(&t, &t); CF_SUB(&Y3, &Y3, &t);
    CF_ADD(&Z3, &p->z, &q->z); CF_SQR(&Z3, &Z3); CF_SUB(&Z3, &Z3, &Z1Z1); CF_SUB(&Z3, &Z3, &Z2Z2);
    CF_MUL(&Z3, &Z3, &H);
    r->x = X3; r->y = Y3; r->z = Z3;
}

static void FN(_jac_add_aff)(FN(_jac_t) *r, const FN(_jac_t) *p, const FN(_aff_t) *q) {
    FN(_jac_t) qj;
    FN(_jac_from_aff)(&qj, q);
    FN(_jac_add)(r, p, &qj);
}

static inline void FN(_jac_neg)(FN(_jac_t) *r, const FN(_jac_t) *p) {
    *r = *p; CF_NEG(&r->y, &p->y);
}

/* scalar k as canonical little-endian u64[4] */
static void FN(_jac_mul)(FN(_jac_t) *r, const FN(_jac_t) *p, const u64 k[4]) {
    FN(_jac_t) acc, base = *p;
    FN(_jac_set_inf)(&acc);
    for (int i = 255; i >= 0; i--) {
        FN(_jac_dbl)(&acc, &acc);
        if ((k[i >> 6] >> (i & 63)) & 1) FN(_jac_add)(&acc, &acc, &base);
    }
    *r = acc;
}

/* batch Jacobian -> affine; infinity -> all-zero */
static void FN(_batch_to_aff)(FN(_aff_t) *out, const FN(_jac_t) *in, size_t n) {
    CF_T *zs = (CF_T *)malloc(sizeof(CF_T) * (n ? n : 1));
    for (size_t i = 0; i < n; i++) zs[i] = in[i].z;
    CF_BATCH_INV(zs, n);
    for (size_t i = 0; i < n; i++) {
        if (CF_ISZERO(&in[i].z)) { memset(&out[i], 0, sizeof(out[i])); continue; }
        CF_T z2, z3;
        CF_SQR(&z2, &zs[i]);
        CF_MUL(&z3, &z2, &zs[i]);
        CF_MUL(&out[i].x, &in[i].x, &z2);
        CF_MUL(&out[i].y, &in[i].y, &z3);
    }
    free(zs);
}

static void FN(_jac_to_aff)(FN(_aff_t) *out, const FN(_jac_t) *in) { FN(_batch_to_aff)(out, in, 1); }

/* ---- XYZZ bucket arithmetic (x = X/ZZ, y = Y/ZZZ) ---- */
static inline void FN(_xyzz_set_inf)(FN(_xyzz_t) *p) { memset(p, 0, sizeof(*p)); }
static inline int FN(_xyzz_is_inf)(const FN(_xyzz_t) *p) { return CF_ISZERO(&p->zz); }

/* dbl-2008-s-1 */
static void FN(_xyzz_dbl)(FN(_xyzz_t) *r, const FN(_xyzz_t) *p) {
    if (FN(_xyzz_is_inf)(p)) { *r = *p; return; }
    CF_T U, V, W, S, M, t;
    CF_DBL(&U, &p->y);
    CF_SQR(&V, &U);
    CF_MUL(&W, &U, &V);
    CF_MUL(&S, &p->x, &V);
    CF_SQR(&M, &p->x); CF_DBL(&t, &M); CF_ADD(&M, &M, &t);
    CF_T X3, Y3;
    CF_SQR(&X3, &M); CF_DBL(&t, &S); CF_SUB(&X3, &X3, &t);
    CF_SUB(&t, &S, &X3); CF_MUL(&Y3, &M, &t);
    CF_MUL(&t, &W, &p->y); CF_SUB(&Y3, &Y3, &t);
    CF_MUL(&r->zz, &V, &p->zz);
    CF_MUL(&r->zzz, &W, &p->zzz);
    r->x = X3; r->y = Y3;
}

/* madd-2008-s with affine q; handles inf / doubling / cancellation */
static void FN(_xyzz_add_aff)(FN(_xyzz_t) *r, const FN(_xyzz_t) *p, const FN(_aff_t) *q, int neg) {
    if (FN(_aff_is_inf)(q)) { *r = *p; return; }
    CF_T qy = q->y;
    if (neg) CF_NEG(&qy, &q->y);
    if (FN(_xyzz_is_inf)(p)) {
        r->x = q->x; r->y = qy; r->zz = CF_ONE; r->zzz = CF_ONE; return;
    }
    CF_T U2, S2, PP, PPP, Pv, Rv, Q, t;
    CF_MUL(&U2, &q->x, &p->zz);
    CF_MUL(&S2, &qy, &p->zzz);
    CF_SUB(&Pv, &U2, &p->x);
    CF_SUB(&Rv, &S2, &p->y);
    if (CF_ISZERO(&Pv)) {
        if (CF_ISZERO(&Rv)) {
            FN(_xyzz_t) a; a.x = q->x; a.y = qy; a.zz = CF_ONE; a.zzz = CF_ONE;
            FN(_xyzz_dbl)(r, &a); return;
        }
        FN(_xyzz_set_inf)(r); return;
    }
    CF_SQR(&PP, &Pv);
    CF_MUL(&PPP, &Pv, &PP);
    CF_MUL(&Q, &p->x, &PP);
    CF_T X3, Y3;
    CF_SQR(&X3, &Rv); CF_SUB(&X3, &X3, &PPP); CF_DBL(&t, &Q); CF_SUB(&X3, &X3, &t);
    CF_SUB(&t, &Q, &X3); CF_MUL(&Y3, &Rv, &t);
    CF_MUL(&t, &p->y, &PPP); CF_SUB(&Y3, &Y3, &t);
    CF_MUL(&r->zz, &p->zz, &PP);
    CF_MUL(&r->zzz, &p->zzz, &PPP);
    r->x = X3; r->y = Y3;
}

/* add-2008-s */
static void FN(_xyzz_add)(FN(_xyzz_t) *r, const FN(_xyzz_t) *p, const FN(_xyzz_t) *q) {
    if (FN(_xyzz_is_inf)(p)) { *r = *q; return; }
    if (FN(_xyzz_is_inf)(q)) { *r = *p; return; }
    CF_T U1, U2, S1, S2, Pv, Rv, PP, PPP, Q, t;
    CF_MUL(&U1, &p->x, &q->zz);
    CF_MUL(&U2, &q->x, &p->zz);
    CF_MUL(&S1, &p->y, &q->zzz);
    CF_MUL(&S2, &q->y, &p->zzz);
    CF_SUB(&Pv, &U2, &U1);
    CF_SUB(&Rv, &S2, &S1);
    if (CF_ISZERO(&Pv)) {
        if (CF_ISZERO(&Rv)) { FN(_xyzz_dbl)(r, p); return; }
        FN(_xyzz_set_inf)(r); return;
    }
    CF_SQR(&PP, &Pv);
    CF_MUL(&PPP, &Pv, &PP);
    CF_MUL(&Q, &U1, &PP);
    CF_T X3, Y3, ZZ3, ZZZ3;
    CF_SQR(&X3, &Rv); CF_SUB(&X3, &X3, &PPP); CF_DBL(&t, &Q); CF_SUB(&X3, &X3, &t);
    CF_SUB(&t, &Q, &X3); CF_MUL(&Y3, &Rv, &t);
    CF_MUL(&t, &S1, &PPP); CF_SUB(&Y3, &Y3, &t);
    CF_MUL(&ZZ3, &p->zz, &q->zz); CF_MUL(&ZZ3, &ZZ3, &PP);
    CF_MUL(&ZZZ3, &p->zzz, &q->zzz); CF_MUL(&ZZZ3, &ZZZ3, &PPP);
    r->x = X3; r->y = Y3; r->zz = ZZ3; r->zzz = ZZZ3;
}

/* XYZZ -> Jacobian (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2): Z' = ZZZ,
 * X' = X*ZZ^2, Y' = Y*ZZZ^2 (gnark-crypto fromJacExtended [ext]). */
static void FN(_xyzz_to_jac)(FN(_jac_t) *r, const FN(_xyzz_t) *p) {
    if (FN(_xyzz_is_inf)(p)) { FN(_jac_set_inf)(r); return; }
    CF_T t;
    CF_SQR(&t, &p->zz);
    CF_MUL(&r->x, &p->x, &t);
    CF_SQR(&t, &p->zzz);
    CF_MUL(&r->y, &p->y, &t);
    r->z = p->zzz;
}

#undef FN
