// Short-Weierstrass (a = 0) arithmetic for BN254 G1 (over Fp) and G2 (over Fp2),
// host + device.  Coordinate systems:
//   Affine<F>  {x, y}            gnark G1Affine/G2Affine layout; infinity = (0, 0)
//   Xyzz<F>    {X, Y, ZZ, ZZZ}   x = X/ZZ, y = Y/ZZZ  (bucket accumulators)
//   Jac<F>     {X, Y, Z}         x = X/Z^2, y = Y/Z^3 (gnark G1Jac/G2Jac layout,
//                                the MsmOnDevice return type at icicle.go:302)
// Formulas: madd-2008-s, add-2008-s, dbl-2008-s-1 (XYZZ); add-2007-bl,
// dbl-2009-l (Jacobian), all for a = 0.
#pragma once
#include "field.cuh"

namespace gg {

template <class F>
struct Affine {
    F x, y;
    GG_HD bool is_inf() const { return x.is_zero() && y.is_zero(); }
    static GG_HD Affine inf() { return Affine{F::zero(), F::zero()}; }
};

template <class F>
struct Xyzz {
    F x, y, zz, zzz;
    static GG_HD Xyzz inf() { return Xyzz{F::zero(), F::zero(), F::zero(), F::zero()}; }
    GG_HD bool is_inf() const { return zz.is_zero(); }
    static GG_HD Xyzz from_affine(const Affine<F>& a) {
        if (a.is_inf()) return inf();
        return Xyzz{a.x, a.y, F::one(), F::one()};
    }
};

template <class F>
struct Jac {
    F x, y, z;
    static GG_HD Jac inf() { return Jac{F::one(), F::one(), F::zero()}; }
    GG_HD bool is_inf() const { return z.is_zero(); }
    static GG_HD Jac from_affine(const Affine<F>& a) {
        if (a.is_inf()) return inf();
        return Jac{a.x, a.y, F::one()};
    }
};

template <class F>
GG_HD Affine<F> neg(const Affine<F>& a) {
    return Affine<F>{a.x, -a.y};
}

// dbl-2008-s-1
template <class F>
GG_HD Xyzz<F> xyzz_dbl(const Xyzz<F>& p) {
    F U = dbl(p.y);
    F V = sqr(U);
    F W = U * V;
    F S = p.x * V;
    F xx = sqr(p.x);
    F M = xx + dbl(xx);
    F X3 = sqr(M) - dbl(S);
    F Y3 = M * (S - X3) - W * p.y;
    return Xyzz<F>{X3, Y3, V * p.zz, W * p.zzz};
}

// mdbl-2008-s-1 (affine input, not infinity)
template <class F>
GG_HD Xyzz<F> xyzz_dbl_affine(const Affine<F>& q) {
    F U = dbl(q.y);
    F V = sqr(U);
    F W = U * V;
    F S = q.x * V;
    F xx = sqr(q.x);
    F M = xx + dbl(xx);
    F X3 = sqr(M) - dbl(S);
    F Y3 = M * (S - X3) - W * q.y;
    return Xyzz<F>{X3, Y3, V, W};
}

// madd-2008-s: p + q, q affine and NOT infinity; handles p = inf, p = q, p = -q.
template <class F>
GG_HD Xyzz<F> xyzz_madd(const Xyzz<F>& p, const Affine<F>& q) {
    if (p.is_inf()) return Xyzz<F>{q.x, q.y, F::one(), F::one()};
    F U2 = q.x * p.zz;
    F S2 = q.y * p.zzz;
    F P = U2 - p.x;
    F R = S2 - p.y;
    if (P.is_zero()) {
        if (R.is_zero()) return xyzz_dbl_affine(q);
        return Xyzz<F>::inf();
    }
    F PP = sqr(P);
    F PPP = P * PP;
    F Q = p.x * PP;
    F X3 = sqr(R) - PPP - dbl(Q);
    F Y3 = mul_sub(R, Q - X3, p.y, PPP);
    return Xyzz<F>{X3, Y3, p.zz * PP, p.zzz * PPP};
}

// madd-2008-s in place, ordered to keep few temporaries live (ZZ/ZZZ are
// updated as soon as PP/PPP exist, X2/Y2 die right after first use).  Same
// results as xyzz_madd; this is the bucket-accumulation hot loop.
template <class F>
GG_HD void xyzz_madd_inplace(Xyzz<F>& p, const Affine<F>& q) {
    if (p.is_inf()) {
        p = Xyzz<F>{q.x, q.y, F::one(), F::one()};
        return;
    }
    F P = q.x * p.zz - p.x;
    F R = q.y * p.zzz - p.y;
    if (P.is_zero()) {
        p = R.is_zero() ? xyzz_dbl_affine(q) : Xyzz<F>::inf();
        return;
    }
    F PP = sqr(P);
    p.zz = p.zz * PP;
    F PPP = P * PP;
    p.zzz = p.zzz * PPP;
    F Q = p.x * PP;
    F X3 = sqr(R) - PPP - dbl(Q);
    p.y = mul_sub(R, Q - X3, p.y, PPP);
    p.x = X3;
}

// add-2008-s
template <class F>
GG_HD Xyzz<F> xyzz_add(const Xyzz<F>& p, const Xyzz<F>& q) {
    if (p.is_inf()) return q;
    if (q.is_inf()) return p;
    F U1 = p.x * q.zz;
    F U2 = q.x * p.zz;
    F S1 = p.y * q.zzz;
    F S2 = q.y * p.zzz;
    F P = U2 - U1;
    F R = S2 - S1;
    if (P.is_zero()) {
        if (R.is_zero()) return xyzz_dbl(p);
        return Xyzz<F>::inf();
    }
    F PP = sqr(P);
    F PPP = P * PP;
    F Q = U1 * PP;
    F X3 = sqr(R) - PPP - dbl(Q);
    F Y3 = mul_sub(R, Q - X3, S1, PPP);
    return Xyzz<F>{X3, Y3, p.zz * q.zz * PP, p.zzz * q.zzz * PPP};
}

// add-2008-s in place (p += q), ordered for low register pressure
template <class F>
GG_HD void xyzz_add_inplace(Xyzz<F>& p, const Xyzz<F>& q) {
    if (q.is_inf()) return;
    if (p.is_inf()) {
        p = q;
        return;
    }
    F U1 = p.x * q.zz;
    F S1 = p.y * q.zzz;
    F P = q.x * p.zz - U1;
    F R = q.y * p.zzz - S1;
    if (P.is_zero()) {
        p = R.is_zero() ? xyzz_dbl(p) : Xyzz<F>::inf();
        return;
    }
    F PP = sqr(P);
    p.zz = p.zz * q.zz * PP;
    F PPP = P * PP;
    p.zzz = p.zzz * q.zzz * PPP;
    F Q = U1 * PP;
    p.x = sqr(R) - PPP - dbl(Q);
    p.y = mul_sub(R, Q - p.x, S1, PPP);
}

// XYZZ -> Jacobian: Z = ZZZ, X = X*ZZ^2, Y = Y*ZZZ^2
template <class F>
GG_HD Jac<F> xyzz_to_jac(const Xyzz<F>& p) {
    if (p.is_inf()) return Jac<F>::inf();
    return Jac<F>{p.x * sqr(p.zz), p.y * sqr(p.zzz), p.zzz};
}

// Jacobian -> XYZZ: ZZ = Z^2, ZZZ = Z^3
template <class F>
GG_HD Xyzz<F> jac_to_xyzz(const Jac<F>& p) {
    if (p.is_inf()) return Xyzz<F>::inf();
    F zz = sqr(p.z);
    return Xyzz<F>{p.x, p.y, zz, zz * p.z};
}

// dbl-2009-l
template <class F>
GG_HD Jac<F> jac_dbl(const Jac<F>& p) {
    if (p.is_inf()) return p;
    F A = sqr(p.x);
    F B = sqr(p.y);
    F C = sqr(B);
    F D = dbl(sqr(p.x + B) - A - C);
    F E = A + dbl(A);
    F Fv = sqr(E);
    F X3 = Fv - dbl(D);
    F C8 = dbl(dbl(dbl(C)));
    F Y3 = E * (D - X3) - C8;
    F Z3 = dbl(p.y * p.z);
    return Jac<F>{X3, Y3, Z3};
}

// add-2007-bl with doubling / cancellation handling
template <class F>
GG_HD Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) {
    if (p.is_inf()) return q;
    if (q.is_inf()) return p;
    F Z1Z1 = sqr(p.z), Z2Z2 = sqr(q.z);
    F U1 = p.x * Z2Z2, U2 = q.x * Z1Z1;
    F S1 = p.y * q.z * Z2Z2, S2 = q.y * p.z * Z1Z1;
    if (U1 == U2) {
        if (S1 == S2) return jac_dbl(p);
        return Jac<F>::inf();
    }
    F H = U2 - U1;
    F I = sqr(dbl(H));
    F J = H * I;
    F r = dbl(S2 - S1);
    F V = U1 * I;
    F X3 = sqr(r) - J - dbl(V);
    F Y3 = r * (V - X3) - dbl(S1 * J);
    F Z3 = (sqr(p.z + q.z) - Z1Z1 - Z2Z2) * H;
    return Jac<F>{X3, Y3, Z3};
}

template <class F>
GG_HD Jac<F> jac_add_affine(const Jac<F>& p, const Affine<F>& q) {
    return jac_add(p, Jac<F>::from_affine(q));
}

// k * p, k canonical (non-Montgomery) little-endian u32[8]
template <class F>
GG_HD Jac<F> jac_mul(const Jac<F>& p, const uint32_t k[8]) {
    Jac<F> acc = Jac<F>::inf();
    int top = 255;
    while (top >= 0 && !((k[top >> 5] >> (top & 31)) & 1)) top--;
    for (int i = top; i >= 0; i--) {
        acc = jac_dbl(acc);
        if ((k[i >> 5] >> (i & 31)) & 1) acc = jac_add(acc, p);
    }
    return acc;
}

template <class F>
GG_HD Affine<F> jac_to_affine(const Jac<F>& p) {
    if (p.is_inf()) return Affine<F>::inf();
    F zi = inverse(p.z);
    F zi2 = sqr(zi);
    return Affine<F>{p.x * zi2, p.y * zi2 * zi};
}

using G1Affine = Affine<Fp>;
using G2Affine = Affine<Fp2>;
using G1Xyzz = Xyzz<Fp>;
using G2Xyzz = Xyzz<Fp2>;
using G1Jac = Jac<Fp>;
using G2Jac = Jac<Fp2>;

}  // namespace gg
