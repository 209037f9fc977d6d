// Asynchronous PlonK BLS12-381 device operations (bls12-381 fr, 32 B
// Montgomery), shared by the C-ABI wrappers of plonk.hip / plonk_poly.hip and
// the prover orchestration of plonk_prover.hip.  Nothing here allocates or
// synchronises: scratch comes from the caller's Arena, work is enqueued on `st`.
#pragma once
#include "common.h"
#include "field.cuh"

struct gg_domain;

namespace gg {
namespace plk {

using FrB = FrBls;
constexpr int MAX_CMT = 8;  // BSB22 commitments per circuit
constexpr int MAX_BCOEF = 4;

// polynomial order ids of prove.go:60-77 (s.x)
enum { ID_L, ID_R, ID_O, ID_Z, ID_ZS, ID_QL, ID_QR, ID_QM, ID_QO, ID_QK, ID_S1, ID_S2, ID_S3, ID_ID,
       ID_LONE, ID_QCI };
constexpr int MAX_X = ID_QCI + 2 * MAX_CMT;

// Every operation is a template over the scalar field F (FrBls for
// backend/plonk/bls12-381, Fr for backend/plonk/bn254: the same generated prover
// over another curve); plonk_poly.hip / plonk.hip instantiate both.

// ---- plonk_poly.hip
size_t scan_arena_bytes(size_t m);
// in place inclusive running product
template <class F>
void scan_prod(F* x, size_t m, hipStream_t st, Arena& ar);
size_t horner_arena_bytes(size_t n);
// value_dev[0] = f(a) (Polynomial.Evaluate); q (nullable, n - 1 fr) = (f - f(a)) / (X - a)
template <class F>
void horner(const F* f, size_t n, const F& a, F* q, F* value_dev, hipStream_t st, Arena& ar);
size_t ratio_arena_bytes(size_t n);
// iop.BuildRatioCopyConstraint into Lagrange/Regular z (prove.go:600-621)
template <class F>
void ratio(const F* l, const F* r, const F* o, const int64_t* perm, size_t n, const F& beta, const F& gamma,
           const F& omega, const F& u, F* z, hipStream_t st, Arena& ar);
// BuildRatioCopyConstraint over the slice [lo, lo + cnt) of the factors
// f_i = prod_j (f_j[i] + b ID(j n + i) + g) / (f_j[i] + b ID(S[j n + i]) + g):
// P = their running product inside the slice (P[cnt - 1] = the slice's product).
// l, r, o, perm0..2 point at the slice's entries.  A device part's share of the
// ratio; ratio_fixup then writes its slice of Z: z[0] = prefix, z[t + 1] =
// prefix P[t] (prefix = the product of the factors before lo).
size_t ratio_range_arena_bytes(size_t n, size_t cnt);
template <class F>
void ratio_range(const F* l, const F* r, const F* o, const int64_t* perm0, const int64_t* perm1,
                 const int64_t* perm2, size_t lo, size_t cnt, size_t n, const F& beta, const F& gamma,
                 const F& omega, const F& u, F* P, hipStream_t st, Arena& ar);
template <class F>
void ratio_fixup(const F* P, size_t cnt, const F& prefix, F* z, hipStream_t st);
size_t batch_invert_arena_bytes(size_t n);
template <class F>
void batch_invert(F* a, size_t n, hipStream_t st, Arena& ar);
// Batched Polynomial.Evaluate at one point (prove.go:640-660, 763-775, 800-810:
// every evaluation of a proof at zeta without a quotient): out_dev[k] =
// sum_i f_k[i] a^i for k < count (<= EVAL_MAX).  One pass over the
// polynomials (coalesced, one product per coefficient: Horner over a
// grid-strided slice with multiplier a^G, scaled by a^g), block sums, then one
// small kernel for the totals -- no scan, no host round trip per polynomial.
constexpr int EVAL_MAX = 16;
size_t eval_many_arena_bytes(size_t max_len, int count);
template <class F>
void eval_many(const F* const* f, const size_t* len, int count, const F& a, F* out_dev, hipStream_t st,
               Arena& ar);
// out[j] = sum_k c_k f_k[j] for j < n_out (f_k zero past lens[k]), count <= EVAL_MAX:
// kzg.BatchOpenSinglePoint's folded polynomial (prove.go:823-830) in one pass
template <class F>
void lincomb(F* out, size_t n_out, const F* const* f, const size_t* len, const F* c, int count, hipStream_t st);
template <class F>
void fold_h(const F* h, size_t n_small, const F& z, F* out, hipStream_t st);
template <class F>
struct LinParamsT {
    F* z;  // blinded Z canonical, in/out
    size_t nz;
    const F* s3;
    size_t ns3;
    const F *ql, *qr, *qm, *qo, *qk;
    size_t nq;
    const F* pi2[MAX_CMT];
    F qcp[MAX_CMT];
    int ncmt;
    F s1, s2, alpha, l, r, rl, o, lag;
};
using LinParams = LinParamsT<FrB>;
template <class F>
void linearized(const LinParamsT<F>& P, hipStream_t st);
template <class F>
void bit_reverse(const F* in, F* out, size_t n, hipStream_t st);
template <class F>
void axpy(F* y, const F* x, size_t n, const F& a, hipStream_t st);  // y += a x
template <class F>
void scale(F* y, size_t n, const F& a, hipStream_t st);  // y *= a
template <class F>
void shift_copy(const F* in, F* out, size_t n, hipStream_t st);  // out[i] = in[(i+1) % n]

// ---- plonk.hip
template <class F>
struct NumParamsT {
    const F* x[MAX_X];  // Lagrange-regular evaluations on this coset, length n
    int nx;
    F bcoef[4][MAX_BCOEF];  // blinding polynomials Bl, Br, Bo, Bz (coset-scaled)
    int bdeg[4];            // number of coefficients
    const F* tw0;           // s.twiddles0: omega_small^j, j < n
    F beta, gamma, alpha, cs, css;
    // orderingConstraint's identity terms: a, b, c use ka, kb, kc times x[ID_ID]
    // (x[ID_ID] = beta X with ka = 1, kb = cs, kc = cs^2; or X with ka = beta, ...)
    F ka, kb, kc;
    uint32_t n, log_big, rho, coset;
    F* cres;  // rho * n, bit-reversed big-domain order
    // local_block = 1: cres is only this coset's block of n (the slots
    // [brev(coset) n, (brev(coset) + 1) n) of the big vector), e.g. on another GPU
    uint32_t local_block;
    // x[ID_ZS] == nullptr: ZS[j] = Z[(j + 1) % n] read from x[ID_Z] (no shifted copy);
    // else ZS[j] = x[ID_ZS][(j + zs_shift) % n]
    uint32_t zs_shift;
    // blinding of ZS at tw1[j] (nullptr: tw0[(j + 1) % n])
    const F* tw1;
    // has_out_scale: every result times out_scale (the quotient unit's 1 / (x^n - 1))
    uint32_t has_out_scale;
    F out_scale;
};
using NumParams = NumParamsT<FrB>;
template <class F>
void numerator(const NumParamsT<F>& P, hipStream_t st);
// divideByXMinusOne in place (prove.go:1223-1276), asynchronous; big: a domain of F's curve
template <class F>
void divide_by_xn_minus_one(gg_domain* big, size_t n_small, F* data, hipStream_t st);
// out (bit-reversed, m = n / S) = the fold sum_t kappa^t f[m' + t m] of a
// bit-reversed polynomial of n coefficients: the coefficients whose size-m
// coset FFT with shift s (kappa = s^m) gives f on s <w^S> (a quotient unit's
// class of the big domain, prove.go:995-1017 split over the GPUs)
template <class F>
void fold_brev(const F* in, size_t n, int S, const F& kappa, F* out, hipStream_t st);
// out[j] = in[(s + S j) % n] for j < n / S (the unit's points' twiddles0)
template <class F>
void gather_strided(const F* in, size_t n, int S, int s, F* out, hipStream_t st);

// ---- ntt.hip (the domain's scalar field)
void ntt(gg_domain* d, void* data, int inverse, int dit, int coset, hipStream_t st);

}  // namespace plk
// the distributed coset iFFT of the quotient (ntt.hip): per block, and the tail
void ntt_inverse_dit_noscale(gg_domain* d, void* data, hipStream_t st);
void ntt_tail_inverse_coset(gg_domain* d, void* data, int u, hipStream_t st);
namespace plk {

}  // namespace plk
}  // namespace gg
