// R1CS solver on the GPU: constraint/bn254/solver.go:418-608
// (run + solveR1C) for R1CS without hint calls, BN254 or BLS12-381 fr
// (gg_r1cs_create_ex; constraint/bls12-381/solver.go is the same code).
//
// The system is handed over once in CSR form -- exactly what gnark's public
// R1CS API yields (r1cs.GetR1Cs() terms, r1cs.Coefficients, r1cs.Levels):
//   term_off[3 c + s] .. term_off[3 c + s + 1]   terms of side s (L, R, O) of c
//   term_wire[t], term_coeff[t]                   wire id and coefficient index
//   coeffs                                        fr table (Montgomery)
//   level_off / level_cons                        r1cs.Levels flattened
// A solve runs one launch per level (constraints of a level are independent,
// solver.go:421-428), a thread per constraint:
//   a, b, c = sum of the solved terms of L, R, O (accumulateInto);
//   at most one unsolved term: its wire gets (c / b - a), (c / a - b) or
//   (a b - c), divided by its coefficient (divByCoeff), and the term joins its
//   side's sum; no unsolved term: a b == c is checked (solver.go:553-571);
//   a zero divisor leaves the wire at 0 after the same check (solver.go:582-601).
// Outputs W (wires) and A, B, C (per-constraint L.w, R.w, O.w: R1CSSolution,
// system.go:269-272) stay in HBM for gg_groth16_prove (inputs_on_device = 1).
// The level loop is captured once into a HIP graph per handle (256+ tiny
// launches per solve otherwise).
#include "common.h"
#include "field.cuh"
#include "strands.h"
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

namespace gg {

template <class FC>
struct R1csDev {
    using Fr = Fe<FC>;
    const uint32_t* off;
    const uint32_t* wire;
    const uint32_t* cidx;
    const Fr* coef;
    const Fr* coef_inv;
    uint32_t ncoef;
    uint32_t one_idx;  // index of the coefficient 1 (CoeffIdOne), ~0 if absent: no product
    uint32_t nin;      // wires < nin are ONE_WIRE + the witness (never written by a solve)
    Fr* W;
    Fr* A;
    Fr* B;
    Fr* C;
    uint8_t* solved;
    uint32_t* fail;  // [0] = first unsatisfied constraint, [1] = first malformed one
};

template <class F>
__device__ __forceinline__ F ldfr(const F* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    F r;
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    return r;
}
template <class F>
__device__ __forceinline__ void stfr(F* p, const F& r) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(r.v[0], r.v[1], r.v[2], r.v[3]);
    q[1] = make_uint4(r.v[4], r.v[5], r.v[6], r.v[7]);
}

template <class FC>
__global__ void __launch_bounds__(256) k_solve_level(R1csDev<FC> d, const uint32_t* cons, uint32_t count) {
    using Fr = Fe<FC>;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t c = cons[i];
    Fr acc[3] = {Fr::zero(), Fr::zero(), Fr::zero()};
    int loc = -1;
    uint32_t ut = 0;
    bool malformed = false;
    for (int s = 0; s < 3; s++) {
        const uint32_t t0 = d.off[3 * c + s], t1 = d.off[3 * c + s + 1];
        for (uint32_t t = t0; t < t1; t++) {
            const uint32_t w = d.wire[t];
            if (d.solved[w]) {
                const uint32_t k = d.cidx[t];
                acc[s] = acc[s] + (k == d.one_idx ? ldfr(d.W + w) : ldfr(d.coef + k) * ldfr(d.W + w));
                continue;
            }
            if (loc >= 0) malformed = true;  // "found more than one wire to instantiate"
            loc = s;
            ut = t;
        }
    }
    bool ok = true;
    if (malformed) {
        atomicMin(d.fail + 1, c);
        ok = false;
    } else if (loc < 0) {
        ok = acc[0] * acc[1] == acc[2];
    } else {
        Fr v = Fr::zero();
        const Fr a = acc[0], b = acc[1], cc = acc[2];
        if (loc == 0) {
            if (!b.is_zero()) { v = cc * inverse(b) - a; acc[0] = a + v; }
            else ok = a * b == cc;
        } else if (loc == 1) {
            if (!a.is_zero()) { v = cc * inverse(a) - b; acc[1] = b + v; }
            else ok = a * b == cc;
        } else {
            v = a * b - cc;
            acc[2] = cc + v;
        }
        const uint32_t k = d.cidx[ut];
        const Fr kinv = ldfr(d.coef_inv + k);
        if (kinv.is_zero()) {  // zero coefficient on the unknown: no division possible
            atomicMin(d.fail + 1, c);
            ok = false;
        }
        const uint32_t w = d.wire[ut];
        stfr(d.W + w, k == d.one_idx ? v : v * kinv);
        d.solved[w] = 1;
    }
    if (!ok) atomicMin(d.fail, c);
    stfr(d.A + c, acc[0]);
    stfr(d.B + c, acc[1]);
    stfr(d.C + c, acc[2]);
}

// W read around the (write-through, non-coherent) L1: within a strand kernel a
// thread reads values it stored earlier in the same launch
template <class F>
__device__ __forceinline__ F ldfr_l2(const F* p) {
    const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
    F r;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t x = __hip_atomic_load(q + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.v[2 * k] = (uint32_t)x;
        r.v[2 * k + 1] = (uint32_t)(x >> 32);
    }
    return r;
}

// Strand schedule (solve_strands): thread s walks segment s of this launch --
// consecutive constraints of one dependency chain -- in order; the unknown
// term of each constraint is known statically (unk[c], ~0 = none), so no
// solved flags are read inside the launch.  Dependencies on other strands were
// solved by earlier launches.
template <class FC>
__global__ void __launch_bounds__(256) k_solve_strands(R1csDev<FC> d, const uint32_t* unk, const uint32_t* order,
                                                       const uint32_t* seg_start, uint32_t nseg) {
    using Fr = Fe<FC>;
    const uint32_t sg = blockIdx.x * blockDim.x + threadIdx.x;
    if (sg >= nseg) return;
    // the last RC wires this thread produced, kept in registers: a chain reads
    // its own recent outputs (the MiMC rounds: all of them)
    constexpr int RC = 4;
    uint32_t cw[RC];
    Fr cv[RC];
#pragma unroll
    for (int k = 0; k < RC; k++) cw[k] = 0xffffffffu;
    int cpos = 0;
    for (uint32_t i = seg_start[sg], e = seg_start[sg + 1]; i < e; i++) {
        const uint32_t c = order[i], ut = unk[c];
        Fr acc[3] = {Fr::zero(), Fr::zero(), Fr::zero()};
        int loc = -1;
        for (int s = 0; s < 3; s++) {
            const uint32_t t0 = d.off[3 * c + s], t1 = d.off[3 * c + s + 1];
            for (uint32_t t = t0; t < t1; t++) {
                if (t == ut) {
                    loc = s;
                    continue;
                }
                const uint32_t k = d.cidx[t], w = d.wire[t];
                Fr x;
                int hit = -1;
#pragma unroll
                for (int q = 0; q < RC; q++)
                    if (cw[q] == w) hit = q;
                if (hit >= 0) {
#pragma unroll
                    for (int q = 0; q < RC; q++)
                        if (q == hit) x = cv[q];
                } else {
                    x = w < d.nin ? ldfr(d.W + w) : ldfr_l2(d.W + w);
                }
                acc[s] = acc[s] + (k == d.one_idx ? x : ldfr(d.coef + k) * x);
            }
        }
        bool ok = true;
        if (loc < 0) {
            ok = acc[0] * acc[1] == acc[2];
        } else {
            Fr v = Fr::zero();
            const Fr a = acc[0], b = acc[1], cc = acc[2];
            if (loc == 0) {
                if (!b.is_zero()) { v = cc * inverse(b) - a; acc[0] = a + v; }
                else ok = a * b == cc;
            } else if (loc == 1) {
                if (!a.is_zero()) { v = cc * inverse(a) - b; acc[1] = b + v; }
                else ok = a * b == cc;
            } else {
                v = a * b - cc;
                acc[2] = cc + v;
            }
            const uint32_t k = d.cidx[ut];
            const Fr kinv = ldfr(d.coef_inv + k);
            if (kinv.is_zero()) {
                atomicMin(d.fail + 1, c);
                ok = false;
            }
            const uint32_t w = d.wire[ut];
            const Fr val = k == d.one_idx ? v : v * kinv;
            stfr(d.W + w, val);
            d.solved[w] = 1;
#pragma unroll
            for (int q = 0; q < RC; q++)
                if (q == cpos) {
                    cw[q] = w;
                    cv[q] = val;
                }
            cpos = (cpos + 1) & (RC - 1);
        }
        if (!ok) atomicMin(d.fail, c);
        stfr(d.A + c, acc[0]);
        stfr(d.B + c, acc[1]);
        stfr(d.C + c, acc[2]);
    }
}

template <class FC>
__global__ void k_solver_init(Fe<FC>* W, uint8_t* solved, size_t nw, const Fe<FC>* inputs, size_t n_in,
                              uint32_t* fail) {
    using Fr = Fe<FC>;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        fail[0] = 0xffffffffu;
        fail[1] = 0xffffffffu;
    }
    if (i >= nw) return;
    if (i == 0) stfr(W, Fr::one());  // ONE_WIRE (solver.go:103-105)
    else if (i <= n_in) stfr(W + i, ldfr(inputs + (i - 1)));
    else stfr(W + i, Fr::zero());
    solved[i] = i <= n_in ? 1 : 0;
}

// number of unsolved wires (solver.go:530-532)
__global__ void k_count_unsolved(const uint8_t* solved, size_t nw, unsigned long long* cnt) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool u = i < nw && !solved[i];
    const unsigned long long b = __ballot(u);
    if (u && (threadIdx.x & 63) == (uint32_t)(__ffsll(b) - 1)) atomicAdd(cnt, (unsigned long long)__popcll(b));
}

}  // namespace gg

using namespace gg;

struct gg_r1cs {
    int device = 0;
    int64_t expect_inputs = -1;  // gg_r1cs_set_inputs: required witness length (-1 = not set)
    int curve = GG_CURVE_BN254;  // scalar field: BN254 fr or BLS12-381 fr
    size_t nw = 0, ncons = 0, nterms = 0, ncoef = 0;
    uint32_t one_idx = 0xffffffffu;
    std::vector<uint32_t> level_off;  // host copy (launch sizes)
    std::vector<uint32_t> h_off, h_wire, h_level_cons;  // host copies for the strand analysis
    DevBuf off, wire, cidx, coef, coef_inv, level_cons, W, A, B, C, solved, fail, inputs, cnt;
    // strand schedule (built at the first solve, per witness length)
    long long strand_nin = -1;   // witness length it was built for
    bool strands = false;        // false: the level-by-level launches
    std::vector<uint32_t> sl_seg_off;  // segments of super-level l: [sl_seg_off[l], sl_seg_off[l+1])
    DevBuf unk, order, seg_start;
    size_t n_super = 0, n_seg = 0;
    hipStream_t st = nullptr;
    hipGraphExec_t graph = nullptr;
    std::mutex mu;
    ~gg_r1cs() {
        if (graph) (void)hipGraphExecDestroy(graph);
        if (st) (void)hipStreamDestroy(st);
    }
};

// Strand schedule for a witness of n_in values (wires 0..n_in are solved up
// front; strands.h): one launch per super-level, a thread per strand segment
// (the MiMC headline: 65,536 chains, one launch instead of 255).  Returns false
// (level launches instead) when the levels do not match the system; the level
// kernel then reports it.
static bool build_strands(gg_r1cs* r, size_t n_in) {
    StrandPlan plan;
    const bool ok = build_strand_plan(
        r->ncons, r->nw, (uint32_t)n_in + 1, r->level_off, r->h_level_cons,
        [&](uint32_t c, auto&& f) {
            for (uint32_t t = r->h_off[3 * c]; t < r->h_off[3 * c + 3]; t++) f(t, r->h_wire[t]);
        },
        [](uint32_t) { return false; }, plan);
    if (!ok) return false;
    auto up = [](DevBuf& b, const void* src, size_t bytes) {
        b.alloc(std::max<size_t>(bytes, 16));
        if (bytes) GG_HIP(hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice));
    };
    up(r->unk, plan.unk.data(), plan.unk.size() * 4);
    up(r->order, plan.order.data(), plan.order.size() * 4);
    up(r->seg_start, plan.seg_start.data(), plan.seg_start.size() * 4);
    r->sl_seg_off = std::move(plan.sl_seg_off);
    r->n_seg = plan.seg_start.size() - 1;
    r->n_super = r->sl_seg_off.size() - 1;
    return true;
}

// divByCoeff: host inverses of the coefficient table (0 for a zero coefficient)
// and the index of the coefficient 1
template <class FC>
static uint32_t invert_coeffs(const void* coeffs, size_t n, std::vector<uint8_t>& out) {
    using F = Fe<FC>;
    const F* cf = (const F*)coeffs;
    out.resize(n * 32);
    F* inv = (F*)out.data();
    uint32_t one_idx = 0xffffffffu;
    for (size_t i = 0; i < n; i++) {
        inv[i] = cf[i].is_zero() ? F::zero() : inverse(cf[i]);
        if (one_idx == 0xffffffffu && cf[i] == F::one()) one_idx = (uint32_t)i;
    }
    return one_idx;
}

extern "C" int gg_r1cs_create_ex(int curve, size_t n_wires, size_t n_constraints, const uint32_t* term_off,
                                 const uint32_t* term_wire, const uint32_t* term_coeff, const void* coeffs,
                                 size_t n_coeffs, const uint32_t* level_off, const uint32_t* level_cons,
                                 size_t n_levels, gg_r1cs_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out && term_off && coeffs && level_off, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "unknown curve");
    GG_CHECK(n_wires >= 1 && n_wires < 0xffffffffu && n_constraints < 0xffffffffu, GG_ERR_INVALID_ARG,
             "wire / constraint count out of range");
    GG_CHECK(n_coeffs >= 1 && n_coeffs < 0xffffffffu, GG_ERR_INVALID_ARG, "empty coefficient table");
    const size_t nterms = term_off[3 * n_constraints];
    GG_CHECK(term_off[0] == 0, GG_ERR_INVALID_ARG, "term_off[0] must be 0");
    for (size_t i = 0; i < 3 * n_constraints; i++)
        GG_CHECK(term_off[i] <= term_off[i + 1], GG_ERR_INVALID_ARG, "term_off not monotonic");
    GG_CHECK(nterms == 0 || (term_wire && term_coeff), GG_ERR_INVALID_ARG, "null term arrays");
    for (size_t t = 0; t < nterms; t++) {
        GG_CHECK(term_wire[t] < n_wires, GG_ERR_INVALID_ARG, "term wire id out of range");
        GG_CHECK(term_coeff[t] < n_coeffs, GG_ERR_INVALID_ARG, "term coefficient id out of range");
    }
    // r1cs.Levels: every constraint exactly once
    GG_CHECK(level_off[0] == 0 && level_off[n_levels] == n_constraints, GG_ERR_INVALID_ARG,
             "levels must cover every constraint once");
    GG_CHECK(n_constraints == 0 || level_cons, GG_ERR_INVALID_ARG, "null level_cons");
    std::vector<uint8_t> seen(n_constraints, 0);
    for (size_t l = 0; l < n_levels; l++) {
        GG_CHECK(level_off[l] <= level_off[l + 1], GG_ERR_INVALID_ARG, "level_off not monotonic");
        for (uint32_t i = level_off[l]; i < level_off[l + 1]; i++) {
            const uint32_t c = level_cons[i];
            GG_CHECK(c < n_constraints && !seen[c], GG_ERR_INVALID_ARG,
                     "levels must cover every constraint once");
            seen[c] = 1;
        }
    }
    std::vector<uint8_t> inv;
    const uint32_t one_idx = curve == GG_CURVE_BN254 ? invert_coeffs<FrCfg>(coeffs, n_coeffs, inv)
                                                     : invert_coeffs<FrBlsCfg>(coeffs, n_coeffs, inv);
    auto* r = new gg_r1cs();
    try {
        GG_HIP(hipGetDevice(&r->device));
        r->curve = curve;
        r->nw = n_wires;
        r->ncons = n_constraints;
        r->nterms = nterms;
        r->ncoef = n_coeffs;
        r->one_idx = one_idx;
        r->level_off.assign(level_off, level_off + n_levels + 1);
        r->h_off.assign(term_off, term_off + 3 * n_constraints + 1);
        r->h_wire.assign(term_wire, term_wire + nterms);
        r->h_level_cons.assign(level_cons, level_cons + n_constraints);
        auto up = [](DevBuf& b, const void* src, size_t bytes) {
            b.alloc(std::max<size_t>(bytes, 16));
            if (bytes) GG_HIP(hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice));
        };
        up(r->off, term_off, (3 * n_constraints + 1) * 4);
        up(r->wire, term_wire, nterms * 4);
        up(r->cidx, term_coeff, nterms * 4);
        up(r->coef, coeffs, n_coeffs * 32);
        up(r->coef_inv, inv.data(), n_coeffs * 32);
        up(r->level_cons, level_cons, n_constraints * 4);
        r->W.alloc(n_wires * 32);
        r->A.alloc(std::max<size_t>(n_constraints, 1) * 32);
        r->B.alloc(std::max<size_t>(n_constraints, 1) * 32);
        r->C.alloc(std::max<size_t>(n_constraints, 1) * 32);
        r->solved.alloc(n_wires);
        r->fail.alloc(16);
        r->cnt.alloc(16);
        GG_HIP(hipStreamCreateWithFlags(&r->st, hipStreamNonBlocking));
    } catch (...) {
        delete r;
        throw;
    }
    *out = r;
    GG_CAPI_END
}

extern "C" int gg_r1cs_create(size_t n_wires, size_t n_constraints, const uint32_t* term_off,
                              const uint32_t* term_wire, const uint32_t* term_coeff, const void* coeffs,
                              size_t n_coeffs, const uint32_t* level_off, const uint32_t* level_cons,
                              size_t n_levels, gg_r1cs_t* out) {
    return gg_r1cs_create_ex(GG_CURVE_BN254, n_wires, n_constraints, term_off, term_wire, term_coeff, coeffs,
                             n_coeffs, level_off, level_cons, n_levels, out);
}

extern "C" int gg_r1cs_release(gg_r1cs_t r) {
    delete r;
    return GG_OK;
}

extern "C" int gg_r1cs_info(gg_r1cs_t r, size_t* n_wires, size_t* n_constraints, size_t* n_levels) {
    GG_CAPI_BEGIN
    GG_CHECK(r, GG_ERR_INVALID_ARG, "null handle");
    if (n_wires) *n_wires = r->nw;
    if (n_constraints) *n_constraints = r->ncons;
    if (n_levels) *n_levels = r->level_off.size() - 1;
    GG_CAPI_END
}

// the per-level (or per-super-level strand) launches, enqueued on r->st
// (recorded once into a graph)
template <class FC>
static void enqueue_levels_t(gg_r1cs* r) {
    using Fr = Fe<FC>;
    R1csDev<FC> d{r->off.as<uint32_t>(), r->wire.as<uint32_t>(), r->cidx.as<uint32_t>(), r->coef.as<Fr>(),
              r->coef_inv.as<Fr>(), (uint32_t)r->ncoef, r->one_idx, (uint32_t)(r->strand_nin + 1), r->W.as<Fr>(),
              r->A.as<Fr>(), r->B.as<Fr>(),
              r->C.as<Fr>(), r->solved.as<uint8_t>(), r->fail.as<uint32_t>()};
    if (r->strands) {
        for (size_t l = 0; l < r->n_super; l++) {
            const uint32_t a = r->sl_seg_off[l], cnt = r->sl_seg_off[l + 1] - a;
            if (!cnt) continue;
            hipLaunchKernelGGL(k_solve_strands<FC>, dim3(grid_for(cnt, 256)), dim3(256), 0, r->st, d,
                               r->unk.as<uint32_t>(), r->order.as<uint32_t>(), r->seg_start.as<uint32_t>() + a,
                               cnt);
            GG_HIP(hipGetLastError());
        }
        return;
    }
    const uint32_t* lc = r->level_cons.as<uint32_t>();
    for (size_t l = 0; l + 1 < r->level_off.size(); l++) {
        const uint32_t a = r->level_off[l], cnt = r->level_off[l + 1] - a;
        if (!cnt) continue;
        hipLaunchKernelGGL(k_solve_level<FC>, dim3(grid_for(cnt, 256)), dim3(256), 0, r->st, d, lc + a, cnt);
        GG_HIP(hipGetLastError());
    }
}
static void enqueue_levels(gg_r1cs* r) {
    if (r->curve == GG_CURVE_BN254) enqueue_levels_t<FrCfg>(r);
    else enqueue_levels_t<FrBlsCfg>(r);
}

// newSolver's witness check (constraint/bn254/solver.go:71-76): a solve then
// requires exactly nb_public - 1 + nb_secret values (ONE_WIRE is not passed)
extern "C" int gg_r1cs_set_inputs(gg_r1cs_t r, size_t nb_public, size_t nb_secret) {
    GG_CAPI_BEGIN
    GG_CHECK(r && nb_public >= 1, GG_ERR_INVALID_ARG, "null handle or nb_public < 1 (ONE_WIRE)");
    GG_CHECK(nb_public + nb_secret <= r->nw, GG_ERR_INVALID_ARG, "more inputs than wires");
    std::lock_guard<std::mutex> lk(r->mu);
    r->expect_inputs = (int64_t)(nb_public - 1 + nb_secret);
    GG_CAPI_END
}

extern "C" int gg_r1cs_solve(gg_r1cs_t r, const void* witness, size_t n_witness, int witness_on_device,
                             void* w_out, void* a_out, void* b_out, void* c_out, int out_on_device,
                             int64_t* unsatisfied) {
    GG_CAPI_BEGIN
    GG_CHECK(r, GG_ERR_INVALID_ARG, "null handle");
    GG_CHECK(n_witness + 1 <= r->nw, GG_ERR_INVALID_ARG, "witness longer than the wire vector");
    if (r->expect_inputs >= 0 && (int64_t)n_witness != r->expect_inputs)
        throw Error(GG_ERR_INVALID_ARG, "invalid witness size, got " + std::to_string(n_witness) + ", expected " +
                                            std::to_string(r->expect_inputs));
    GG_CHECK(n_witness == 0 || witness, GG_ERR_INVALID_ARG, "null witness");
    std::lock_guard<std::mutex> lk(r->mu);
    GG_HIP(hipSetDevice(r->device));
    if (unsatisfied) *unsatisfied = -1;
    const void* in = witness;
    if (n_witness && !witness_on_device) {
        r->inputs.reserve(n_witness * 32);
        GG_HIP(hipMemcpyAsync(r->inputs.p, witness, n_witness * 32, hipMemcpyHostToDevice, r->st));
        in = r->inputs.p;
    }
    if (r->curve == GG_CURVE_BN254)
        hipLaunchKernelGGL(k_solver_init<FrCfg>, dim3(grid_for(r->nw, 256)), dim3(256), 0, r->st, r->W.as<Fr>(),
                           r->solved.as<uint8_t>(), r->nw, (const Fr*)in, n_witness, r->fail.as<uint32_t>());
    else
        hipLaunchKernelGGL(k_solver_init<FrBlsCfg>, dim3(grid_for(r->nw, 256)), dim3(256), 0, r->st,
                           r->W.as<FrBls>(), r->solved.as<uint8_t>(), r->nw, (const FrBls*)in, n_witness,
                           r->fail.as<uint32_t>());
    GG_HIP(hipGetLastError());
    // schedule: strands when the levels allow it (GG_SOLVER_LEVELS=1: level launches)
    if (r->strand_nin != (long long)n_witness) {
        const bool levels_only = getenv("GG_SOLVER_LEVELS") && atoi(getenv("GG_SOLVER_LEVELS"));
        r->strands = !levels_only && build_strands(r, n_witness);
        r->strand_nin = (long long)n_witness;
        if (r->graph) {
            (void)hipGraphExecDestroy(r->graph);
            r->graph = nullptr;
        }
    }
    // the launches: captured once into a graph, replayed afterwards
    if (!r->graph) {
        hipGraph_t g;
        GG_HIP(hipStreamBeginCapture(r->st, hipStreamCaptureModeThreadLocal));
        try {
            enqueue_levels(r);
        } catch (...) {
            (void)hipStreamEndCapture(r->st, &g);
            throw;
        }
        GG_HIP(hipStreamEndCapture(r->st, &g));
        hipError_t e = hipGraphInstantiate(&r->graph, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        GG_HIP(e);
    }
    GG_HIP(hipGraphLaunch(r->graph, r->st));
    GG_HIP(hipMemsetAsync(r->cnt.p, 0, 8, r->st));
    hipLaunchKernelGGL(k_count_unsolved, dim3(grid_for(r->nw, 256)), dim3(256), 0, r->st,
                       r->solved.as<uint8_t>(), r->nw, r->cnt.as<unsigned long long>());
    GG_HIP(hipGetLastError());
    uint32_t fail[2];
    unsigned long long unsolved = 0;
    GG_HIP(hipMemcpyAsync(fail, r->fail.p, 8, hipMemcpyDeviceToHost, r->st));
    GG_HIP(hipMemcpyAsync(&unsolved, r->cnt.p, 8, hipMemcpyDeviceToHost, r->st));
    GG_WAIT_STREAM(r->st);
    GG_CHECK(fail[1] == 0xffffffffu, GG_ERR_INVALID_ARG,
             "constraint #" + std::to_string(fail[1]) +
                 ": more than one unsolved wire at its level, or a zero coefficient on the unknown "
                 "(the levels do not match the system)");
    if (fail[0] != 0xffffffffu) {
        if (unsatisfied) *unsatisfied = fail[0];
        throw Error(GG_ERR_UNSATISFIED, "constraint #" + std::to_string(fail[0]) + " is not satisfied");
    }
    GG_CHECK(unsolved == 0, GG_ERR_UNSATISFIED,
             "solver didn't assign a value to all wires (" + std::to_string(unsolved) + " left)");
    const hipMemcpyKind k = out_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (w_out) GG_HIP(hipMemcpyAsync(w_out, r->W.p, r->nw * 32, k, r->st));
    if (a_out && r->ncons) GG_HIP(hipMemcpyAsync(a_out, r->A.p, r->ncons * 32, k, r->st));
    if (b_out && r->ncons) GG_HIP(hipMemcpyAsync(b_out, r->B.p, r->ncons * 32, k, r->st));
    if (c_out && r->ncons) GG_HIP(hipMemcpyAsync(c_out, r->C.p, r->ncons * 32, k, r->st));
    GG_WAIT_STREAM(r->st);
    GG_CAPI_END
}

// device pointers of the resident solution (valid until the next solve / release)
extern "C" int gg_r1cs_solution_dev(gg_r1cs_t r, void** w, void** a, void** b, void** c) {
    GG_CAPI_BEGIN
    GG_CHECK(r, GG_ERR_INVALID_ARG, "null handle");
    if (w) *w = r->W.p;
    if (a) *a = r->A.p;
    if (b) *b = r->B.p;
    if (c) *c = r->C.p;
    GG_CAPI_END
}

extern "C" int gg_r1cs_schedule(gg_r1cs_t r, int* strands, size_t* launches, size_t* segments) {
    GG_CAPI_BEGIN
    GG_CHECK(r, GG_ERR_INVALID_ARG, "null handle");
    std::lock_guard<std::mutex> lk(r->mu);
    size_t nl = 0;
    if (r->strands) {
        for (size_t l = 0; l < r->n_super; l++) nl += r->sl_seg_off[l + 1] > r->sl_seg_off[l];
    } else {
        for (size_t l = 0; l + 1 < r->level_off.size(); l++) nl += r->level_off[l + 1] > r->level_off[l];
    }
    if (strands) *strands = r->strands ? 1 : 0;
    if (launches) *launches = nl;
    if (segments) *segments = r->strands ? r->n_seg : 0;
    GG_CAPI_END
}
