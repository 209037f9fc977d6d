// Sparse-R1CS (PlonK) solver on the GPU: the SCS blueprints' Solve
// (constraint/blueprint_scs.go:53-151, BlueprintGenericSparseR1C and the
// Mul/Add forms it generalises) run level by level as in solver.go:418-533,
// then evaluateLROSmallDomain (constraint/bls12-381/system.go:221-264) builds
// the L, R, O columns the PlonK prover takes (gg_plonk_prove, inputs on
// device).  Hint-free systems; BLS12-381 fr (PlonK, BASELINE configs[4]) and
// BN254 fr.
//
// Constraint c: qL xa + qR xb + qO xc + qM xa xb + qC = 0 with
//   wires[3c + 0..2] = xa, xb, xc and qidx[5c + 0..4] = qL, qR, qO, qM, qC
//   (indices into the coefficient table), flags[c] & 1 = a BSB22 commitment
//   constraint (skipped when solving, blueprint_scs.go:56-60).
// The witness is public then secret at wires 0.. (no ONE_WIRE for SCS,
// solver.go:66-69).  A thread per constraint of a level:
//   xa unsolved: xa = -(qR xb + qO xc + qC) / (qM xb + qL)
//   xb unsolved: xb = -(qL xa + qO xc + qC) / (qM xa + qR)
//   xc unsolved: xc = -(qM xa xb + qL xa + qR xb + qC) / qO
//   all solved:  checkConstraint (blueprint_scs.go:129-151)
// A zero denominator is errDivideByZero.
#include "common.h"
#include "field.cuh"
#include "strands.h"
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>
#include <cstring>

namespace gg {

template <class C>
struct ScsDev {
    const uint32_t* wires;
    const uint32_t* qidx;
    const uint8_t* flags;
    const Fe<C>* coef;
    const Fe<C>* coef_inv;
    Fe<C>* W;
    uint8_t* solved;
    uint32_t* fail;  // [0] unsatisfied, [1] malformed (two unknowns), [2] division by zero
};

template <class C>
__device__ __forceinline__ Fe<C> ldfe(const Fe<C>* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    Fe<C> r;
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    return r;
}
template <class C>
__device__ __forceinline__ void stfe(Fe<C>* p, const Fe<C>& r) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(r.v[0], r.v[1], r.v[2], r.v[3]);
    q[1] = make_uint4(r.v[4], r.v[5], r.v[6], r.v[7]);
}

template <class C>
__global__ void __launch_bounds__(256) k_scs_level(ScsDev<C> d, const uint32_t* cons, uint32_t count) {
    using F = Fe<C>;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t c = cons[i];
    if (d.flags && (d.flags[c] & 1u)) return;
    const uint32_t xa = d.wires[3 * c], xb = d.wires[3 * c + 1], xc = d.wires[3 * c + 2];
    const bool sa = d.solved[xa], sb = d.solved[xb], sc = d.solved[xc];
    if ((int)!sa + (int)!sb + (int)!sc > 1 || (!sa && xa == xb)) {
        atomicMin(d.fail + 1, c);
        return;
    }
    const uint32_t* q = d.qidx + 5 * c;
    const F qL = ldfe(d.coef + q[0]), qR = ldfe(d.coef + q[1]), qM = ldfe(d.coef + q[3]),
            qC = ldfe(d.coef + q[4]);
    const F a = sa ? ldfe(d.W + xa) : F::zero(), b = sb ? ldfe(d.W + xb) : F::zero(),
            o = sc ? ldfe(d.W + xc) : F::zero();
    if (!sa || !sb) {
        const F qO = ldfe(d.coef + q[2]);
        const F den = !sa ? qM * b + qL : qM * a + qR;
        if (den.is_zero()) {
            atomicMin(d.fail + 2, c);
            return;
        }
        const F num = (!sa ? qR * b : qL * a) + qO * o + qC;
        const F v = -(num * inverse(den));
        const uint32_t w = !sa ? xa : xb;
        stfe(d.W + w, v);
        d.solved[w] = 1;
    } else if (!sc) {
        const F qOinv = ldfe(d.coef_inv + q[2]);
        if (qOinv.is_zero()) {
            atomicMin(d.fail + 2, c);
            return;
        }
        const F t = (qM * a) * b + qL * a + qR * b + qC;
        stfe(d.W + xc, -(t * qOinv));
        d.solved[xc] = 1;
    } else {
        const F qO = ldfe(d.coef + q[2]);
        const F t = (qM * a) * b + qL * a + qR * b + qO * o + qC;
        if (!t.is_zero()) atomicMin(d.fail, c);
    }
}

// W read around the (write-through, non-coherent) L1: a strand reads values
// it stored earlier in the same launch
template <class C>
__device__ __forceinline__ Fe<C> ldfe_l2(const Fe<C>* p) {
    const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
    Fe<C> r;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t x = __hip_atomic_load(q + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.v[2 * k] = (uint32_t)x;
        r.v[2 * k + 1] = (uint32_t)(x >> 32);
    }
    return r;
}

// Strand schedule (strands.h): thread s walks segment s of this launch --
// consecutive constraints of one dependency chain -- in order.  The unknown's
// position is fixed per constraint (unk[c] = 3 c + {0, 1, 2}: xa, xb, xc;
// ~0: none, the constraint is checked), so no solved flags are read; the
// same formulas as k_scs_level.  The chain's last RC outputs stay in registers.
template <class C>
__global__ void __launch_bounds__(256) k_scs_strands(ScsDev<C> d, const uint32_t* unk, const uint32_t* order,
                                                     const uint32_t* seg_start, uint32_t nseg, uint32_t nin) {
    using F = Fe<C>;
    const uint32_t sg = blockIdx.x * blockDim.x + threadIdx.x;
    if (sg >= nseg) return;
    constexpr int RC = 4;
    uint32_t cw[RC];
    F cv[RC];
#pragma unroll
    for (int k = 0; k < RC; k++) cw[k] = 0xffffffffu;
    int cpos = 0;
    auto value = [&](uint32_t w) {
        F x;
        int hit = -1;
#pragma unroll
        for (int q = 0; q < RC; q++)
            if (cw[q] == w) hit = q;
        if (hit >= 0) {
#pragma unroll
            for (int q = 0; q < RC; q++)
                if (q == hit) x = cv[q];
        } else {
            x = w < nin ? ldfe(d.W + w) : ldfe_l2(d.W + w);
        }
        return x;
    };
    for (uint32_t i = seg_start[sg], e = seg_start[sg + 1]; i < e; i++) {
        const uint32_t c = order[i], u = unk[c];
        const int pos = u == 0xffffffffu ? 3 : (int)(u - 3 * c);
        const uint32_t xa = d.wires[3 * c], xb = d.wires[3 * c + 1], xc = d.wires[3 * c + 2];
        const uint32_t* q = d.qidx + 5 * c;
        const F qL = ldfe(d.coef + q[0]), qR = ldfe(d.coef + q[1]), qM = ldfe(d.coef + q[3]),
                qC = ldfe(d.coef + q[4]);
        const F a = pos != 0 ? value(xa) : F::zero(), b = pos != 1 ? value(xb) : F::zero(),
                o = pos != 2 ? value(xc) : F::zero();
        uint32_t w = 0xffffffffu;
        F v;
        if (pos <= 1) {
            const F qO = ldfe(d.coef + q[2]);
            const F den = pos == 0 ? qM * b + qL : qM * a + qR;
            if (den.is_zero()) {
                atomicMin(d.fail + 2, c);
                return;  // the solve fails: the rest of this strand is never read
            }
            const F num = (pos == 0 ? qR * b : qL * a) + qO * o + qC;
            v = -(num * inverse(den));
            w = pos == 0 ? xa : xb;
        } else if (pos == 2) {
            const F qOinv = ldfe(d.coef_inv + q[2]);
            if (qOinv.is_zero()) {
                atomicMin(d.fail + 2, c);
                return;
            }
            const F t = (qM * a) * b + qL * a + qR * b + qC;
            v = -(t * qOinv);
            w = xc;
        } else {
            const F qO = ldfe(d.coef + q[2]);
            const F t = (qM * a) * b + qL * a + qR * b + qO * o + qC;
            if (!t.is_zero()) atomicMin(d.fail, c);
        }
        if (w != 0xffffffffu) {
            stfe(d.W + w, v);
            d.solved[w] = 1;
#pragma unroll
            for (int k = 0; k < RC; k++)
                if (k == cpos) {
                    cw[k] = w;
                    cv[k] = v;
                }
            cpos = (cpos + 1) & (RC - 1);
        }
    }
}

template <class C>
__global__ void k_scs_init(Fe<C>* W, uint8_t* solved, size_t nw, const Fe<C>* in, size_t n_in, uint32_t* fail) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) fail[0] = fail[1] = fail[2] = 0xffffffffu;
    if (i >= nw) return;
    stfe(W + i, i < n_in ? ldfe(in + i) : Fe<C>::zero());
    solved[i] = i < n_in ? 1 : 0;
}

// evaluateLROSmallDomain (system.go:221-264): public placeholder rows, the
// constraints, padding to the power of two -- unused slots carry solution[0]
template <class C>
__global__ void k_scs_lro(const Fe<C>* W, const uint32_t* wires, size_t nb_public, size_t ncons, size_t s,
                          Fe<C>* L, Fe<C>* R, Fe<C>* O) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s) return;
    const Fe<C> s0 = ldfe(W);
    if (i < nb_public) {
        stfe(L + i, ldfe(W + i));
        stfe(R + i, s0);
        stfe(O + i, s0);
    } else if (i < nb_public + ncons) {
        const size_t j = i - nb_public;
        stfe(L + i, ldfe(W + wires[3 * j]));
        stfe(R + i, ldfe(W + wires[3 * j + 1]));
        stfe(O + i, ldfe(W + wires[3 * j + 2]));
    } else {
        stfe(L + i, s0);
        stfe(R + i, s0);
        stfe(O + i, s0);
    }
}

__global__ void k_scs_count_unsolved(const uint8_t* solved, size_t nw, unsigned long long* cnt) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool u = i < nw && !solved[i];
    const unsigned long long b = __ballot(u);
    if (u && (threadIdx.x & 63) == (uint32_t)(__ffsll(b) - 1)) atomicAdd(cnt, (unsigned long long)__popcll(b));
}

}  // namespace gg

using namespace gg;

struct gg_scs {
    int device = 0, curve = 0;
    int64_t expect_inputs = -1;  // gg_scs_set_inputs: required witness length (-1 = not set)
    size_t nw = 0, ncons = 0, nb_public = 0, dom = 0, ncoef = 0;
    std::vector<uint32_t> level_off;
    std::vector<uint32_t> h_wires, h_level_cons;  // host copies for the strand analysis
    std::vector<uint8_t> h_flags;
    DevBuf wires, qidx, flags, coef, coef_inv, level_cons, W, L, R, O, solved, fail, inputs, cnt;
    bool has_flags = false;
    // strand schedule (built at the first solve, per witness length; strands.h)
    long long strand_nin = -1;
    bool strands = false;  // false: the level-by-level launches
    std::vector<uint32_t> sl_seg_off;
    DevBuf unk, order, seg_start;
    size_t n_super = 0, n_seg = 0;
    hipStream_t st = nullptr;
    hipGraphExec_t graph = nullptr;
    std::mutex mu;
    ~gg_scs() {
        if (graph) (void)hipGraphExecDestroy(graph);
        if (st) (void)hipStreamDestroy(st);
    }
};

namespace {
template <class C>
void invert_table(const void* coeffs, size_t n, std::vector<Fe<C>>& inv) {
    const Fe<C>* cf = (const Fe<C>*)coeffs;
    inv.resize(n);
    for (size_t i = 0; i < n; i++) inv[i] = cf[i].is_zero() ? Fe<C>::zero() : inverse(cf[i]);
}

template <class C>
void enqueue_scs_levels(gg_scs* h) {
    ScsDev<C> d{h->wires.as<uint32_t>(), h->qidx.as<uint32_t>(), h->has_flags ? h->flags.as<uint8_t>() : nullptr,
                h->coef.as<Fe<C>>(), h->coef_inv.as<Fe<C>>(), h->W.as<Fe<C>>(), h->solved.as<uint8_t>(),
                h->fail.as<uint32_t>()};
    if (h->strands) {
        for (size_t l = 0; l < h->n_super; l++) {
            const uint32_t a = h->sl_seg_off[l], cnt = h->sl_seg_off[l + 1] - a;
            if (!cnt) continue;
            hipLaunchKernelGGL(k_scs_strands<C>, dim3(grid_for(cnt, 256)), dim3(256), 0, h->st, d,
                               h->unk.as<uint32_t>(), h->order.as<uint32_t>(), h->seg_start.as<uint32_t>() + a, cnt,
                               (uint32_t)h->strand_nin);
            GG_HIP(hipGetLastError());
        }
        return;
    }
    const uint32_t* lc = h->level_cons.as<uint32_t>();
    for (size_t l = 0; l + 1 < h->level_off.size(); l++) {
        const uint32_t a = h->level_off[l], cnt = h->level_off[l + 1] - a;
        if (!cnt) continue;
        hipLaunchKernelGGL(k_scs_level<C>, dim3(grid_for(cnt, 256)), dim3(256), 0, h->st, d, lc + a, cnt);
        GG_HIP(hipGetLastError());
    }
}

// Strand schedule for a witness of n_in values (wires 0..n_in-1 solved up
// front, no ONE_WIRE); commitment rows solve nothing and are left out
bool build_scs_strands(gg_scs* h, size_t n_in) {
    StrandPlan plan;
    const bool ok = build_strand_plan(
        h->ncons, h->nw, (uint32_t)n_in, h->level_off, h->h_level_cons,
        [&](uint32_t c, auto&& f) {
            for (uint32_t k = 0; k < 3; k++) f(3 * c + k, h->h_wires[3 * c + k]);
        },
        [&](uint32_t c) { return h->has_flags && (h->h_flags[c] & 1u); }, plan);
    if (!ok) return false;
    auto up = [](DevBuf& b, const void* src, size_t bytes) {
        b.alloc(std::max<size_t>(bytes, 16));
        if (bytes) GG_HIP(hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice));
    };
    up(h->unk, plan.unk.data(), plan.unk.size() * 4);
    up(h->order, plan.order.data(), plan.order.size() * 4);
    up(h->seg_start, plan.seg_start.data(), plan.seg_start.size() * 4);
    h->sl_seg_off = std::move(plan.sl_seg_off);
    h->n_seg = plan.seg_start.size() - 1;
    h->n_super = h->sl_seg_off.size() - 1;
    return true;
}

template <class C>
void scs_solve_impl(gg_scs* h, const void* in, size_t n_in) {
    hipLaunchKernelGGL(k_scs_init<C>, dim3(grid_for(h->nw, 256)), dim3(256), 0, h->st, h->W.as<Fe<C>>(),
                       h->solved.as<uint8_t>(), h->nw, (const Fe<C>*)in, n_in, h->fail.as<uint32_t>());
    GG_HIP(hipGetLastError());
    // schedule: strands when the levels allow it (GG_SOLVER_LEVELS=1: level launches)
    if (h->strand_nin != (long long)n_in) {
        const bool levels_only = getenv("GG_SOLVER_LEVELS") && atoi(getenv("GG_SOLVER_LEVELS"));
        h->strands = !levels_only && build_scs_strands(h, n_in);
        h->strand_nin = (long long)n_in;
        if (h->graph) {
            (void)hipGraphExecDestroy(h->graph);
            h->graph = nullptr;
        }
    }
    if (!h->graph) {
        hipGraph_t g;
        GG_HIP(hipStreamBeginCapture(h->st, hipStreamCaptureModeThreadLocal));
        try {
            enqueue_scs_levels<C>(h);
        } catch (...) {
            (void)hipStreamEndCapture(h->st, &g);
            throw;
        }
        GG_HIP(hipStreamEndCapture(h->st, &g));
        hipError_t e = hipGraphInstantiate(&h->graph, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        GG_HIP(e);
    }
    GG_HIP(hipGraphLaunch(h->graph, h->st));
    hipLaunchKernelGGL(k_scs_lro<C>, dim3(grid_for(h->dom, 256)), dim3(256), 0, h->st, h->W.as<Fe<C>>(),
                       h->wires.as<uint32_t>(), h->nb_public, h->ncons, h->dom, h->L.as<Fe<C>>(),
                       h->R.as<Fe<C>>(), h->O.as<Fe<C>>());
    GG_HIP(hipGetLastError());
}
}  // namespace

extern "C" int gg_scs_create(int curve, size_t n_wires, size_t n_constraints, size_t nb_public,
                             const uint32_t* wires, const uint32_t* qidx, const uint8_t* flags, const void* coeffs,
                             size_t n_coeffs, const uint32_t* level_off, const uint32_t* level_cons,
                             size_t n_levels, gg_scs_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out && coeffs && level_off, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "unknown curve");
    GG_CHECK(n_wires >= 1 && n_wires < 0xffffffffu && n_constraints < 0xffffffffu && nb_public <= n_wires,
             GG_ERR_INVALID_ARG, "wire / constraint count out of range");
    GG_CHECK(n_coeffs >= 1 && n_coeffs < 0xffffffffu, GG_ERR_INVALID_ARG, "empty coefficient table");
    GG_CHECK(n_constraints == 0 || (wires && qidx && level_cons), GG_ERR_INVALID_ARG, "null constraint arrays");
    for (size_t t = 0; t < 3 * n_constraints; t++)
        GG_CHECK(wires[t] < n_wires, GG_ERR_INVALID_ARG, "wire id out of range");
    for (size_t t = 0; t < 5 * n_constraints; t++)
        GG_CHECK(qidx[t] < n_coeffs, GG_ERR_INVALID_ARG, "coefficient id out of range");
    GG_CHECK(level_off[0] == 0 && level_off[n_levels] == n_constraints, GG_ERR_INVALID_ARG,
             "levels must cover every constraint once");
    std::vector<uint8_t> seen(n_constraints, 0);
    for (size_t l = 0; l < n_levels; l++) {
        GG_CHECK(level_off[l] <= level_off[l + 1], GG_ERR_INVALID_ARG, "level_off not monotonic");
        for (uint32_t i = level_off[l]; i < level_off[l + 1]; i++) {
            const uint32_t c = level_cons[i];
            GG_CHECK(c < n_constraints && !seen[c], GG_ERR_INVALID_ARG, "levels must cover every constraint once");
            seen[c] = 1;
        }
    }
    size_t dom = 1;
    while (dom < n_constraints + nb_public) dom <<= 1;  // ecc.NextPowerOfTwo (system.go:224-225)
    std::vector<uint8_t> inv_bytes(n_coeffs * 32);
    if (curve == GG_CURVE_BN254) {
        std::vector<Fr> inv;
        invert_table<FrCfg>(coeffs, n_coeffs, inv);
        memcpy(inv_bytes.data(), inv.data(), n_coeffs * 32);
    } else {
        std::vector<FrBls> inv;
        invert_table<FrBlsCfg>(coeffs, n_coeffs, inv);
        memcpy(inv_bytes.data(), inv.data(), n_coeffs * 32);
    }
    auto* h = new gg_scs();
    try {
        GG_HIP(hipGetDevice(&h->device));
        h->curve = curve;
        h->nw = n_wires;
        h->ncons = n_constraints;
        h->nb_public = nb_public;
        h->dom = dom;
        h->ncoef = n_coeffs;
        h->level_off.assign(level_off, level_off + n_levels + 1);
        h->h_wires.assign(wires, wires + 3 * n_constraints);
        h->h_level_cons.assign(level_cons, level_cons + n_constraints);
        if (flags) h->h_flags.assign(flags, flags + n_constraints);
        auto up = [](DevBuf& b, const void* src, size_t bytes) {
            b.alloc(std::max<size_t>(bytes, 16));
            if (bytes) GG_HIP(hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice));
        };
        up(h->wires, wires, 3 * n_constraints * 4);
        up(h->qidx, qidx, 5 * n_constraints * 4);
        h->has_flags = flags != nullptr;
        if (flags) up(h->flags, flags, n_constraints);
        up(h->coef, coeffs, n_coeffs * 32);
        up(h->coef_inv, inv_bytes.data(), n_coeffs * 32);
        up(h->level_cons, level_cons, n_constraints * 4);
        h->W.alloc(n_wires * 32);
        h->L.alloc(dom * 32);
        h->R.alloc(dom * 32);
        h->O.alloc(dom * 32);
        h->solved.alloc(n_wires);
        h->fail.alloc(16);
        h->cnt.alloc(16);
        GG_HIP(hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking));
    } catch (...) {
        delete h;
        throw;
    }
    *out = h;
    GG_CAPI_END
}

extern "C" int gg_scs_release(gg_scs_t h) {
    delete h;
    return GG_OK;
}

extern "C" int gg_scs_info(gg_scs_t h, size_t* n_wires, size_t* n_constraints, size_t* domain) {
    GG_CAPI_BEGIN
    GG_CHECK(h, GG_ERR_INVALID_ARG, "null handle");
    if (n_wires) *n_wires = h->nw;
    if (n_constraints) *n_constraints = h->ncons;
    if (domain) *domain = h->dom;
    GG_CAPI_END
}

// newSolver's witness check (constraint/bls12-381/solver.go:71-76) for a
// sparse R1CS: a solve then requires exactly nb_public + nb_secret values
extern "C" int gg_scs_set_inputs(gg_scs_t h, size_t nb_public, size_t nb_secret) {
    GG_CAPI_BEGIN
    GG_CHECK(h && nb_public + nb_secret >= 1 && nb_public + nb_secret <= h->nw, GG_ERR_INVALID_ARG,
             "null handle or input count outside [1, wires]");
    std::lock_guard<std::mutex> lk(h->mu);
    h->expect_inputs = (int64_t)(nb_public + nb_secret);
    GG_CAPI_END
}

extern "C" int gg_scs_solve(gg_scs_t h, const void* witness, size_t n_witness, int witness_on_device, void* w_out,
                            void* l_out, void* r_out, void* o_out, int out_on_device, int64_t* failed) {
    GG_CAPI_BEGIN
    GG_CHECK(h, GG_ERR_INVALID_ARG, "null handle");
    GG_CHECK(n_witness >= 1 && n_witness <= h->nw, GG_ERR_INVALID_ARG,
             "witness must hold at least one value (solution[0] pads L, R, O) and fit the wires");
    GG_CHECK(witness, GG_ERR_INVALID_ARG, "null witness");
    if (h->expect_inputs >= 0 && (int64_t)n_witness != h->expect_inputs)
        throw Error(GG_ERR_INVALID_ARG, "invalid witness size, got " + std::to_string(n_witness) + ", expected " +
                                            std::to_string(h->expect_inputs));
    std::lock_guard<std::mutex> lk(h->mu);
    GG_HIP(hipSetDevice(h->device));
    if (failed) *failed = -1;
    const void* in = witness;
    if (!witness_on_device) {
        h->inputs.reserve(n_witness * 32);
        GG_HIP(hipMemcpyAsync(h->inputs.p, witness, n_witness * 32, hipMemcpyHostToDevice, h->st));
        in = h->inputs.p;
    }
    if (h->curve == GG_CURVE_BN254) scs_solve_impl<FrCfg>(h, in, n_witness);
    else scs_solve_impl<FrBlsCfg>(h, in, n_witness);
    GG_HIP(hipMemsetAsync(h->cnt.p, 0, 8, h->st));
    hipLaunchKernelGGL(k_scs_count_unsolved, dim3(grid_for(h->nw, 256)), dim3(256), 0, h->st,
                       h->solved.as<uint8_t>(), h->nw, h->cnt.as<unsigned long long>());
    GG_HIP(hipGetLastError());
    uint32_t fail[3];
    unsigned long long unsolved = 0;
    GG_HIP(hipMemcpyAsync(fail, h->fail.p, 12, hipMemcpyDeviceToHost, h->st));
    GG_HIP(hipMemcpyAsync(&unsolved, h->cnt.p, 8, hipMemcpyDeviceToHost, h->st));
    GG_WAIT_STREAM(h->st);
    GG_CHECK(fail[1] == 0xffffffffu, GG_ERR_INVALID_ARG,
             "constraint #" + std::to_string(fail[1]) +
                 ": more than one unsolved wire at its level (the levels do not match the system)");
    const uint32_t bad = std::min(fail[0], fail[2]);
    if (bad != 0xffffffffu) {
        if (failed) *failed = bad;
        throw Error(GG_ERR_UNSATISFIED, "constraint #" + std::to_string(bad) +
                                            (bad == fail[2] ? ": division by zero" : " is not satisfied"));
    }
    GG_CHECK(unsolved == 0, GG_ERR_UNSATISFIED,
             "solver didn't assign a value to all wires (" + std::to_string(unsolved) + " left)");
    const hipMemcpyKind k = out_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (w_out) GG_HIP(hipMemcpyAsync(w_out, h->W.p, h->nw * 32, k, h->st));
    if (l_out) GG_HIP(hipMemcpyAsync(l_out, h->L.p, h->dom * 32, k, h->st));
    if (r_out) GG_HIP(hipMemcpyAsync(r_out, h->R.p, h->dom * 32, k, h->st));
    if (o_out) GG_HIP(hipMemcpyAsync(o_out, h->O.p, h->dom * 32, k, h->st));
    GG_WAIT_STREAM(h->st);
    GG_CAPI_END
}

extern "C" int gg_scs_solution_dev(gg_scs_t h, void** w, void** l, void** r, void** o) {
    GG_CAPI_BEGIN
    GG_CHECK(h, GG_ERR_INVALID_ARG, "null handle");
    if (w) *w = h->W.p;
    if (l) *l = h->L.p;
    if (r) *r = h->R.p;
    if (o) *o = h->O.p;
    GG_CAPI_END
}

extern "C" int gg_scs_schedule(gg_scs_t h, int* strands, size_t* launches, size_t* segments) {
    GG_CAPI_BEGIN
    GG_CHECK(h, GG_ERR_INVALID_ARG, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    size_t nl = 0;
    if (h->strands) {
        for (size_t l = 0; l < h->n_super; l++) nl += h->sl_seg_off[l + 1] > h->sl_seg_off[l];
    } else {
        for (size_t l = 0; l + 1 < h->level_off.size(); l++) nl += h->level_off[l + 1] > h->level_off[l];
    }
    if (strands) *strands = h->strands ? 1 : 0;
    if (launches) *launches = nl;
    if (segments) *segments = h->strands ? h->n_seg : 0;
    GG_CAPI_END
}
