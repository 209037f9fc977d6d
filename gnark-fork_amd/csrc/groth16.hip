// Groth16 BN254 prover on one MI355X: the device section of gnark's
// icicle_bn254.Prove (icicle.go:133-422) / groth16_bn254.Prove (prove.go:127-320).
//
//   stream 1: computeH (6 fused NTTs) -> Z-MSM over h
//   streams 2, 3, 4, 0: A-MSM, B1-MSM, K-MSM, G2-MSM, concurrently (wire
//                       scalars gathered through per-base index maps)
//   host pool: r*delta, s*delta, kr*delta, s*delta2 while the GPU works;
//              s*Ar, r*Bs1 after the MSMs
// Combination formulas are prove.go:206-299 verbatim.
#include "common.h"
#include "curve.cuh"
#include "stage.h"
#include <chrono>
#include <future>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>
#include <cstdlib>
#include <cstring>

struct gg_domain;
struct gg_msm_base;

namespace gg {
struct MsmSort;
struct MsmScratch;
struct MsmWork;
void compute_h_device(gg_domain* d, Fr* A, Fr* B, Fr* C, Fr* H, hipStream_t st);
void msm_device(gg_msm_base* b, const Fr* scalars_dev, void* out_jac, hipStream_t st);
size_t msm_scalars_needed(gg_msm_base* b);
gg_msm_base* msm_base_create_internal(int group, const void* host_points, size_t n,
                                      const uint32_t* sidx, int window_bits, bool keep_inf, int groups);
int choose_groups_multi(const double* bytes, const int* W, int k, double extra);
bool msm_same_shape(const gg_msm_base* a, const gg_msm_base* b);
MsmSort* msm_own_sort(gg_msm_base* b);
void msm_prepare_dev(gg_msm_base* b, MsmSort* s, const Fr* scalars_dev, hipStream_t st, int slog = 0,
                     uint32_t sres = 0);
void msm_finish_dev(gg_msm_base* b, MsmSort* s, void* out_jac, hipStream_t st, MsmScratch* scr = nullptr);
MsmWork* msm_work_new();
void msm_work_delete(MsmWork* w);
MsmSort* msm_work_sort(MsmWork* w);
void msm_prepare_derived_dev(gg_msm_base* a, MsmSort* sa, gg_msm_base* b, MsmSort* sb, const uint32_t* bmap,
                             hipStream_t st);
bool msm_derivable(const gg_msm_base* a, const gg_msm_base* b);
void msm_build_bmap(const gg_msm_base* a, const gg_msm_base* b, DevBuf& bmap);
MsmScratch* msm_work_scratch(MsmWork* w);
int msm_base_window(const gg_msm_base* b);
int choose_c(size_t n, size_t point_bytes, int total_bits);
void hshard_run(gg_hshard* hs, const Fr* a, const Fr* b, const Fr* c, size_t len, bool compact, Fr* send,
                Fr* recv, gg_exchange_fn xchg, void* ctx, hipStream_t st);
size_t hshard_m(const gg_hshard* hs, int* rank, int* world, int* log_n);
Fr* hshard_h(gg_hshard* hs);
int hshard_curve(const gg_hshard* hs);
}  // namespace gg

// distributed computeH of a shard (gg_groth16_prove_partial_dist)
struct DistH {
    gg_hshard* hs;
    gg_exchange_fn xchg;
    void* ctx;
    gg::Fr *send, *recv;
};

using namespace gg;

// curve traits of the prover: BN254 (backend/groth16/bn254) and BLS12-381
// (backend/groth16/bls12-381; prove.go there is the same code over another curve)
struct CurveBn254 {
    using FrT = Fr;
    using G1F = Fp;
    using G2F = Fp2;
    static constexpr int curve = GG_CURVE_BN254, g1 = GG_G1, g2 = GG_G2, total_bits = 255;
};
struct CurveBls12381 {
    using FrT = FrBls;
    using G1F = FpBls;
    using G2F = Fp2Bls;
    static constexpr int curve = GG_CURVE_BLS12_381, g1 = GG_BLS12_381_G1, g2 = GG_BLS12_381_G2, total_bits = 256;
};
// byte sizes of the curve's affine / Jacobian points
struct PointSizes {
    size_t g1a, g2a, g1j, g2j;
};
static PointSizes point_sizes(int curve) {
    if (curve == GG_CURVE_BN254) return {64, 128, 96, 192};
    return {96, 192, 144, 288};
}

// The wire-indexed tables of a key (or of a wire shard): A and K (infinity
// holes kept, one sort of the wires), B and G2 B (B-filtered, one sort).  A
// bucket-stripe multi-GPU key keeps ONE whole copy per device, shared by the
// stripe shards placed there.
struct WireBases {
    gg_msm_base_t A = nullptr, B = nullptr, K = nullptr, B2 = nullptr;
    bool share_AK = false, share_B = false;
    // B1 / G2 on A's window: their sorted entries filtered from the A / K sort
    // (msm_prepare_derived) instead of a sort of their own; bmap: wire -> B point
    bool derive_B = false;
    DevBuf bmap;
    int groups = 1;
    WireBases() = default;
    WireBases(const WireBases&) = delete;
    WireBases& operator=(const WireBases&) = delete;
    ~WireBases() {
        for (gg_msm_base_t b : {A, B, K, B2})
            if (b) gg_msm_base_release(b);
    }
};

// MSM sort + scratch of one prove over shared tables (a stripe shard's own)
struct WorkSet {
    MsmWork *A = nullptr, *B = nullptr, *K = nullptr, *B2 = nullptr;
    WorkSet() {
        A = msm_work_new();
        B = msm_work_new();
        K = msm_work_new();
        B2 = msm_work_new();
    }
    WorkSet(const WorkSet&) = delete;
    WorkSet& operator=(const WorkSet&) = delete;
    ~WorkSet() {
        for (MsmWork* w : {A, B, K, B2})
            if (w) msm_work_delete(w);
    }
};

struct gg_groth16_pk {
    int curve = GG_CURVE_BN254;
    int log_n = 0;
    size_t n = 0;
    gg_domain_t dom = nullptr;
    // A, B, K, B2 alias wb's tables (shared between the stripe shards of one device)
    std::shared_ptr<WireBases> wb;
    gg_msm_base_t A = nullptr, B = nullptr, K = nullptr, Z = nullptr, B2 = nullptr;
    // bucket stripe of a multi-GPU key: the A, B1, K and G2 MSMs of this shard
    // take the buckets b = spart mod 2^slog of the whole tables (slog = 0: all)
    int slog = 0;
    uint32_t spart = 0;
    std::unique_ptr<WorkSet> work;  // stripe shards: their own sorts / scratch over the shared tables
    // pk.G1.{Alpha, Beta, Delta}, pk.G2.{Beta, Delta} in the curve's affine layout
    uint8_t alpha[96], beta[96], delta[96], beta2[192], delta2[192];
    size_t n_wires = 0, nb_public = 0;
    // shard of a multi-GPU key: wires [wire_lo, wire_hi), Z positions [z_lo, z_lo + |Z|)
    size_t wire_lo = 0, wire_hi = 0, z_lo = 0, nZ = 0;
    // A and K are wire-indexed tables (infinity holes kept) sharing one sort of
    // the wires; B1 and G2 share the sort of the B-filtered wires (same index map
    // and window).  Falls back to separate sorts if the shapes ever differ.
    bool share_AK = false, share_B = false;
    DevBuf wires, sa, sb, sc;
    hipStream_t s0 = nullptr, s1 = nullptr, s2 = nullptr, s3 = nullptr, s4 = nullptr;
    TaskQueue tq[5];  // the task slots behind s0..s4 (common.h: own stream + borrowed dedicated queue)
    hipStream_t* const* active() {
        act[0] = &s0, act[1] = &s1, act[2] = &s2, act[3] = &s3, act[4] = &s4;
        return act;
    }
    hipStream_t* act[5] = {};
    hipStream_t hprio = nullptr;  // GG_G16_H_PRIORITY=1: s1 on a stream of the greatest priority
    std::unique_ptr<Stager> stager;  // host inputs -> HBM (created on first host-input prove)
    int device = 0;
    std::mutex mu;
    ~gg_groth16_pk() {
        stager.reset();
        work.reset();
        wb.reset();
        if (Z) gg_msm_base_release(Z);
        if (dom) gg_domain_release(dom);
        task_streams_release(tq, 5, device);
        if (hprio) (void)hipStreamDestroy(hprio);
    }
};

static thread_local double g_timings[9];
// [0] = host staging of A, B, C (inside the H task, overlapped with the MSMs);
// [1], [2] = steady-clock ms at entry to / return from the last prove call
static thread_local double g_ext[3];

static void ck(int rc) {
    if (rc != GG_OK) throw Error(rc, gg_last_error());
}

// The A, K, B and G2 B tables of wires [lo, hi) (pk order, setup.go:259-275):
// g1_A = the non-infinity A points of those wires, likewise g1_B / g2_B; g1_K =
// the K points whose wires lie in the range (k_wire_index gives their absolute
// wire ids; NULL = the default nb_public + j numbering of the full key).  One
// precompute-group count for every table (bases that share a sort need equal
// shapes), the smallest whose tables fit HBM beside the proof's scratch and
// the nZ Z points that will sit beside them.
static std::shared_ptr<WireBases> wire_bases_build(int curve, int log_n, const void* g1_A, size_t nA,
                                                   const void* g1_B, size_t nB, const void* g1_K, size_t nK,
                                                   const void* g2_B, const uint8_t* inf_A, const uint8_t* inf_B,
                                                   size_t n_wires, size_t nb_public, const uint32_t* k_wire_index,
                                                   size_t lo, size_t hi, size_t nZ) {
    GG_CHECK(inf_A && inf_B, GG_ERR_INVALID_ARG, "null infinity masks");
    GG_CHECK(nb_public <= n_wires, GG_ERR_INVALID_ARG, "nb_public > n_wires");
    GG_CHECK(lo <= hi && hi <= n_wires, GG_ERR_INVALID_ARG, "bad wire shard range");
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "bad curve");
    const PointSizes ps = point_sizes(curve);
    const int g1 = curve == GG_CURVE_BN254 ? GG_G1 : GG_BLS12_381_G1;
    const int g2 = curve == GG_CURVE_BN254 ? GG_G2 : GG_BLS12_381_G2;
    const int tbits = curve == GG_CURVE_BN254 ? 255 : 256;
    // wire index maps (prove.go:151-175: drop wires whose A/B point is infinity),
    // relative to the shard's first wire
    std::vector<uint32_t> ia, ib, ik;
    for (size_t i = lo; i < hi; i++) {
        if (!inf_A[i]) ia.push_back((uint32_t)(i - lo));
        if (!inf_B[i]) ib.push_back((uint32_t)(i - lo));
    }
    GG_CHECK(ia.size() == nA, GG_ERR_INVALID_ARG, "len(pk.G1.A) != n_wires - NbInfinityA (shard)");
    GG_CHECK(ib.size() == nB, GG_ERR_INVALID_ARG, "len(pk.G1.B) != n_wires - NbInfinityB (shard)");
    ik.resize(nK);
    const size_t k0 = std::max(lo, nb_public);
    for (size_t i = 0; i < nK; i++) {
        size_t w = k_wire_index ? (size_t)k_wire_index[i] : k0 + i;
        GG_CHECK(w >= lo && w < hi, GG_ERR_INVALID_ARG, "K wire index outside the shard");
        ik[i] = (uint32_t)(w - lo);
    }
    GG_CHECK(nA == 0 || g1_A, GG_ERR_INVALID_ARG, "null g1_A");
    GG_CHECK(nB == 0 || (g1_B && g2_B), GG_ERR_INVALID_ARG, "null g1_B / g2_B");
    GG_CHECK(nK == 0 || g1_K, GG_ERR_INVALID_ARG, "null g1_K");
    const size_t nw = hi - lo;
    const int cAK = choose_c(std::max<size_t>(nw, 1), ps.g1a, tbits);
    int cB = choose_c(std::max<size_t>(nB, 1), 128, tbits);  // B1 shares its sort with G2
    // B1 / G2 take A's window when it is at most two bits wider than their own:
    // their entries then come out of the A / K sort by a filter (one sort fewer
    // per proof; at 2^24 the window 22 B1 / G2 MSMs cost what window 20 did,
    // profiles/r03_ah_*).  Opt-in until measured: GG_G16_B_DERIVE=1
    const bool try_derive = getenv("GG_G16_B_DERIVE") && atoi(getenv("GG_G16_B_DERIVE")) != 0;
    if (try_derive && cAK >= cB && cAK - cB <= 2 && nB) cB = cAK;
    if (const char* e = getenv("GG_G16_B_WINDOW")) cB = std::max(4, std::min(24, atoi(e)));  // A/B
    const int cZ = choose_c(std::max<size_t>(nZ, 1), ps.g1a, tbits);
    auto wb = std::make_shared<WireBases>();
    {
        auto W = [&](int c) { return (tbits + c - 1) / c; };
        const double g1a = (double)ps.g1a, g2a = (double)ps.g2a;
        const double bytes[5] = {W(cAK) * (double)nw * g1a, W(cAK) * (double)nw * g1a, W(cB) * (double)nB * g1a,
                                 W(cB) * (double)nB * g2a, W(cZ) * (double)nZ * g1a};
        const int ws[5] = {W(cAK), W(cAK), W(cB), W(cB), W(cZ)};
        const double extra = 16.0 * (W(cAK) * (double)nw + W(cB) * (double)nB + W(cZ) * (double)nZ) +
                             12.0 * 32.0 * (double)((size_t)1 << log_n);
        wb->groups = choose_groups_multi(bytes, ws, 5, extra);
    }
    // dense wire-indexed A and K (holes = infinity), one window size for both
    {
        const size_t pb = ps.g1a;
        std::vector<uint8_t> dense(nw * pb, 0);
        for (size_t j = 0; j < nA; j++) memcpy(&dense[(size_t)ia[j] * pb], (const uint8_t*)g1_A + j * pb, pb);
        wb->A = msm_base_create_internal(g1, dense.data(), nw, nullptr, cAK, true, wb->groups);
        std::fill(dense.begin(), dense.end(), 0);
        for (size_t j = 0; j < nK; j++) memcpy(&dense[(size_t)ik[j] * pb], (const uint8_t*)g1_K + j * pb, pb);
        wb->K = msm_base_create_internal(g1, dense.data(), nw, nullptr, cAK, true, wb->groups);
    }
    wb->B = msm_base_create_internal(g1, g1_B, nB, ib.data(), cB, false, wb->groups);
    wb->B2 = msm_base_create_internal(g2, g2_B, nB, ib.data(), msm_base_window(wb->B), false, wb->groups);
    wb->share_AK = msm_same_shape(wb->A, wb->K);
    wb->share_B = msm_same_shape(wb->B, wb->B2);
    if (try_derive && wb->share_B && msm_derivable(wb->A, wb->B)) {
        msm_build_bmap(wb->A, wb->B, wb->bmap);
        wb->derive_B = true;
    }
    return wb;
}

// The rest of a resident key (shard) around its wire tables: domain, Z
// positions [z_lo, z_lo + nZ), the fixed points, streams.  slog > 0: a bucket
// stripe shard over whole (shared) wire tables.
// A/B (GG_G16_H_PRIORITY=1): the computeH -> Z-MSM task on a stream of the
// greatest priority, its kernels dispatched ahead of the other tasks'
static void h_priority_ab(gg_groth16_pk* pk) {
    if (!(getenv("GG_G16_H_PRIORITY") && atoi(getenv("GG_G16_H_PRIORITY")))) return;
    if (!pk->hprio) create_copy_stream(&pk->hprio);
    pk->s1 = pk->hprio;
}

static void pk_finish(gg_groth16_pk* pk, std::shared_ptr<WireBases> wb, int curve, int log_n,
                      const void* omega_mont, const void* coset_gen_mont, const void* g1_Z, size_t z_lo, size_t nZ,
                      const void* alpha1, const void* beta1, const void* delta1, const void* beta2,
                      const void* delta2, size_t n_wires, size_t nb_public, size_t lo, size_t hi, int slog,
                      uint32_t spart) {
    GG_CHECK(omega_mont && coset_gen_mont && alpha1 && beta1 && delta1 && beta2 && delta2,
             GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(log_n >= 0 && log_n <= 28, GG_ERR_INVALID_ARG, "log_n out of range");
    const PointSizes ps = point_sizes(curve);
    const int g1 = curve == GG_CURVE_BN254 ? GG_G1 : GG_BLS12_381_G1;
    const int tbits = curve == GG_CURVE_BN254 ? 255 : 256;
    pk->curve = curve;
    pk->log_n = log_n;
    pk->n = (size_t)1 << log_n;
    pk->n_wires = n_wires;
    pk->nb_public = nb_public;
    pk->wire_lo = lo;
    pk->wire_hi = hi;
    pk->z_lo = z_lo;
    pk->nZ = nZ;
    const size_t nz_full = pk->n > 1 ? pk->n - 1 : 0;
    GG_CHECK(z_lo + nZ <= nz_full, GG_ERR_INVALID_ARG,
             "Z shard beyond domain cardinality - 1 (setup.go:266)");
    GG_CHECK(nZ == 0 || g1_Z, GG_ERR_INVALID_ARG, "null g1_Z");
    GG_HIP(hipGetDevice(&pk->device));
    memcpy(pk->alpha, alpha1, ps.g1a);
    memcpy(pk->beta, beta1, ps.g1a);
    memcpy(pk->delta, delta1, ps.g1a);
    memcpy(pk->beta2, beta2, ps.g2a);
    memcpy(pk->delta2, delta2, ps.g2a);
    ck(gg_domain_create_ex(curve, log_n, omega_mont, coset_gen_mont, &pk->dom));
    pk->wb = std::move(wb);
    pk->A = pk->wb->A;
    pk->B = pk->wb->B;
    pk->K = pk->wb->K;
    pk->B2 = pk->wb->B2;
    pk->share_AK = pk->wb->share_AK;
    pk->share_B = pk->wb->share_B;
    if (slog) {
        int cmin = 64;
        for (gg_msm_base_t b : {pk->A, pk->B})
            if (msm_scalars_needed(b)) cmin = std::min(cmin, msm_base_window(b));
        GG_CHECK(slog <= cmin - 2, GG_ERR_INVALID_ARG, "bucket stripe too fine for the tables' windows");
        GG_CHECK(spart < (1u << slog), GG_ERR_INVALID_ARG, "stripe part out of range");
        pk->slog = slog;
        pk->spart = spart;
        pk->work.reset(new WorkSet());
    }
    const int cZ = choose_c(std::max<size_t>(nZ, 1), ps.g1a, tbits);
    pk->Z = msm_base_create_internal(g1, g1_Z, nZ, nullptr, cZ, false, pk->wb->groups);
    // the longest task (G2) and the computeH chain first to a queue of their own
    int cur = 0;
    GG_HIP(hipGetDevice(&cur));
    task_streams_init(pk->active(), pk->tq, 5, cur, true);
    h_priority_ab(pk);
}

// Builds the resident key of one shard: wires [wire_lo, wire_hi) of the A, B, K
// and G2 tables and domain positions [z_lo, z_lo + nZ) of Z.  The full key is
// the single shard (0, n_wires, 0, n - 1).
static void pk_build(gg_groth16_pk* pk, int curve, int log_n, const void* omega_mont, const void* coset_gen_mont,
                     const void* g1_A, size_t nA, const void* g1_B, size_t nB, const void* g1_Z,
                     size_t z_lo, size_t nZ, const void* g1_K, size_t nK, const void* alpha1,
                     const void* beta1, const void* delta1, const void* g2_B, const void* beta2,
                     const void* delta2, const uint8_t* inf_A, const uint8_t* inf_B, size_t n_wires,
                     size_t nb_public, const uint32_t* k_wire_index, size_t lo, size_t hi) {
    GG_CHECK(log_n >= 0 && log_n <= 28, GG_ERR_INVALID_ARG, "log_n out of range");
    auto wb = wire_bases_build(curve, log_n, g1_A, nA, g1_B, nB, g1_K, nK, g2_B, inf_A, inf_B, n_wires, nb_public,
                               k_wire_index, lo, hi, nZ);
    pk_finish(pk, std::move(wb), curve, log_n, omega_mont, coset_gen_mont, g1_Z, z_lo, nZ, alpha1, beta1, delta1,
              beta2, delta2, n_wires, nb_public, lo, hi, 0, 0);
}

namespace gg {
// for the one-process multi-GPU key (groth16_multi.hip): whole wire tables
// once per device, stripe shards over them
std::shared_ptr<WireBases> g16_wire_bases(int curve, int log_n, const void* g1_A, size_t nA, const void* g1_B,
                                          size_t nB, const void* g1_K, size_t nK, const void* g2_B,
                                          const uint8_t* inf_A, const uint8_t* inf_B, size_t n_wires,
                                          size_t nb_public, const uint32_t* k_wire_index, size_t nZ) {
    return wire_bases_build(curve, log_n, g1_A, nA, g1_B, nB, g1_K, nK, g2_B, inf_A, inf_B, n_wires, nb_public,
                            k_wire_index, 0, n_wires, nZ);
}
gg_groth16_pk* g16_stripe_shard(std::shared_ptr<WireBases> wb, int curve, int log_n, const void* omega_mont,
                                const void* coset_gen_mont, const void* g1_Z, size_t z_lo, size_t nZ,
                                const void* alpha1, const void* beta1, const void* delta1, const void* beta2,
                                const void* delta2, size_t n_wires, size_t nb_public, int slog, uint32_t spart) {
    std::unique_ptr<gg_groth16_pk> pk(new gg_groth16_pk());
    pk_finish(pk.get(), std::move(wb), curve, log_n, omega_mont, coset_gen_mont, g1_Z, z_lo, nZ, alpha1, beta1,
              delta1, beta2, delta2, n_wires, nb_public, 0, n_wires, slog, spart);
    return pk.release();
}
// the smallest window of a key's wire tables (a stripe needs log2(world) <= it - 2)
int g16_wire_window(int curve, size_t n_wires, size_t nB) {
    const PointSizes ps = point_sizes(curve);
    const int tbits = curve == GG_CURVE_BN254 ? 255 : 256;
    int c = 64;
    if (n_wires) c = std::min(c, choose_c(n_wires, ps.g1a, tbits));
    if (nB) c = std::min(c, choose_c(nB, 128, tbits));
    return c;
}
// a key's task slots between proofs: `dedicated` false = the slots' own plain
// streams (the key's dedicated queues go back to the device's set), true =
// dedicated queues while the device has them (the timing rehearsal gives its
// solo shard what one GPU of a node gives its only shard).  No stream is
// created or destroyed (common.h TaskQueue).
void g16_restream(gg_groth16_pk* pk, bool dedicated) {
    std::lock_guard<std::mutex> lk(pk->mu);
    task_streams_switch(pk->active(), pk->tq, 5, pk->device, dedicated);
    h_priority_ab(pk);
}
}  // namespace gg

extern "C" int gg_groth16_pk_create_ex(int curve, int log_n, const void* omega_mont, const void* coset_gen_mont,
                                       const void* g1_A, size_t nA, const void* g1_B, size_t nB,
                                       const void* g1_Z, size_t nZ, const void* g1_K, size_t nK,
                                       const void* alpha1, const void* beta1, const void* delta1,
                                       const void* g2_B, const void* beta2, const void* delta2,
                                       const uint8_t* inf_A, const uint8_t* inf_B, size_t n_wires,
                                       size_t nb_public, const uint32_t* k_wire_index,
                                       gg_groth16_pk_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(log_n >= 0 && log_n <= 28, GG_ERR_INVALID_ARG, "log_n out of range");
    const size_t n = (size_t)1 << log_n;
    GG_CHECK(nZ + 1 == n || (n == 1 && nZ == 0), GG_ERR_INVALID_ARG,
             "len(pk.G1.Z) must be domain cardinality - 1 (setup.go:266)");
    std::unique_ptr<gg_groth16_pk> pk(new gg_groth16_pk());
    if (!k_wire_index) GG_CHECK(nb_public + nK <= n_wires, GG_ERR_INVALID_ARG, "len(pk.G1.K) too large");
    pk_build(pk.get(), curve, log_n, omega_mont, coset_gen_mont, g1_A, nA, g1_B, nB, g1_Z, 0, nZ, g1_K, nK,
             alpha1, beta1, delta1, g2_B, beta2, delta2, inf_A, inf_B, n_wires, nb_public,
             k_wire_index, 0, n_wires);
    *out = pk.release();
    GG_CAPI_END
}

extern "C" int gg_groth16_pk_create(int log_n, const void* omega_mont, const void* coset_gen_mont,
                                    const void* g1_A, size_t nA, const void* g1_B, size_t nB,
                                    const void* g1_Z, size_t nZ, const void* g1_K, size_t nK,
                                    const void* alpha1, const void* beta1, const void* delta1,
                                    const void* g2_B, const void* beta2, const void* delta2,
                                    const uint8_t* inf_A, const uint8_t* inf_B, size_t n_wires,
                                    size_t nb_public, const uint32_t* k_wire_index,
                                    gg_groth16_pk_t* out) {
    return gg_groth16_pk_create_ex(GG_CURVE_BN254, log_n, omega_mont, coset_gen_mont, g1_A, nA, g1_B, nB, g1_Z,
                                   nZ, g1_K, nK, alpha1, beta1, delta1, g2_B, beta2, delta2, inf_A, inf_B,
                                   n_wires, nb_public, k_wire_index, out);
}

extern "C" int gg_groth16_pk_create_shard_ex(int curve, int log_n, const void* omega_mont,
                                             const void* coset_gen_mont, const void* g1_A, size_t nA,
                                             const void* g1_B, size_t nB, const void* g1_Z, size_t z_lo,
                                             size_t nZ, const void* g1_K, size_t nK, const void* alpha1,
                                             const void* beta1, const void* delta1, const void* g2_B,
                                             const void* beta2, const void* delta2, const uint8_t* inf_A,
                                             const uint8_t* inf_B, size_t n_wires, size_t nb_public,
                                             const uint32_t* k_wire_index, size_t wire_lo, size_t wire_hi,
                                             gg_groth16_pk_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out, GG_ERR_INVALID_ARG, "null argument");
    std::unique_ptr<gg_groth16_pk> pk(new gg_groth16_pk());
    pk_build(pk.get(), curve, log_n, omega_mont, coset_gen_mont, g1_A, nA, g1_B, nB, g1_Z, z_lo, nZ, g1_K, nK,
             alpha1, beta1, delta1, g2_B, beta2, delta2, inf_A, inf_B, n_wires, nb_public, k_wire_index, wire_lo,
             wire_hi);
    *out = pk.release();
    GG_CAPI_END
}

extern "C" int gg_groth16_pk_create_shard(int log_n, const void* omega_mont, const void* coset_gen_mont,
                                          const void* g1_A, size_t nA, const void* g1_B, size_t nB,
                                          const void* g1_Z, size_t z_lo, size_t nZ, const void* g1_K,
                                          size_t nK, const void* alpha1, const void* beta1,
                                          const void* delta1, const void* g2_B, const void* beta2,
                                          const void* delta2, const uint8_t* inf_A,
                                          const uint8_t* inf_B, size_t n_wires, size_t nb_public,
                                          const uint32_t* k_wire_index, size_t wire_lo,
                                          size_t wire_hi, gg_groth16_pk_t* out) {
    return gg_groth16_pk_create_shard_ex(GG_CURVE_BN254, log_n, omega_mont, coset_gen_mont, g1_A, nA, g1_B, nB,
                                         g1_Z, z_lo, nZ, g1_K, nK, alpha1, beta1, delta1, g2_B, beta2, delta2,
                                         inf_A, inf_B, n_wires, nb_public, k_wire_index, wire_lo, wire_hi, out);
}

extern "C" int gg_groth16_pk_create_stripe_ex(int curve, int log_n, const void* omega_mont,
                                              const void* coset_gen_mont, const void* g1_A, size_t nA,
                                              const void* g1_B, size_t nB, const void* g1_Z, size_t z_lo,
                                              size_t nZ, const void* g1_K, size_t nK, const void* alpha1,
                                              const void* beta1, const void* delta1, const void* g2_B,
                                              const void* beta2, const void* delta2, const uint8_t* inf_A,
                                              const uint8_t* inf_B, size_t n_wires, size_t nb_public,
                                              const uint32_t* k_wire_index, int stripe_log, int stripe_part,
                                              gg_groth16_pk_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(stripe_log >= 0 && stripe_log <= 8 && stripe_part >= 0 && stripe_part < (1 << stripe_log),
             GG_ERR_INVALID_ARG, "stripe_log in [0, 8], stripe_part < 2^stripe_log");
    GG_CHECK(log_n >= 0 && log_n <= 28, GG_ERR_INVALID_ARG, "log_n out of range");
    if (!k_wire_index) GG_CHECK(nb_public + nK <= n_wires, GG_ERR_INVALID_ARG, "len(pk.G1.K) too large");
    auto wb = wire_bases_build(curve, log_n, g1_A, nA, g1_B, nB, g1_K, nK, g2_B, inf_A, inf_B, n_wires, nb_public,
                               k_wire_index, 0, n_wires, nZ);
    *out = g16_stripe_shard(std::move(wb), curve, log_n, omega_mont, coset_gen_mont, g1_Z, z_lo, nZ, alpha1, beta1,
                            delta1, beta2, delta2, n_wires, nb_public, stripe_log, (uint32_t)stripe_part);
    GG_CAPI_END
}

extern "C" int gg_groth16_pk_stripe(gg_groth16_pk_t pk, int* stripe_log, int* stripe_part) {
    GG_CAPI_BEGIN
    GG_CHECK(pk, GG_ERR_INVALID_ARG, "null key");
    if (stripe_log) *stripe_log = pk->slog;
    if (stripe_part) *stripe_part = (int)pk->spart;
    GG_CAPI_END
}

extern "C" int gg_groth16_pk_base_info(gg_groth16_pk_t pk, int which, size_t* n_points, int* window_bits,
                                       int* n_windows) {
    GG_CAPI_BEGIN
    GG_CHECK(pk && which >= 0 && which <= 4, GG_ERR_INVALID_ARG, "bad argument");
    gg_msm_base_t b[5] = {pk->A, pk->B, pk->K, pk->Z, pk->B2};
    return gg_msm_base_info(b[which], n_points, window_bits, n_windows);
    GG_CAPI_END
}

extern "C" int gg_groth16_pk_base_layout(gg_groth16_pk_t pk, int which, int* groups, int* stored_windows,
                                         size_t* table_bytes) {
    GG_CAPI_BEGIN
    GG_CHECK(pk && which >= 0 && which <= 4, GG_ERR_INVALID_ARG, "bad argument");
    gg_msm_base_t b[5] = {pk->A, pk->B, pk->K, pk->Z, pk->B2};
    return gg_msm_base_layout(b[which], groups, stored_windows, table_bytes);
    GG_CAPI_END
}

extern "C" int gg_groth16_pk_release(gg_groth16_pk_t pk) {
    GG_CAPI_BEGIN
    delete pk;
    GG_CAPI_END
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

template <class T>
static T from_bytes(const void* p) {
    T x;
    memcpy(&x, p, sizeof(T));
    return x;
}

// MSM partials of one key (shard): the device section of prove.go:198-301, as
// the curve's Jacobian points (BN254 96 / 192 B, BLS12-381 144 / 288 B)
struct G16Partials {
    alignas(16) uint8_t a[144], b1[144], k[144], z[144];  // Σ w·A, Σ w·B1, Σ w·K (filtered), Σ h·Z
    alignas(16) uint8_t b2[288];                          // Σ w·B2
};
static void set_g1_inf(int curve, void* p) {
    if (curve == GG_CURVE_BN254) {
        G1Jac j = G1Jac::inf();
        memcpy(p, &j, sizeof(j));
    } else {
        Jac<FpBls> j = Jac<FpBls>::inf();
        memcpy(p, &j, sizeof(j));
    }
}
// partials <-> the flat layout of gg_groth16_prove_partial: a | b1 | k | z | b2
static void partials_put(int curve, const G16Partials& p, void* out) {
    const PointSizes ps = point_sizes(curve);
    uint8_t* o = (uint8_t*)out;
    memcpy(o, p.a, ps.g1j);
    memcpy(o + ps.g1j, p.b1, ps.g1j);
    memcpy(o + 2 * ps.g1j, p.k, ps.g1j);
    memcpy(o + 3 * ps.g1j, p.z, ps.g1j);
    memcpy(o + 4 * ps.g1j, p.b2, ps.g2j);
}
static void partials_get(int curve, const void* in, G16Partials& p) {
    const PointSizes ps = point_sizes(curve);
    const uint8_t* q = (const uint8_t*)in;
    memcpy(p.a, q, ps.g1j);
    memcpy(p.b1, q + ps.g1j, ps.g1j);
    memcpy(p.k, q + 2 * ps.g1j, ps.g1j);
    memcpy(p.z, q + 3 * ps.g1j, ps.g1j);
    memcpy(p.b2, q + 4 * ps.g1j, ps.g2j);
}

// Joins every worker on scope exit, also while an exception unwinds (the
// workers reference locals of prove_device, declared before the joiner).
struct Joiner {
    std::vector<gg::Task<void>>& v;
    ~Joiner() {
        for (auto& t : v)
            if (t.valid()) t.wait();
    }
};

// Uploads the solution and runs computeH + the five MSMs of `pk` (a shard, or
// the whole key).  Host inputs go through the key's pinned stager: the wires
// first (the MSM sorts start as soon as they land), then A, B, C from the H
// task while the MSMs already run (icicle.go:231-278, 478-480 copy them
// synchronously before any compute).  g_timings[0..6] and g_ext[0..1] are filled.
static void prove_device(gg_groth16_pk* pk, const void* wires, const void* sol_a,
                         const void* sol_b, const void* sol_c, size_t n_cons,
                         bool inputs_on_device, void* h_dev_out, G16Partials& out,
                         const DistH* dh = nullptr) {
    double t0 = now_ms();
    const size_t n = pk->n;
    const size_t nbytes = n * 32;
    const size_t nw_shard = pk->wire_hi - pk->wire_lo;
    const Fr* wdev = (const Fr*)wires;
    if (!inputs_on_device) {
        if (!pk->stager) pk->stager.reset(new Stager(pk->device));
        // the shard's tables are indexed from its first wire: upload only its wires
        pk->wires.reserve(std::max<size_t>(nw_shard, 1) * 32);
        pk->stager->upload(pk->wires.p, (const uint8_t*)wires + pk->wire_lo * 32, nw_shard * 32);
        const hipStream_t cons[4] = {pk->s0, pk->s2, pk->s3, pk->s4};
        pk->stager->ready(cons, 4);
        wdev = pk->wires.as<Fr>();
    } else {
        wdev += pk->wire_lo;
    }
    double t_up = now_ms();

    // Five concurrent tasks, one host thread + HIP stream each (MSM tails are
    // latency-bound, so overlapping them fills the chip):
    //   s1: [A, B, C upload] computeH -> Z-MSM (h lands in A's buffer)
    //   s2: A-MSM    s3: B1-MSM    s4: K-MSM    s0 (this thread): G2-MSM
    set_g1_inf(pk->curve, out.z);
    double t_h = 0, t_z = 0, t_a = 0, t_b = 0, t_k = 0, t_upabc = 0;
    std::mutex emu;
    std::string werr;
    int wcode = GG_OK;
    const int dev = pk->device;
    auto guarded = [&](auto fn) {
        return [&, fn]() {
            try {
                GG_HIP(hipSetDevice(dev));
                fn();
            } catch (const Error& e) {
                std::lock_guard<std::mutex> g(emu);
                if (wcode == GG_OK) { werr = e.what(); wcode = e.code; }
            } catch (const std::exception& e) {
                std::lock_guard<std::mutex> g(emu);
                if (wcode == GG_OK) { werr = e.what(); wcode = GG_ERR_INTERNAL; }
            }
        };
    };
    // GG_G16_SERIAL=1 runs the tasks one after another (per-stage isolated timings)
    const bool serial = getenv("GG_G16_SERIAL") && atoi(getenv("GG_G16_SERIAL"));
    std::vector<gg::Task<void>> workers;  // on kept worker threads (common.h run_task)
    Joiner joiner{workers};
    auto spawn = [&](auto fn) {
        if (serial) fn();
        else workers.push_back(gg::run_task(fn));
    };
    // A, B, C -> device (or the distributed H's cyclic slices), on the H task
    auto inputs_abc = [&](Fr*& A, Fr*& B, Fr*& C, size_t& len) {
        const void* src[3] = {sol_a, sol_b, sol_c};
        Fr* dst[3] = {pk->sa.as<Fr>(), pk->sb.as<Fr>(), pk->sc.as<Fr>()};
        len = n_cons;
        const double a = now_ms();
        if (inputs_on_device) {
            for (int i = 0; i < 3; i++) {
                if (dh) { dst[i] = (Fr*)src[i]; continue; }
                if (n_cons) GG_HIP(hipMemcpyAsync(dst[i], src[i], n_cons * 32, hipMemcpyDeviceToDevice, pk->s1));
                if (n_cons < n) GG_HIP(hipMemsetAsync((char*)dst[i] + n_cons * 32, 0, nbytes - n_cons * 32, pk->s1));
            }
        } else if (dh) {
            // rank r of the distributed computeH reads x[r + N j] only: gather that
            // cyclic slice on the host (1/N of the bytes over this GPU's link)
            int rank = 0, world = 1, lg = 0;
            hshard_m(dh->hs, &rank, &world, &lg);
            len = n_cons > (size_t)rank ? (n_cons - (size_t)rank + world - 1) / world : 0;
            for (int i = 0; i < 3; i++)
                pk->stager->upload_strided(dst[i], src[i], 32, (size_t)rank, (size_t)world, len);
            pk->stager->ready(&pk->s1, 1);
        } else {
            for (int i = 0; i < 3; i++) {
                if (n_cons < n) GG_HIP(hipMemsetAsync((char*)dst[i] + n_cons * 32, 0, nbytes - n_cons * 32, pk->s1));
                pk->stager->upload(dst[i], src[i], n_cons * 32);
            }
            pk->stager->ready(&pk->s1, 1);
        }
        t_upabc = now_ms() - a;
        A = dst[0];
        B = dst[1];
        C = dst[2];
    };
    pk->sa.reserve(nbytes);
    pk->sb.reserve(nbytes);
    pk->sc.reserve(nbytes);
    if (dh) spawn(guarded([&] {
        Fr *A, *B, *C;
        size_t len;
        double a = now_ms();
        inputs_abc(A, B, C, len);
        const bool compact = !inputs_on_device;
        hshard_run(dh->hs, A, B, C, len, compact, dh->send, dh->recv, dh->xchg, dh->ctx, pk->s1);
        GG_WAIT_STREAM(pk->s1);
        double b = now_ms();
        t_h = b - a;
        msm_device(pk->Z, hshard_h(dh->hs), out.z, pk->s1);
        t_z = now_ms() - b;
    }));
    else spawn(guarded([&] {
        Fr *A, *B, *C;
        size_t len;
        double a = now_ms();
        inputs_abc(A, B, C, len);
        compute_h_device(pk->dom, A, B, C, A, pk->s1);
        GG_WAIT_STREAM(pk->s1);
        double b = now_ms();
        t_h = b - a;
        if (h_dev_out) GG_HIP(hipMemcpyAsync(h_dev_out, A, nbytes, hipMemcpyDeviceToDevice, pk->s1));
        if (n > 1) msm_device(pk->Z, A + pk->z_lo, out.z, pk->s1);
        t_z = now_ms() - b;
    }));
    // wire sorts, enqueued from this thread before any finisher waits on their
    // events: A's (shared with K) on s2, B1's (shared with G2) on s3
    // (a stripe shard sorts its bucket stripe into its own work set: the tables
    // are shared with the other shards on this device)
    MsmSort *sAK = nullptr, *sB = nullptr, *sK = nullptr, *sB2 = nullptr;
    MsmScratch *xA = nullptr, *xB = nullptr, *xK = nullptr, *xB2 = nullptr;
    WorkSet* ws = pk->work.get();
    guarded([&] {
        sAK = ws ? msm_work_sort(ws->A) : msm_own_sort(pk->A);
        sB = ws ? msm_work_sort(ws->B) : msm_own_sort(pk->B);
        sK = pk->share_AK ? sAK : (ws ? msm_work_sort(ws->K) : msm_own_sort(pk->K));
        sB2 = pk->share_B ? sB : (ws ? msm_work_sort(ws->B2) : msm_own_sort(pk->B2));
        if (ws) {
            xA = msm_work_scratch(ws->A);
            xB = msm_work_scratch(ws->B);
            xK = msm_work_scratch(ws->K);
            xB2 = msm_work_scratch(ws->B2);
        }
        msm_prepare_dev(pk->A, sAK, wdev, pk->s2, pk->slog, pk->spart);
        if (pk->wb->derive_B)  // B1 / G2's entries filtered out of the A / K sort
            msm_prepare_derived_dev(pk->A, sAK, pk->B, sB, pk->wb->bmap.as<uint32_t>(), pk->s3);
        else
            msm_prepare_dev(pk->B, sB, wdev, pk->s3, pk->slog, pk->spart);
        if (!pk->share_AK) msm_prepare_dev(pk->K, sK, wdev, pk->s4, pk->slog, pk->spart);
        if (!pk->share_B) msm_prepare_dev(pk->B2, sB2, wdev, pk->s0, pk->slog, pk->spart);
    })();
    double t2 = now_ms(), te = t2;
    if (wcode == GG_OK) {  // the sorts are enqueued: run the finishers
        spawn(guarded([&] { double a = now_ms(); msm_finish_dev(pk->A, sAK, out.a, pk->s2, xA); t_a = now_ms() - a; }));
        spawn(guarded([&] { double a = now_ms(); msm_finish_dev(pk->B, sB, out.b1, pk->s3, xB); t_b = now_ms() - a; }));
        spawn(guarded([&] { double a = now_ms(); msm_finish_dev(pk->K, sK, out.k, pk->s4, xK); t_k = now_ms() - a; }));
        t2 = now_ms();
        guarded([&] { msm_finish_dev(pk->B2, sB2, out.b2, pk->s0, xB2); })();
        te = now_ms();
    }
    for (auto& w : workers) w.wait();
    if (wcode != GG_OK) throw Error(wcode, werr);
    g_timings[0] = t_up - t0;
    g_timings[1] = t_h;
    g_timings[2] = t_a;
    g_timings[3] = t_b;
    g_timings[4] = t_k;
    g_timings[5] = t_z;
    g_timings[6] = te - t2;
    g_ext[0] = t_upabc;
}

// Fixed-point terms of the proof (prove.go:177-192, 293-296): kr = -r*s and
// r*delta, s*delta, kr*delta, s*delta2 -- independent of the MSMs.
template <class Cv>
struct G16Fixed {
    typename Cv::FrT rc, sc;  // r, s in canonical form (scalar-mul digits)
    Jac<typename Cv::G1F> rd, sd, krd;
    Jac<typename Cv::G2F> sd2;
};

template <class Cv>
static gg::Task<G16Fixed<Cv>> fixed_terms_async(const void* delta_aff, const void* delta2_aff, const void* r_mont,
                                                   const void* s_mont) {
    using G1 = typename Cv::G1F;
    using G2 = typename Cv::G2F;
    using FrT = typename Cv::FrT;
    const Affine<G1> delta = from_bytes<Affine<G1>>(delta_aff);
    const Affine<G2> delta2 = from_bytes<Affine<G2>>(delta2_aff);
    const FrT r = from_bytes<FrT>(r_mont), s = from_bytes<FrT>(s_mont);
    return gg::run_task([delta, delta2, r, s] {
        G16Fixed<Cv> f;
        FrT kr = -(r * s);
        f.rc = from_mont(r);
        f.sc = from_mont(s);
        FrT krc = from_mont(kr);
        Jac<G1> dl = Jac<G1>::from_affine(delta);
        auto f_rd = gg::run_task([&] { return jac_mul(dl, f.rc.v); });
        auto f_sd = gg::run_task([&] { return jac_mul(dl, f.sc.v); });
        auto f_sd2 = gg::run_task([&] { return jac_mul(Jac<G2>::from_affine(delta2), f.sc.v); });
        f.krd = jac_mul(dl, krc.v);
        f.rd = f_rd.get();
        f.sd = f_sd.get();
        f.sd2 = f_sd2.get();
        return f;
    });
}

// Combination of the (summed) MSM partials, prove.go:206-299 verbatim:
//   Ar  = Σ w·A + α + r·δ                  Bs1 = Σ w·B1 + β + s·δ
//   Krs = Σ w·K + kr·δ + Σ h·Z + s·Ar + r·Bs1
//   Bs  = Σ w·B2 + s·δ2 + β2
template <class Cv>
static void g16_combine(const G16Partials& p, const G16Fixed<Cv>& f, const void* alpha_aff, const void* beta_aff,
                        const void* beta2_aff, void* ar_aff, void* bs_aff, void* krs_aff) {
    using G1 = typename Cv::G1F;
    using G2 = typename Cv::G2F;
    const Affine<G1> alpha = from_bytes<Affine<G1>>(alpha_aff), beta = from_bytes<Affine<G1>>(beta_aff);
    const Affine<G2> beta2 = from_bytes<Affine<G2>>(beta2_aff);
    const Jac<G1> pa = from_bytes<Jac<G1>>(p.a), pb1 = from_bytes<Jac<G1>>(p.b1), pk = from_bytes<Jac<G1>>(p.k),
                  pz = from_bytes<Jac<G1>>(p.z);
    const Jac<G2> pb2 = from_bytes<Jac<G2>>(p.b2);
    Jac<G1> ar = jac_add(jac_add_affine(pa, alpha), f.rd);
    Jac<G1> bs1 = jac_add(jac_add_affine(pb1, beta), f.sd);
    auto f_sar = gg::run_task([&] { return jac_mul(ar, f.sc.v); });
    Jac<G1> rbs = jac_mul(bs1, f.rc.v);
    Jac<G1> krs = jac_add(jac_add(pk, f.krd), pz);
    krs = jac_add(krs, f_sar.get());
    krs = jac_add(krs, rbs);
    Jac<G2> bs = jac_add_affine(jac_add(pb2, f.sd2), beta2);
    const Affine<G1> o_ar = jac_to_affine(ar), o_krs = jac_to_affine(krs);
    const Affine<G2> o_bs = jac_to_affine(bs);
    memcpy(ar_aff, &o_ar, sizeof(o_ar));
    memcpy(krs_aff, &o_krs, sizeof(o_krs));
    memcpy(bs_aff, &o_bs, sizeof(o_bs));
}

template <class Cv>
static void prove_whole(gg_groth16_pk* pk, const void* wires, const void* sol_a, const void* sol_b,
                        const void* sol_c, size_t n_cons, bool on_dev, const void* r_mont, const void* s_mont,
                        void* ar_aff, void* bs_aff, void* krs_aff, void* h_dev_out) {
    double t0 = now_ms();
    // host pool computes the fixed-point terms while the GPU works
    auto fixed = fixed_terms_async<Cv>(pk->delta, pk->delta2, r_mont, s_mont);
    G16Partials p;
    prove_device(pk, wires, sol_a, sol_b, sol_c, n_cons, on_dev, h_dev_out, p);
    double tep = now_ms();
    g16_combine<Cv>(p, fixed.get(), pk->alpha, pk->beta, pk->beta2, ar_aff, bs_aff, krs_aff);
    double tend = now_ms();
    g_timings[7] = tend - tep;
    g_timings[8] = tend - t0;
}

static void check_prove_args(gg_groth16_pk_t pk, const void* wires, size_t n_wires, const void* a,
                             const void* b, const void* c, size_t n_cons) {
    GG_CHECK(pk && wires && a && b && c, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(n_wires == pk->n_wires, GG_ERR_INVALID_ARG, "len(wires) != pk wires");
    GG_CHECK(n_cons <= pk->n, GG_ERR_INVALID_ARG, "nbConstraints > domain cardinality");
}

extern "C" int gg_groth16_prove(gg_groth16_pk_t pk, const void* wires, size_t n_wires,
                                const void* sol_a, const void* sol_b, const void* sol_c,
                                size_t n_cons, int inputs_on_device, const void* r_mont,
                                const void* s_mont, void* ar_aff, void* bs_aff, void* krs_aff,
                                void* h_dev_out) {
    GG_CAPI_BEGIN
    check_prove_args(pk, wires, n_wires, sol_a, sol_b, sol_c, n_cons);
    GG_CHECK(r_mont && s_mont && ar_aff && bs_aff && krs_aff, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(pk->wire_lo == 0 && pk->wire_hi == pk->n_wires && pk->z_lo == 0 && pk->slog == 0 &&
                 pk->nZ == (pk->n > 1 ? pk->n - 1 : 0),
             GG_ERR_INVALID_ARG, "gg_groth16_prove needs the whole key; a shard proves with "
                                 "gg_groth16_prove_partial + gg_groth16_finalize");
    g_ext[1] = now_ms();
    std::lock_guard<std::mutex> lk(pk->mu);
    g_ext[0] = 0;
    if (pk->curve == GG_CURVE_BN254)
        prove_whole<CurveBn254>(pk, wires, sol_a, sol_b, sol_c, n_cons, inputs_on_device != 0, r_mont, s_mont,
                                ar_aff, bs_aff, krs_aff, h_dev_out);
    else
        prove_whole<CurveBls12381>(pk, wires, sol_a, sol_b, sol_c, n_cons, inputs_on_device != 0, r_mont, s_mont,
                                   ar_aff, bs_aff, krs_aff, h_dev_out);
    g_ext[2] = now_ms();
    if (kAccumProbe) {
        set_last_error("traffic-probe build (GG_ACCUM_PROBE): the MSM sums are wrong, the proof is NOT valid");
        return GG_REHEARSAL;
    }
    GG_CAPI_END
}

extern "C" int gg_groth16_prove_partial(gg_groth16_pk_t pk, const void* wires, size_t n_wires,
                                        const void* sol_a, const void* sol_b, const void* sol_c,
                                        size_t n_cons, int inputs_on_device, void* partials,
                                        void* h_dev_out) {
    GG_CAPI_BEGIN
    check_prove_args(pk, wires, n_wires, sol_a, sol_b, sol_c, n_cons);
    GG_CHECK(partials, GG_ERR_INVALID_ARG, "null argument");
    std::lock_guard<std::mutex> lk(pk->mu);
    g_ext[0] = 0;
    double t0 = now_ms();
    G16Partials p;
    prove_device(pk, wires, sol_a, sol_b, sol_c, n_cons, inputs_on_device != 0, h_dev_out, p);
    partials_put(pk->curve, p, partials);
    g_timings[7] = 0;
    g_timings[8] = now_ms() - t0;
    GG_PROBE_GUARD();
    GG_CAPI_END
}

extern "C" int gg_groth16_prove_partial_dist(gg_groth16_pk_t pk, gg_hshard_t hs, const void* wires,
                                             size_t n_wires, const void* sol_a, const void* sol_b,
                                             const void* sol_c, size_t n_cons, int inputs_on_device,
                                             gg_exchange_fn xchg, void* xchg_ctx, void* send_dev,
                                             void* recv_dev, void* partials) {
    GG_CAPI_BEGIN
    check_prove_args(pk, wires, n_wires, sol_a, sol_b, sol_c, n_cons);
    GG_CHECK(hs && xchg && send_dev && recv_dev && partials, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(hshard_curve(hs) == pk->curve, GG_ERR_INVALID_ARG, "hshard and key are over different curves");
    int rank = 0, world = 1, log_n = 0;
    size_t m = hshard_m(hs, &rank, &world, &log_n);
    GG_CHECK(log_n == pk->log_n, GG_ERR_INVALID_ARG, "hshard and key have different domains");
    GG_CHECK(pk->z_lo == (size_t)rank * m && pk->nZ == std::min(m, pk->n - 1 - pk->z_lo),
             GG_ERR_INVALID_ARG, "key shard must own Z positions [rank*m, (rank+1)*m)");
    std::lock_guard<std::mutex> lk(pk->mu);
    g_ext[0] = 0;
    double t0 = now_ms();
    G16Partials p;
    DistH dh{hs, xchg, xchg_ctx, (Fr*)send_dev, (Fr*)recv_dev};
    prove_device(pk, wires, sol_a, sol_b, sol_c, n_cons, inputs_on_device != 0, nullptr, p, &dh);
    partials_put(pk->curve, p, partials);
    g_timings[7] = 0;
    g_timings[8] = now_ms() - t0;
    GG_PROBE_GUARD();
    GG_CAPI_END
}

extern "C" int gg_groth16_finalize_ex(int curve, const void* alpha1, const void* beta1, const void* delta1,
                                      const void* beta2, const void* delta2, const void* partials,
                                      const void* r_mont, const void* s_mont, void* ar_aff, void* bs_aff,
                                      void* krs_aff) {
    GG_CAPI_BEGIN
    GG_CHECK(alpha1 && beta1 && delta1 && beta2 && delta2 && partials && r_mont && s_mont && ar_aff && bs_aff &&
                 krs_aff,
             GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "bad curve");
    G16Partials p;
    partials_get(curve, partials, p);
    if (curve == GG_CURVE_BN254) {
        auto fixed = fixed_terms_async<CurveBn254>(delta1, delta2, r_mont, s_mont);
        g16_combine<CurveBn254>(p, fixed.get(), alpha1, beta1, beta2, ar_aff, bs_aff, krs_aff);
    } else {
        auto fixed = fixed_terms_async<CurveBls12381>(delta1, delta2, r_mont, s_mont);
        g16_combine<CurveBls12381>(p, fixed.get(), alpha1, beta1, beta2, ar_aff, bs_aff, krs_aff);
    }
    GG_CAPI_END
}

struct gg_g16_fixed {
    int curve = GG_CURVE_BN254;
    gg::Task<G16Fixed<CurveBn254>> bn;
    gg::Task<G16Fixed<CurveBls12381>> bls;
};

extern "C" int gg_groth16_finalize_begin(int curve, const void* delta1, const void* delta2, const void* r_mont,
                                         const void* s_mont, gg_g16_fixed_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(delta1 && delta2 && r_mont && s_mont && out, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "bad curve");
    std::unique_ptr<gg_g16_fixed> h(new gg_g16_fixed());
    h->curve = curve;
    if (curve == GG_CURVE_BN254) h->bn = fixed_terms_async<CurveBn254>(delta1, delta2, r_mont, s_mont);
    else h->bls = fixed_terms_async<CurveBls12381>(delta1, delta2, r_mont, s_mont);
    *out = h.release();
    GG_CAPI_END
}

extern "C" int gg_groth16_finalize_end(gg_g16_fixed_t h, const void* alpha1, const void* beta1, const void* beta2,
                                       const void* partials, void* ar_aff, void* bs_aff, void* krs_aff) {
    GG_CAPI_BEGIN
    GG_CHECK(h, GG_ERR_INVALID_ARG, "null handle");
    std::unique_ptr<gg_g16_fixed> own(h);  // released on every path (the futures join their threads)
    if (!partials) return GG_OK;
    GG_CHECK(alpha1 && beta1 && beta2 && ar_aff && bs_aff && krs_aff, GG_ERR_INVALID_ARG, "null argument");
    G16Partials p;
    partials_get(h->curve, partials, p);
    if (h->curve == GG_CURVE_BN254) g16_combine<CurveBn254>(p, h->bn.get(), alpha1, beta1, beta2, ar_aff, bs_aff, krs_aff);
    else g16_combine<CurveBls12381>(p, h->bls.get(), alpha1, beta1, beta2, ar_aff, bs_aff, krs_aff);
    GG_CAPI_END
}

extern "C" int gg_groth16_finalize(const void* alpha1, const void* beta1, const void* delta1,
                                   const void* beta2, const void* delta2, const void* partials,
                                   const void* r_mont, const void* s_mont, void* ar_aff,
                                   void* bs_aff, void* krs_aff) {
    return gg_groth16_finalize_ex(GG_CURVE_BN254, alpha1, beta1, delta1, beta2, delta2, partials, r_mont, s_mont,
                                  ar_aff, bs_aff, krs_aff);
}

extern "C" int gg_groth16_last_timings_ex(double* ms, int cap) {
    GG_CAPI_BEGIN
    GG_CHECK(ms && cap >= 0, GG_ERR_INVALID_ARG, "null argument");
    double all[12];
    memcpy(all, g_timings, sizeof(g_timings));
    all[9] = g_ext[0];
    all[10] = g_ext[1];
    all[11] = g_ext[2];
    memcpy(ms, all, sizeof(double) * (size_t)std::min(cap, 12));
    GG_CAPI_END
}

extern "C" int gg_groth16_last_timings(double* ms9) {
    GG_CAPI_BEGIN
    GG_CHECK(ms9, GG_ERR_INVALID_ARG, "null argument");
    memcpy(ms9, g_timings, sizeof(g_timings));
    GG_CAPI_END
}
