// C ABI of the MSM engine (see msm_impl.cuh for the algorithm).
#include "msm_impl.cuh"
#include <cmath>

namespace gg {
void create_base_g1(gg_msm_base* b, const void* points, size_t n, int on_device,
                    const uint32_t* sidx, int window_bits, bool keep_inf, int groups);
void create_base_g2(gg_msm_base* b, const void* points, size_t n, int on_device,
                    const uint32_t* sidx, int window_bits, bool keep_inf, int groups);
void create_base_bls(gg_msm_base* b, const void* points, size_t n, int on_device,
                     const uint32_t* sidx, int window_bits, bool keep_inf, int groups);
void create_base_bls2(gg_msm_base* b, const void* points, size_t n, int on_device,
                      const uint32_t* sidx, int window_bits, bool keep_inf, int groups);
void msm_run_bls2(gg_msm_base* b, MsmWork* w, const Fr* scalars_dev, void* out_jac, hipStream_t st);
void msm_finish_bls2(gg_msm_base* b, MsmSort* s, MsmScratch* scr, void* out_jac, hipStream_t st);
void msm_run_g1(gg_msm_base* b, MsmWork* w, const Fr* scalars_dev, void* out_jac, hipStream_t st);
void msm_run_g2(gg_msm_base* b, MsmWork* w, const Fr* scalars_dev, void* out_jac, hipStream_t st);
void msm_run_bls(gg_msm_base* b, MsmWork* w, const Fr* scalars_dev, void* out_jac, hipStream_t st);
void msm_finish_g1(gg_msm_base* b, MsmSort* s, MsmScratch* scr, void* out_jac, hipStream_t st);
void msm_finish_g2(gg_msm_base* b, MsmSort* s, MsmScratch* scr, void* out_jac, hipStream_t st);
void msm_finish_bls(gg_msm_base* b, MsmSort* s, MsmScratch* scr, void* out_jac, hipStream_t st);
void msm_run_batch_g1(gg_msm_base* b, MsmWork* w, const VecPtrs& vp, int nvec, void* const* out_jac, hipStream_t st);
void msm_run_batch_g2(gg_msm_base* b, MsmWork* w, const VecPtrs& vp, int nvec, void* const* out_jac, hipStream_t st);
void msm_run_batch_bls(gg_msm_base* b, MsmWork* w, const VecPtrs& vp, int nvec, void* const* out_jac, hipStream_t st);
void msm_run_batch_bls2(gg_msm_base* b, MsmWork* w, const VecPtrs& vp, int nvec, void* const* out_jac,
                        hipStream_t st);
}  // namespace gg

using namespace gg;

extern "C" int gg_msm_base_create(int group, const void* points, size_t n, int points_on_device,
                                  const uint32_t* scalar_index, int window_bits,
                                  gg_msm_base_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out, GG_ERR_INVALID_ARG, "null out");
    GG_CHECK(group == GG_G1 || group == GG_G2 || group == GG_BLS12_381_G1 || group == GG_BLS12_381_G2,
             GG_ERR_INVALID_ARG, "group must be GG_G1, GG_G2, GG_BLS12_381_G1 or GG_BLS12_381_G2");
    GG_CHECK(n == 0 || points, GG_ERR_INVALID_ARG, "null points");
    GG_CHECK(n < 0x80000000ull, GG_ERR_INVALID_ARG, "n too large");
    std::unique_ptr<gg_msm_base> b(new gg_msm_base());
    b->group = group;
    if (group == GG_G1) create_base_g1(b.get(), points, n, points_on_device, scalar_index, window_bits, false, 0);
    else if (group == GG_G2) create_base_g2(b.get(), points, n, points_on_device, scalar_index, window_bits, false, 0);
    else if (group == GG_BLS12_381_G1) create_base_bls(b.get(), points, n, points_on_device, scalar_index, window_bits, false, 0);
    else create_base_bls2(b.get(), points, n, points_on_device, scalar_index, window_bits, false, 0);
    *out = b.release();
    GG_CAPI_END
}

extern "C" int gg_msm_base_release(gg_msm_base_t b) {
    GG_CAPI_BEGIN
    delete b;
    GG_CAPI_END
}

extern "C" int gg_msm_base_layout(gg_msm_base_t b, int* groups, int* stored_windows, size_t* table_bytes) {
    GG_CAPI_BEGIN
    GG_CHECK(b, GG_ERR_INVALID_ARG, "null base");
    if (groups) *groups = b->G;
    if (stored_windows) *stored_windows = b->Ws;
    if (table_bytes) *table_bytes = b->pts.bytes;
    GG_CAPI_END
}

extern "C" int gg_msm_base_info(gg_msm_base_t b, size_t* n_points, int* window_bits, int* n_windows) {
    GG_CAPI_BEGIN
    GG_CHECK(b, GG_ERR_INVALID_ARG, "null base");
    if (n_points) *n_points = b->n;
    if (window_bits) *window_bits = b->c;
    if (n_windows) *n_windows = b->W;
    GG_CAPI_END
}

namespace gg {
// one MSM over b with the work state w (no lock: b is read-only, w is the caller's)
void msm_device_work(gg_msm_base* b, MsmWork* w, const Fr* scalars_dev, void* out_jac, hipStream_t st) {
    if (b->group == GG_G1) msm_run_g1(b, w, scalars_dev, out_jac, st);
    else if (b->group == GG_G2) msm_run_g2(b, w, scalars_dev, out_jac, st);
    else if (b->group == GG_BLS12_381_G1) msm_run_bls(b, w, scalars_dev, out_jac, st);
    else msm_run_bls2(b, w, scalars_dev, out_jac, st);
}
// nvec (<= kMaxBatch) MSMs over b as one (same-base commitments); out_jac[v]
// receives the v-th
void msm_device_work_batch(gg_msm_base* b, MsmWork* w, const Fr* const* scalars_dev, int nvec, void* const* out_jac,
                           hipStream_t st) {
    GG_CHECK(nvec >= 1 && nvec <= kMaxBatch, GG_ERR_INVALID_ARG, "batch of 1..4 scalar vectors");
    VecPtrs vp{};
    for (int v = 0; v < nvec; v++) vp.p[v] = scalars_dev[v];
    if (b->group == GG_G1) msm_run_batch_g1(b, w, vp, nvec, out_jac, st);
    else if (b->group == GG_G2) msm_run_batch_g2(b, w, vp, nvec, out_jac, st);
    else if (b->group == GG_BLS12_381_G1) msm_run_batch_bls(b, w, vp, nvec, out_jac, st);
    else msm_run_batch_bls2(b, w, vp, nvec, out_jac, st);
}
static void msm_device_locked(gg_msm_base* b, const Fr* scalars_dev, void* out_jac, hipStream_t st) {
    msm_device_work(b, &b->own, scalars_dev, out_jac, st);
}
// used by the Groth16 prover as well
void msm_device(gg_msm_base* b, const Fr* scalars_dev, void* out_jac, hipStream_t st) {
    std::lock_guard<std::mutex> lk(b->mu);
    msm_device_locked(b, scalars_dev, out_jac, st);
}
// ---- shared sorts (Groth16): bases of one shape reuse one MsmSort
gg_msm_base* msm_base_create_internal(int group, const void* host_points, size_t n,
                                      const uint32_t* sidx, int window_bits, bool keep_inf, int groups) {
    std::unique_ptr<gg_msm_base> b(new gg_msm_base());
    b->group = group;
    if (group == GG_G1) create_base_g1(b.get(), host_points, n, 0, sidx, window_bits, keep_inf, groups);
    else if (group == GG_G2) create_base_g2(b.get(), host_points, n, 0, sidx, window_bits, keep_inf, groups);
    else if (group == GG_BLS12_381_G1) create_base_bls(b.get(), host_points, n, 0, sidx, window_bits, keep_inf, groups);
    else create_base_bls2(b.get(), host_points, n, 0, sidx, window_bits, keep_inf, groups);
    return b.release();
}
bool msm_same_shape(const gg_msm_base* a, const gg_msm_base* b) {
    if (a->n != b->n || a->c != b->c || a->W != b->W || a->G != b->G || a->has_sidx != b->has_sidx) return false;
    if (!a->has_sidx || a->n == 0) return true;
    std::vector<uint32_t> x(a->n), y(b->n);
    GG_HIP(hipMemcpy(x.data(), a->sidx.p, a->n * 4, hipMemcpyDeviceToHost));
    GG_HIP(hipMemcpy(y.data(), b->sidx.p, b->n * 4, hipMemcpyDeviceToHost));
    return x == y;
}
MsmSort* msm_own_sort(gg_msm_base* b) { return &b->own.sort; }
MsmWork* msm_work_new() { return new MsmWork(); }
void msm_work_delete(MsmWork* w) { delete w; }
int msm_base_window(const gg_msm_base* b) { return b->c; }
int msm_base_groups(const gg_msm_base* b) { return b->G; }
void msm_prepare_dev(gg_msm_base* b, MsmSort* s, const Fr* scalars_dev, hipStream_t st, int slog, uint32_t sres) {
    if (b->n) msm_prepare(b, s, scalars_dev, st, slog, sres);
}
// scr: the MSM's scratch (nullptr = the base's own)
void msm_finish_dev(gg_msm_base* b, MsmSort* s, void* out_jac, hipStream_t st, MsmScratch* scr) {
    if (!scr) scr = &b->own.scr;
    if (b->group == GG_G1) msm_finish_g1(b, s, scr, out_jac, st);
    else if (b->group == GG_G2) msm_finish_g2(b, s, scr, out_jac, st);
    else if (b->group == GG_BLS12_381_G1) msm_finish_bls(b, s, scr, out_jac, st);
    else msm_finish_bls2(b, s, scr, out_jac, st);
}
void msm_prepare_derived_dev(gg_msm_base* a, MsmSort* sa, gg_msm_base* b, MsmSort* sb, const uint32_t* bmap,
                             hipStream_t st) {
    if (b->n) msm_prepare_derived(a, sa, b, sb, bmap, st);
}
// bmap[i] = j where b's point j takes a's scalar i (b's index map), else ~0
__global__ void k_bmap_scatter(const uint32_t* sidx, size_t nb_pts, uint32_t na, uint32_t* bmap) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < nb_pts && sidx[j] < na) bmap[sidx[j]] = (uint32_t)j;
}
void msm_build_bmap(const gg_msm_base* a, const gg_msm_base* b, DevBuf& bmap) {
    bmap.alloc(std::max<size_t>(a->n, 1) * 4);
    GG_HIP(hipMemset(bmap.p, 0xff, std::max<size_t>(a->n, 1) * 4));
    if (b->n) {
        hipLaunchKernelGGL(k_bmap_scatter, dim3(grid_for(b->n, 256)), dim3(256), 0, hipStreamPerThread,
                           b->sidx.as<uint32_t>(), b->n, (uint32_t)a->n, bmap.as<uint32_t>());
        GG_HIP(hipGetLastError());
    }
    GG_WAIT_STREAM(hipStreamPerThread);
}
bool msm_derivable(const gg_msm_base* a, const gg_msm_base* b) {
    if (a->c != b->c || a->W != b->W || a->G != b->G || a->has_sidx || !b->has_sidx) return false;
    for (int w = 0; w < a->W; w++)
        if (a->win.bits[w] != b->win.bits[w] || a->win.off[w] != b->win.off[w]) return false;
    return (double)a->W * (double)a->n < 4294967295.0;
}
MsmSort* msm_work_sort(MsmWork* w) { return &w->sort; }
MsmScratch* msm_work_scratch(MsmWork* w) { return &w->scr; }
// A batch's sort counts and positions nvec W n entries and numbers kp G 2^(c-1)
// buckets (kp = the power of two >= nvec) in 32-bit words whose bit 31 is a
// digit's sign and whose all-ones value means "no key" (W n alone is
// checked at base creation; a batch multiplies both).
bool msm_batch_fits(size_t n, int W, int c, int G, int nvec) {
    int kp = 1;
    while (kp < nvec) kp <<= 1;
    const double entries = (double)W * (double)n * (double)nvec;
    const double buckets = (double)G * std::ldexp(1.0, c - 1) * (double)kp;
    return entries + 64.0 < 4294967296.0 && buckets < 2147483648.0;
}
bool msm_base_batch_fits(const gg_msm_base* b, int nvec) { return msm_batch_fits(b->n, b->W, b->c, b->G, nvec); }
size_t msm_scalars_needed(gg_msm_base* b) {
    return b->has_sidx ? (b->n ? (size_t)b->max_sidx + 1 : 0) : b->n;
}
}  // namespace gg

extern "C" int gg_msm(gg_msm_base_t b, const void* scalars, size_t n_scalars, int scalars_on_device,
                      void* out_jac, void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(b && out_jac, GG_ERR_INVALID_ARG, "null argument");
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : hipStreamPerThread;
    size_t need = msm_scalars_needed(b);
    GG_CHECK(n_scalars >= need, GG_ERR_INVALID_ARG,
             "scalar vector shorter than the points/index map require");
    GG_CHECK(need == 0 || scalars, GG_ERR_INVALID_ARG, "null scalars");
    std::lock_guard<std::mutex> lk(b->mu);
    const Fr* sdev = (const Fr*)scalars;
    if (!scalars_on_device && need) {
        b->own.scr.scal.reserve(need * 32);
        GG_HIP(hipMemcpyAsync(b->own.scr.scal.p, scalars, need * 32, hipMemcpyHostToDevice, st));
        sdev = b->own.scr.scal.as<Fr>();
    }
    msm_device_locked(b, sdev, out_jac, st);
    GG_PROBE_GUARD();
    GG_CAPI_END
}

extern "C" int gg_msm_batch(gg_msm_base_t b, const void* const* scalars, int n_vectors, size_t n_scalars,
                            int scalars_on_device, void* const* out_jac, void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(b && scalars && out_jac, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(n_vectors >= 1 && n_vectors <= kMaxBatch, GG_ERR_INVALID_ARG, "n_vectors must be 1..4");
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : hipStreamPerThread;
    const size_t need = msm_scalars_needed(b);
    GG_CHECK(n_scalars >= need, GG_ERR_INVALID_ARG, "scalar vector shorter than the points/index map require");
    for (int v = 0; v < n_vectors; v++) {
        GG_CHECK(need == 0 || scalars[v], GG_ERR_INVALID_ARG, "null scalars");
        GG_CHECK(out_jac[v], GG_ERR_INVALID_ARG, "null out_jac");
    }
    GG_CHECK(msm_base_batch_fits(b, n_vectors), GG_ERR_UNSUPPORTED,
             "MSM batch too large for 32-bit sort indices (gg_msm_batch_shape); use one MSM per vector");
    std::lock_guard<std::mutex> lk(b->mu);
    const Fr* sdev[kMaxBatch] = {};
    if (!scalars_on_device && need) {
        b->own.scr.scal.reserve((size_t)n_vectors * need * 32);
        for (int v = 0; v < n_vectors; v++) {
            sdev[v] = b->own.scr.scal.as<Fr>() + (size_t)v * need;
            GG_HIP(hipMemcpyAsync((void*)sdev[v], scalars[v], need * 32, hipMemcpyHostToDevice, st));
        }
    } else {
        for (int v = 0; v < n_vectors; v++) sdev[v] = (const Fr*)scalars[v];
    }
    msm_device_work_batch(b, &b->own, sdev, n_vectors, out_jac, st);
    GG_PROBE_GUARD();
    GG_CAPI_END
}

extern "C" int gg_msm_stripe(gg_msm_base_t b, const void* scalars, size_t n_scalars, int scalars_on_device,
                             int stripe_log, int stripe_part, void* out_jac, void* hip_stream) {
    GG_CAPI_BEGIN
    GG_CHECK(b && out_jac, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(stripe_log >= 0 && stripe_log <= b->c - 2 && stripe_part >= 0 && stripe_part < (1 << stripe_log),
             GG_ERR_INVALID_ARG, "bucket stripe out of range (stripe_log <= window_bits - 2, part < 2^stripe_log)");
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : hipStreamPerThread;
    size_t need = msm_scalars_needed(b);
    GG_CHECK(n_scalars >= need, GG_ERR_INVALID_ARG,
             "scalar vector shorter than the points/index map require");
    GG_CHECK(need == 0 || scalars, GG_ERR_INVALID_ARG, "null scalars");
    std::lock_guard<std::mutex> lk(b->mu);
    const Fr* sdev = (const Fr*)scalars;
    if (!scalars_on_device && need) {
        b->own.scr.scal.reserve(need * 32);
        GG_HIP(hipMemcpyAsync(b->own.scr.scal.p, scalars, need * 32, hipMemcpyHostToDevice, st));
        sdev = b->own.scr.scal.as<Fr>();
    }
    if (b->n == 0) {  // the identity, in the group's Jacobian layout
        msm_device_work(b, &b->own, sdev, out_jac, st);
        return GG_OK;
    }
    msm_prepare_dev(b, &b->own.sort, sdev, st, stripe_log, (uint32_t)stripe_part);
    msm_finish_dev(b, &b->own.sort, out_jac, st, nullptr);
    GG_PROBE_GUARD();
    GG_CAPI_END
}

extern "C" int gg_msm_batch_shape(size_t n_points, int window_bits, int n_windows, int groups, int n_vectors) {
    GG_CAPI_BEGIN
    GG_CHECK(window_bits >= 2 && window_bits <= 30 && n_windows >= 1 && groups >= 1 && (groups & (groups - 1)) == 0,
             GG_ERR_INVALID_ARG, "window_bits 2..30, n_windows >= 1, groups a power of two");
    GG_CHECK(n_vectors >= 1 && n_vectors <= kMaxBatch, GG_ERR_INVALID_ARG, "n_vectors must be 1..4");
    GG_CHECK(msm_batch_fits(n_points, n_windows, window_bits, groups, n_vectors), GG_ERR_UNSUPPORTED,
             "MSM batch too large for 32-bit sort indices: n_vectors * n_windows * n_points entries must stay "
             "below 2^32 and n_vectors' bucket spaces below 2^31 buckets; use one MSM per vector");
    GG_CAPI_END
}
