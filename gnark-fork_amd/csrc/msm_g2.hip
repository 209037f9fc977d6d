// G2 instantiation of the bucket MSM (separate TU for build parallelism).
#include "msm_impl.cuh"

namespace gg {
void create_base_g2(gg_msm_base* b, const void* points, size_t n, int on_device,
                    const uint32_t* sidx, int window_bits, bool keep_inf, int groups) {
    create_base<Fp2>(b, points, n, on_device, sidx, window_bits, keep_inf, 0, groups);
}
void msm_run_g2(gg_msm_base* b, MsmWork* w, const Fr* scalars_dev, void* out_jac, hipStream_t st) {
    G2Jac j = xyzz_to_jac(msm_run<Fp2>(b, w, scalars_dev, st));
    memcpy(out_jac, &j, sizeof(j));
}
void msm_finish_g2(gg_msm_base* b, MsmSort* s, MsmScratch* scr, void* out_jac, hipStream_t st) {
    G2Jac j = xyzz_to_jac(msm_finish<Fp2>(b, s, scr, st));
    memcpy(out_jac, &j, sizeof(j));
}
// a batch of nvec MSMs over b (msm_run_batch): out_jac[v] = the v-th result
void msm_run_batch_g2(gg_msm_base* b, MsmWork* w, const VecPtrs& vp, int nvec, void* const* out_jac,
                        hipStream_t st) {
    Xyzz<Fp2> r[kMaxBatch];
    msm_run_batch<Fp2>(b, w, vp, nvec, st, r);
    for (int v = 0; v < nvec; v++) {
        G2Jac j = xyzz_to_jac(r[v]);
        memcpy(out_jac[v], &j, sizeof(j));
    }
}
}  // namespace gg
