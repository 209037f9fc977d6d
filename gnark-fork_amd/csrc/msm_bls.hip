// BLS12-381 G1 instantiation of the bucket MSM (KZG commitments of the PlonK
// prover: backend/plonk/bls12-381/prove.go:336, 494, 769, 1165-1169, 1203-1213).
// Coordinates in the 12-limb Fp (R = 2^384), scalars BLS12-381 fr (255-bit).
#include "msm_impl.cuh"

namespace gg {
void create_base_bls(gg_msm_base* b, const void* points, size_t n, int on_device,
                     const uint32_t* sidx, int window_bits, bool keep_inf, int groups) {
    create_base<FpBls>(b, points, n, on_device, sidx, window_bits, keep_inf, 1, groups);
}
void msm_run_bls(gg_msm_base* b, MsmWork* w, const Fr* scalars_dev, void* out_jac, hipStream_t st) {
    Jac<FpBls> j = xyzz_to_jac(msm_run<FpBls>(b, w, scalars_dev, st));
    memcpy(out_jac, &j, sizeof(j));
}
void msm_finish_bls(gg_msm_base* b, MsmSort* s, MsmScratch* scr, void* out_jac, hipStream_t st) {
    Jac<FpBls> j = xyzz_to_jac(msm_finish<FpBls>(b, s, scr, st));
    memcpy(out_jac, &j, sizeof(j));
}
// a batch of nvec MSMs over b (msm_run_batch): out_jac[v] = the v-th result
void msm_run_batch_bls(gg_msm_base* b, MsmWork* w, const VecPtrs& vp, int nvec, void* const* out_jac,
                        hipStream_t st) {
    Xyzz<FpBls> r[kMaxBatch];
    msm_run_batch<FpBls>(b, w, vp, nvec, st, r);
    for (int v = 0; v < nvec; v++) {
        Jac<FpBls> j = xyzz_to_jac(r[v]);
        memcpy(out_jac[v], &j, sizeof(j));
    }
}
}  // namespace gg
