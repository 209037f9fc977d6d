// BLS12-381 G2 instantiation of the bucket MSM: the B MSM of a BLS12-381
// Groth16 prove (backend/groth16/bls12-381/prove.go:280-301, G2Jac.MultiExp).
// Coordinates in Fp2 over the 12-limb Fp, scalars BLS12-381 fr.
#include "msm_impl.cuh"

namespace gg {
void create_base_bls2(gg_msm_base* b, const void* points, size_t n, int on_device,
                      const uint32_t* sidx, int window_bits, bool keep_inf, int groups) {
    create_base<Fp2Bls>(b, points, n, on_device, sidx, window_bits, keep_inf, 1, groups);
}
void msm_run_bls2(gg_msm_base* b, MsmWork* w, const Fr* scalars_dev, void* out_jac, hipStream_t st) {
    Jac<Fp2Bls> j = xyzz_to_jac(msm_run<Fp2Bls>(b, w, scalars_dev, st));
    memcpy(out_jac, &j, sizeof(j));
}
void msm_finish_bls2(gg_msm_base* b, MsmSort* s, MsmScratch* scr, void* out_jac, hipStream_t st) {
    Jac<Fp2Bls> j = xyzz_to_jac(msm_finish<Fp2Bls>(b, s, scr, st));
    memcpy(out_jac, &j, sizeof(j));
}
// a batch of nvec MSMs over b (msm_run_batch): out_jac[v] = the v-th result
void msm_run_batch_bls2(gg_msm_base* b, MsmWork* w, const VecPtrs& vp, int nvec, void* const* out_jac,
                        hipStream_t st) {
    Xyzz<Fp2Bls> r[kMaxBatch];
    msm_run_batch<Fp2Bls>(b, w, vp, nvec, st, r);
    for (int v = 0; v < nvec; v++) {
        Jac<Fp2Bls> j = xyzz_to_jac(r[v]);
        memcpy(out_jac[v], &j, sizeof(j));
    }
}
}  // namespace gg
