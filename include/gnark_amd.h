/*
 * gnark_amd.h -- C ABI of the MI355X-native (gfx950) proving backend for gnark.
 *
 * This is the drop-in boundary that replaces the iciclegnark cgo calls made by
 * gnark's `icicle` build-tag path (backend/groth16/bn254/icicle/icicle.go) and
 * the gnark-crypto CPU kernels on the Groth16 hot path
 * (backend/groth16/bn254/prove.go:127-396).  A Go binding (cgo) is shown in
 * INTEGRATION.md; Python tests/bench bind it with ctypes.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Every field element / point buffer uses
 *    gnark-crypto's in-memory layout: Montgomery form (R = 2^256), [4]uint64
 *    little-endian limbs.  fr.Element = 32 B, G1Affine = 64 B {X,Y},
 *    G2Affine = 128 B {X.A0,X.A1,Y.A0,Y.A1}, G1Jac = 96 B, G2Jac = 192 B.
 *    Affine infinity is all-zero (as gnark's G1Affine zero value).
 *  - Host buffers are borrowed for the duration of a call only (cgo rule).
 *  - Every function returns 0 (GG_OK) on success or a GG_ERR_* code; the
 *    message of the last failure on the calling thread is gg_last_error().
 *  - Thread-safe: objects may be used from several host threads; each call
 *    uses its own HIP stream unless one is passed explicitly.
 */
#ifndef GNARK_AMD_H
#define GNARK_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GG_OK 0
#define GG_ERR_INVALID_ARG 1
#define GG_ERR_DEVICE 2
#define GG_ERR_OOM 3
#define GG_ERR_UNSUPPORTED 4
#define GG_ERR_INTERNAL 5
#define GG_ERR_UNSATISFIED 6 /* R1CS solver: a constraint is not satisfied */
/* a multi-GPU prove ran as a timing rehearsal (gg_groth16_mpk_set_rehearsal,
 * gg_plonk_pk_set_rehearsal): the proof written is NOT valid.  Never GG_OK, so
 * a caller checking for success cannot pass such a proof on. */
#define GG_REHEARSAL 7
/* a host wait of the library (for GPU work, or for another part / shard of a
 * multi-GPU proof) passed its deadline (gg_set_wait_timeout); gg_last_error()
 * names the part, the stage and what was awaited.  The work it waited for may
 * still be in flight on the GPU: release the key (or end the process) rather
 * than proving with it again. */
#define GG_ERR_TIMEOUT 8
/* gg_build_flags() bits: a diagnostic build whose MSM sums are wrong by design
 * (traffic attribution, never shipped); its provers return GG_REHEARSAL */
#define GG_BUILD_ACCUM_PROBE 1

#define GG_G1 1
#define GG_G2 2
/* BLS12-381 G1 (PlonK KZG commitments): affine 96 B (12-limb fp, R = 2^384),
 * Jacobian 144 B, scalars BLS12-381 fr (32 B Montgomery) */
#define GG_BLS12_381_G1 3
/* BLS12-381 G2 (BLS12-381 Groth16 B MSM): affine 192 B ({X.A0, X.A1, Y.A0, Y.A1},
 * 12-limb fp each), Jacobian 288 B, scalars BLS12-381 fr */
#define GG_BLS12_381_G2 4

/* curves of a domain (scalar field of the NTT) */
#define GG_CURVE_BN254 0
#define GG_CURVE_BLS12_381 1

/* decimation (gnark-crypto fft.DIF / fft.DIT) */
#define GG_DIF 0
#define GG_DIT 1

typedef struct gg_domain *gg_domain_t;
typedef struct gg_msm_base *gg_msm_base_t;
typedef struct gg_groth16_pk *gg_groth16_pk_t;
typedef struct gg_hshard *gg_hshard_t;
typedef struct gg_plonk_pk *gg_plonk_pk_t;
/* One-shot hash for Fiat-Shamir transcripts: out[0..*out_len) = H(data[0..len)),
 * *out_len = capacity of out on entry (128 B), digest length on return; 0 = ok.
 * A Go caller wraps its hash.Hash (Reset, Write, Sum).  NULL = SHA-256, gnark's
 * default ChallengeHash / KZGFoldingHash (backend/backend.go:74-75). */
typedef int (*gg_hash_fn)(void *ctx, const void *data, size_t len, void *out, size_t *out_len);
/* All-to-all exchange supplied by the caller's transport (RCCL over xGMI via
 * torch.distributed, or a Go RCCL binding): chunk r (bytes_per_rank bytes) of
 * send_dev goes to rank r, chunk k of recv_dev comes from rank k.  Device
 * buffers; must not return before recv_dev holds the data.  0 = success. */
typedef int (*gg_exchange_fn)(void *ctx, const void *send_dev, void *recv_dev,
                              size_t bytes_per_rank);

/* ---------------------------------------------------------------- runtime */
const char *gg_last_error(void);
int gg_version(void);
/* GG_BUILD_* bits of this library build (0 for the product library) */
int gg_build_flags(void);
int gg_device_count(int *count);
/* binds the calling host thread to a GPU (one process per GPU is the norm) */
int gg_set_device(int device);

/* ----------------------------------------------------------- device memory
 * Replaces iciclegnark.CopyToDevice / FreeDevicePointer
 * (icicle.go:44-47, 245, 269, 352, 356, 416-418, 478-480, 505-507). */
int gg_malloc(void **dev_ptr, size_t bytes);
int gg_free(void *dev_ptr);
int gg_copy_to_device(void *dev_dst, const void *host_src, size_t bytes);
int gg_copy_to_host(void *host_dst, const void *dev_src, size_t bytes);
int gg_copy_device(void *dev_dst, const void *dev_src, size_t bytes);
int gg_memset_device(void *dev_dst, int value, size_t bytes);
int gg_synchronize(void);

/* ------------------------------------------------------------- NTT domain
 * Replaces iciclegnark.GenerateTwiddleFactors + the CosetTable/CosetTableInv/
 * den uploads (icicle.go:44-76).  omega and coset_gen are taken from gnark's
 * pk.Domain (Generator, FrMultiplicativeGen) so no roots are hard-coded:
 * omega_mont: primitive 2^log_n-th root of unity (fr, Montgomery);
 * coset_gen_mont: coset shift g (fr, Montgomery). */
int gg_domain_create(int log_n, const void *omega_mont, const void *coset_gen_mont,
                     gg_domain_t *out);
/* Same for a chosen scalar field: GG_CURVE_BN254 (= gg_domain_create) or
 * GG_CURVE_BLS12_381 -- the PlonK prover's pk.Domain[0] / Domain[1] FFTs
 * (backend/plonk/bls12-381/prove.go:995-1061, 1223-1276; fr 32 B Montgomery). */
int gg_domain_create_ex(int curve, int log_n, const void *omega_mont, const void *coset_gen_mont,
                        gg_domain_t *out);
int gg_domain_release(gg_domain_t d);
int gg_domain_log_n(gg_domain_t d, int *log_n);

/* In-place transform of 2^log_n device fr elements with gnark-crypto
 * semantics (replaces INttOnDevice / NttOnDevice / ReverseScalars,
 * icicle.go:489-510, and domain.FFT / domain.FFTInverse, prove.go:369-393):
 *   inverse = 0: domain.FFT(a, decimation, [OnCoset()])
 *   inverse = 1: domain.FFTInverse(a, decimation, [OnCoset()])
 * DIF: natural -> bit-reversed; DIT: bit-reversed -> natural. */
int gg_ntt(gg_domain_t d, void *data_dev, int inverse, int decimation, int coset,
           void *hip_stream);

/* Fused Groth16 computeH (prove.go:353-396; icicle.go:453-513):
 *   h = FFTInverse_coset_DIF( (FFT_coset_DIT(iFFT_DIF(a)) o ... b) - ...c ) / (g^n - 1)
 * a, b, c: `len` <= 2^log_n fr elements (zero-padded to 2^log_n), host or
 * device memory per inputs_on_device.  h_dev: device buffer of 2^log_n fr;
 * h comes out in bit-reversed order, the order pk.G1.Z is stored in
 * (setup.go:265), so it feeds the Z-MSM directly. */
int gg_groth16_compute_h(gg_domain_t d, const void *a, const void *b, const void *c, size_t len,
                         int inputs_on_device, void *h_dev, void *hip_stream);

/* --------------------------------------------------------- MSM point bases
 * Replaces iciclegnark.CopyPointsToDevice / CopyG2PointsToDevice
 * (icicle.go:88-126).  Points stay resident in HBM together with the
 * window-shifted copies 2^(c*w) * P_i that the bucket MSM uses, so every
 * window shares one bucket set (fixed-base precomputation sized for 288 GB).
 * group: GG_G1 or GG_G2 (BN254), GG_BLS12_381_G2 (BLS12-381 Groth16), GG_BLS12_381_G1 (PlonK KZG commitments:
 *   kzg.Commit / MultiExp at backend/plonk/bls12-381/prove.go:336, 494, 769,
 *   1165-1169, 1203-1213).  points: n affine points (host or device memory).
 * Infinity points are dropped at upload (fixes the index shift of
 * icicle.go:343-347).
 * scalar_index (nullable, host): scalar of point i is scalars[scalar_index[i]]
 *   in gg_msm -- this expresses gnark's wire filtering (prove.go:151-175,
 *   filterHeap prove.go:328-351) without copying the witness.
 * window_bits: 0 = automatic. */
int gg_msm_base_create(int group, const void *points, size_t n, int points_on_device,
                       const uint32_t *scalar_index, int window_bits, gg_msm_base_t *out);
int gg_msm_base_release(gg_msm_base_t b);
/* number of resident (non-infinity) points, and window size actually used */
int gg_msm_base_info(gg_msm_base_t b, size_t *n_points, int *window_bits, int *n_windows);
/* memory layout of the precomputed table: every `groups`-th window shift is
 * stored (stored_windows copies of the points, table_bytes of HBM); groups > 1
 * trades HBM for more buckets.  Chosen at creation from the free HBM (and the
 * gg_set_hbm_budget cap; GG_MSM_GROUPS=1|2|4|8|16 forces it) */
int gg_msm_base_layout(gg_msm_base_t b, int *groups, int *stored_windows, size_t *table_bytes);
/* process-wide cap (bytes, per device) on what new precomputed tables may
 * take beside the scratch their proofs need; 0 = the free HBM less a reserve
 * (gnark sizes nothing like this: its keys live in host memory, setup.go:111) */
int gg_set_hbm_budget(size_t bytes);
/* Deadline (seconds) of every host wait inside the library: a stream / event
 * wait, a wait for a peer part's thread, the one-process exchange barrier.
 * 0 = GG_WAIT_TIMEOUT_S from the environment, else 300 s.  A wait past it
 * returns GG_ERR_TIMEOUT instead of blocking (gnark's provers end a proof at
 * the first failing task: prove.go:198-209 channels, plonk prove.go:132-173
 * errgroup; a hang ends nothing). */
int gg_set_wait_timeout(double seconds);
/* Destroys the dedicated hardware queues (CU-masked streams: at most
 * GG_TASK_QUEUES per device, lent to the keys' prove tasks) that no live key
 * holds.  The library does this itself when a device's last key is released;
 * call it before process exit if keys may still be alive then (the Python
 * mirror does, atexit), so no stream is left for the runtime's own teardown. */
int gg_release_task_queues(void);
double gg_get_wait_timeout(void);
/* Host-only self-test of the bounded wait (no GPU needed): `parties` threads
 * meet at a barrier, `arriving` of them come; GG_OK if all arrive, else every
 * waiter returns GG_ERR_TIMEOUT after timeout_s (the message names the wait). */
int gg_wait_selftest(int parties, int arriving, double timeout_s);
/* The same deadline on a real stream: one wave sleeps `sleeps` x ~3.4 us on the
 * calling thread's stream and the library's bounded stream wait waits for it
 * under timeout_s: GG_ERR_TIMEOUT (message names the wait) if it was still
 * running, else GG_OK.  The wave always drains before the call returns. */
int gg_wait_selftest_device(uint32_t sleeps, double timeout_s);
/* Host-only self-test of the library's kept worker threads (no GPU needed): n
 * tasks that all meet at one barrier (so the worker set must grow to n), the
 * last failing after it; GG_OK if all ran and the failure came back to the
 * waiter, a dropped deferred task never ran and a waited one ran once. */
int gg_task_selftest(int n);
size_t gg_get_hbm_budget(void);

/* out = sum_i scalars[idx(i)] * P_i as a Jacobian point (gnark G1Jac/G2Jac
 * layout, Montgomery).  Replaces MsmOnDevice / MsmG2OnDevice
 * (icicle.go:302-382) and G1Jac/G2Jac.MultiExp (prove.go:201-290).
 * scalars: fr Montgomery (host or device per scalars_on_device);
 * n_scalars: length of the scalar vector (must cover every referenced index).
 * hip_stream may be NULL. */
int gg_msm(gg_msm_base_t b, const void *scalars, size_t n_scalars, int scalars_on_device,
           void *out_jac, void *hip_stream);
/* n_vectors (1..4) MSMs over the same base as one: out_jac[v] = sum_i
 * scalars[v][idx(i)] * P_i, with one sort, one accumulation launch, one level 2
 * and one bucket reduction for all of them (the vectors' buckets are disjoint
 * groups of one bucket space).  Replaces the same-base kzg.Commit calls of
 * commitToLRO (backend/plonk/bls12-381/prove.go:425-502: L, R, O on
 * pk.KzgLagrange) and commitToQuotient (:1199-1218: h1, h2, h3 on pk.Kzg).
 * Arguments as gg_msm's, one scalar vector and one output per v. */
int gg_msm_batch(gg_msm_base_t b, const void *const *scalars, int n_vectors, size_t n_scalars,
                 int scalars_on_device, void *const *out_jac, void *hip_stream);
/* GG_OK if a batch of n_vectors over a base of n_points points, n_windows
 * windows of window_bits bits and `groups` precompute groups (gg_msm_base_layout)
 * fits the batched sort's 32-bit entry positions and bucket ids, else
 * GG_ERR_UNSUPPORTED: gg_msm_batch refuses such a batch (one gg_msm per vector
 * instead; the PlonK prover falls back to that by itself).  Host only. */
int gg_msm_batch_shape(size_t n_points, int window_bits, int n_windows, int groups, int n_vectors);
/* One bucket stripe of gg_msm: with N = 2^stripe_log, the part of the MSM whose
 * signed-digit buckets b (|digit| - 1, every window) satisfy b mod N ==
 * stripe_part, i.e. sum over those buckets of (b + 1) S_b.  The N stripes'
 * results add up to gg_msm's.  This is how one MSM splits over N GPUs that each
 * hold the whole base (MI355X: 288 GB of HBM per GPU): every GPU reads all
 * scalars but sorts, accumulates and reduces only 1/N of the entries and
 * buckets -- unlike a split by points, whose every part pays the whole bucket
 * reduction.  Replaces the point-sharded MultiExp of a multi-GPU prover
 * (prove.go:201-290 on one node's GPUs).  stripe_log <= window_bits - 2. */
int gg_msm_stripe(gg_msm_base_t b, const void *scalars, size_t n_scalars, int scalars_on_device,
                  int stripe_log, int stripe_part, void *out_jac, void *hip_stream);

/* host-side point helpers (epilogue of prove.go:206-299) */
int gg_g1_jac_to_affine(const void *jac, void *aff);
int gg_g2_jac_to_affine(const void *jac, void *aff);
int gg_g1_jac_add(const void *a_jac, const void *b_jac, void *out_jac);
int gg_g2_jac_add(const void *a_jac, const void *b_jac, void *out_jac);
/* out = k * p, k fr Montgomery, p affine */
int gg_g1_scalar_mul(const void *p_aff, const void *k_mont, void *out_jac);
int gg_g2_scalar_mul(const void *p_aff, const void *k_mont, void *out_jac);
/* BLS12-381 G1 (curve.G1Jac.FromJacobian / AddAssign of gnark-crypto bls12-381) */
int gg_bls12_381_g1_jac_to_affine(const void *jac, void *aff);
int gg_bls12_381_g1_jac_add(const void *a_jac, const void *b_jac, void *out_jac);
/* out (Jacobian) = k * p, p affine, k bls12-381 fr Montgomery (host; KZG digest folding) */
int gg_bls12_381_g1_scalar_mul(const void *p_aff, const void *k_mont, void *out_jac);
/* BLS12-381 G2 (G2Jac.FromJacobian / AddAssign / ScalarMultiplication, BLS12-381 Groth16 epilogue) */
int gg_bls12_381_g2_jac_to_affine(const void *jac, void *aff);
int gg_bls12_381_g2_jac_add(const void *a_jac, const void *b_jac, void *out_jac);
int gg_bls12_381_g2_scalar_mul(const void *p_aff, const void *k_mont, void *out_jac);

/* Fixed-base batch scalar multiplication out[i] = k_i * base (affine,
 * infinity for k_i = 0): replaces curve.BatchScalarMultiplicationG1/G2
 * (setup.go:240-251, 306-318; prove.go:192).  Used to build proving keys on
 * the GPU.  group: GG_G1, GG_G2 or GG_BLS12_381_G1 (scalars of that curve's
 * fr).  scalars: n fr Montgomery; out: n affine points. */
int gg_batch_scalar_mul(int group, const void *base_aff, const void *scalars, size_t n,
                        int scalars_on_device, void *out_aff, int out_on_device);

/* ------------------------------------------------------------ Groth16 BN254
 * Device-resident proving key: replaces setupDevicePointers (icicle.go:31-130)
 * and holds the pk.G1/G2 arrays (setup.go:35-58).
 *   log_n, omega, coset_gen : pk.Domain
 *   g1_A[nA], g1_B[nB], g1_Z[nZ = 2^log_n - 1], g1_K[nK] : pk.G1.{A,B,Z,K}
 *   alpha1, beta1, delta1 : pk.G1.{Alpha,Beta,Delta};  g2_B[nB], beta2, delta2
 *   inf_A, inf_B : pk.InfinityA/B (n_wires bytes, 1 = infinity)
 *   nb_public : r1cs.GetNbPublicVariables()
 *   k_wire_index (nullable): wire index of the scalar for each pk.G1.K point,
 *     i.e. the filterHeap result (prove.go:238-248); NULL = nb_public + i. */
int gg_groth16_pk_create(int log_n, const void *omega_mont, const void *coset_gen_mont,
                         const void *g1_A, size_t nA, const void *g1_B, size_t nB,
                         const void *g1_Z, size_t nZ, const void *g1_K, size_t nK,
                         const void *alpha1, const void *beta1, const void *delta1,
                         const void *g2_B, const void *beta2, const void *delta2,
                         const uint8_t *inf_A, const uint8_t *inf_B, size_t n_wires,
                         size_t nb_public, const uint32_t *k_wire_index, gg_groth16_pk_t *out);
/* Same for a chosen curve: GG_CURVE_BN254 (= gg_groth16_pk_create) or
 * GG_CURVE_BLS12_381 (backend/groth16/bls12-381: the same prover over
 * BLS12-381; points in that curve's layout: G1 affine 96 B, G2 affine 192 B,
 * fr 32 B).  Output points of gg_groth16_prove then have those sizes too. */
int gg_groth16_pk_create_ex(int curve, int log_n, const void *omega_mont, const void *coset_gen_mont,
                            const void *g1_A, size_t nA, const void *g1_B, size_t nB,
                            const void *g1_Z, size_t nZ, const void *g1_K, size_t nK,
                            const void *alpha1, const void *beta1, const void *delta1,
                            const void *g2_B, const void *beta2, const void *delta2,
                            const uint8_t *inf_A, const uint8_t *inf_B, size_t n_wires,
                            size_t nb_public, const uint32_t *k_wire_index, gg_groth16_pk_t *out);
int gg_groth16_pk_release(gg_groth16_pk_t pk);
/* resident MSM base `which` of a key (0 = G1.A, 1 = G1.B, 2 = G1.K, 3 = G1.Z,
 * 4 = G2.B): as gg_msm_base_info */
int gg_groth16_pk_base_info(gg_groth16_pk_t pk, int which, size_t *n_points, int *window_bits,
                            int *n_windows);
/* as gg_msm_base_layout for base `which` of the key (one groups value per key) */
int gg_groth16_pk_base_layout(gg_groth16_pk_t pk, int which, int *groups, int *stored_windows,
                              size_t *table_bytes);

/* Groth16 Prove after Solve (prove.go:127-320; icicle.go:198-420):
 *   wires[n_wires] = solution.W; sol_a/b/c[n_cons] = solution.A/B/C
 *   (host or device memory per inputs_on_device)
 *   r_mont, s_mont: the proof randomness (prove.go:177-189 samples it with
 *   SetRandom; the caller passes it so tests can pin it).
 * Outputs (host): Ar (G1Affine 64 B), Bs (G2Affine 128 B), Krs (G1Affine 64 B);
 * h_dev_out (nullable): device buffer of 2^log_n fr receiving h (bit-reversed). */
int gg_groth16_prove(gg_groth16_pk_t pk, const void *wires, size_t n_wires, const void *sol_a,
                     const void *sol_b, const void *sol_c, size_t n_cons, int inputs_on_device,
                     const void *r_mont, const void *s_mont, void *ar_aff, void *bs_aff,
                     void *krs_aff, void *h_dev_out);

/* ---- multi-GPU Groth16: one key shard per GPU.
 * A shard owns wires [wire_lo, wire_hi) of pk.G1.A / G1.B / G1.K / G2.B and
 * positions [z_lo, z_lo + nZ) of pk.G1.Z (bit-reversed order, setup.go:265).
 * The point arguments are the shard's slices of the key arrays, in key order:
 * g1_A = the non-infinity A points of the shard's wires (inf_A/inf_B are the
 * full n_wires masks), g1_B / g2_B likewise, g1_K = the K points whose wires
 * lie in the shard; k_wire_index (nullable) their absolute wire ids, NULL =
 * max(wire_lo, nb_public) + j.  The shards of a key partition it; every GPU
 * holds the domain and computes h itself (no exchange on the H path). */
int gg_groth16_pk_create_shard(int log_n, const void *omega_mont, const void *coset_gen_mont,
                               const void *g1_A, size_t nA, const void *g1_B, size_t nB,
                               const void *g1_Z, size_t z_lo, size_t nZ, const void *g1_K,
                               size_t nK, const void *alpha1, const void *beta1,
                               const void *delta1, const void *g2_B, const void *beta2,
                               const void *delta2, const uint8_t *inf_A, const uint8_t *inf_B,
                               size_t n_wires, size_t nb_public, const uint32_t *k_wire_index,
                               size_t wire_lo, size_t wire_hi, gg_groth16_pk_t *out);
/* gg_groth16_pk_create_shard for a chosen curve (GG_CURVE_BN254 or
 * GG_CURVE_BLS12_381: backend/groth16/bls12-381/prove.go:63-322, points in that
 * curve's layout); a BLS12-381 shard computes h itself (no distributed computeH). */
int gg_groth16_pk_create_shard_ex(int curve, int log_n, const void *omega_mont, const void *coset_gen_mont,
                                  const void *g1_A, size_t nA, const void *g1_B, size_t nB,
                                  const void *g1_Z, size_t z_lo, size_t nZ, const void *g1_K,
                                  size_t nK, const void *alpha1, const void *beta1,
                                  const void *delta1, const void *g2_B, const void *beta2,
                                  const void *delta2, const uint8_t *inf_A, const uint8_t *inf_B,
                                  size_t n_wires, size_t nb_public, const uint32_t *k_wire_index,
                                  size_t wire_lo, size_t wire_hi, gg_groth16_pk_t *out);
/* Bucket-stripe shard of a multi-GPU key: the WHOLE A, B, K and
 * G2 B tables (arguments as gg_groth16_pk_create_ex) and Z positions
 * [z_lo, z_lo + nZ); its A, B1, K and G2 MSMs take the bucket stripe
 * stripe_part of 2^stripe_log (gg_msm_stripe).  Shard r of N = 2^stripe_log
 * takes stripe r and the Z slice the distributed computeH leaves on rank r;
 * gg_groth16_prove_partial(_dist) over the whole solution, partials added as
 * for wire shards.  The per-GPU MSM work is 1/N of the whole key's with no
 * per-shard bucket reduction of the full bucket space. */
int gg_groth16_pk_create_stripe_ex(int curve, int log_n, const void *omega_mont, const void *coset_gen_mont,
                                   const void *g1_A, size_t nA, const void *g1_B, size_t nB,
                                   const void *g1_Z, size_t z_lo, size_t nZ, const void *g1_K,
                                   size_t nK, const void *alpha1, const void *beta1,
                                   const void *delta1, const void *g2_B, const void *beta2,
                                   const void *delta2, const uint8_t *inf_A, const uint8_t *inf_B,
                                   size_t n_wires, size_t nb_public, const uint32_t *k_wire_index,
                                   int stripe_log, int stripe_part, gg_groth16_pk_t *out);
/* stripe of a key: 0 / 0 for a whole key or a wire shard */
int gg_groth16_pk_stripe(gg_groth16_pk_t pk, int *stripe_log, int *stripe_part);
/* Device section of Prove on one key (shard): computeH and the five MSMs of
 * prove.go:198-301 without the combination.  Inputs as gg_groth16_prove (the
 * whole solution).  partials (host, 576 B): G1Jac sum w.A | sum w.B1 |
 * sum w.K | sum h.Z (96 B each) then G2Jac sum w.B2 (192 B).  The partials of
 * all shards are added (gg_g1_jac_add / gg_g2_jac_add, e.g. after an RCCL
 * all-gather) and handed to gg_groth16_finalize. */
int gg_groth16_prove_partial(gg_groth16_pk_t pk, const void *wires, size_t n_wires,
                             const void *sol_a, const void *sol_b, const void *sol_c,
                             size_t n_cons, int inputs_on_device, void *partials,
                             void *h_dev_out);
/* Host-only combination of summed partials into the proof (prove.go:177-299):
 * Ar = A + alpha + r.delta; Bs1 = B1 + beta + s.delta;
 * Krs = K + kr.delta + Z + s.Ar + r.Bs1 (kr = -rs); Bs = B2 + s.delta2 + beta2. */
int gg_groth16_finalize(const void *alpha1, const void *beta1, const void *delta1,
                        const void *beta2, const void *delta2, const void *partials,
                        const void *r_mont, const void *s_mont, void *ar_aff, void *bs_aff,
                        void *krs_aff);
/* gg_groth16_finalize for a chosen curve (BLS12-381 partials: 4 x 144 + 288 B) */
int gg_groth16_finalize_ex(int curve, const void *alpha1, const void *beta1, const void *delta1,
                           const void *beta2, const void *delta2, const void *partials,
                           const void *r_mont, const void *s_mont, void *ar_aff, void *bs_aff,
                           void *krs_aff);
/* gg_groth16_finalize in two halves, so the fixed-point terms of
 * prove.go:177-192, 293-296 (r.delta, s.delta, kr.delta, s.delta2: host scalar
 * multiplications independent of the MSMs) run on host threads while a
 * sharded prove's GPU work and partial exchange are in flight.  begin starts
 * them; end waits for them, combines them with the summed partials
 * (prove.go:206-299) and releases the handle.  end with partials == NULL only
 * releases it (a prove that failed). */
typedef struct gg_g16_fixed *gg_g16_fixed_t;
int gg_groth16_finalize_begin(int curve, const void *delta1, const void *delta2, const void *r_mont,
                              const void *s_mont, gg_g16_fixed_t *out);
int gg_groth16_finalize_end(gg_g16_fixed_t h, const void *alpha1, const void *beta1,
                            const void *beta2, const void *partials, void *ar_aff, void *bs_aff,
                            void *krs_aff);

/* ---- distributed computeH ("four-step multi-GPU NTT";
 * computeH of groth16/bn254/prove.go:353-396 and groth16/bls12-381/prove.go:353-396).
 * n = 2^log_n = m * world (world a power of two <= 16, n >= world^2).  Rank r
 * computes the local transforms of the cyclic slices x[r + world*j] and, after
 * three all-to-alls, holds h_bitrev[r*m, (r+1)*m): exactly the Z positions of
 * its key shard (gg_groth16_pk_create_shard with z_lo = r*m).
 * gg_hshard_create = gg_hshard_create_ex(GG_CURVE_BN254, ...); _ex takes the
 * curve whose fr the vectors hold (BN254 or BLS12-381).
 * gg_hshard_info: m and the size of the send / recv device buffers the caller
 * provides (bytes, all ranks' chunks: the largest exchange).
 * gg_hshard_exchange_bytes: bytes per rank pair of the all-to-all that follows
 * phase `phase` (1: a, b, c = 3 m/world^2 fr; 2: a, b = 2; 3: the product = 1).
 * gg_hshard_phase (the building blocks, synchronous on hip_stream):
 *   1: a, b, c (len <= n, full vectors, host or device per inputs_on_device)
 *      -> send;   2: recv -> send;   3: recv -> send;   4: recv -> h (m fr)
 * with an all-to-all send -> recv between consecutive phases.  State carried
 * between calls: phase 2 leaves den * c's coefficients in the handle and
 * phase 4 subtracts them (h = den coset_iFFT(a b) - den c, by linearity), so
 * the phases of one proof run in order 1, 2, 3, 4 on one handle, one proof at
 * a time; a phase out of that order fails (GG_ERR_INVALID_ARG) instead of
 * returning a wrong h (phase 1 may always start a new proof). */
int gg_hshard_create(int log_n, const void *omega_mont, const void *coset_gen_mont, int rank,
                     int world, gg_hshard_t *out);
int gg_hshard_create_ex(int curve, int log_n, const void *omega_mont, const void *coset_gen_mont,
                        int rank, int world, gg_hshard_t *out);
int gg_hshard_release(gg_hshard_t hs);
int gg_hshard_info(gg_hshard_t hs, size_t *m, size_t *exchange_bytes);
int gg_hshard_exchange_bytes(gg_hshard_t hs, int phase, size_t *bytes_per_rank);
int gg_hshard_phase(gg_hshard_t hs, int phase, const void *a, const void *b, const void *c,
                    size_t len, int inputs_on_device, const void *recv, void *send_or_h,
                    void *hip_stream);
/* gg_groth16_prove_partial with the distributed computeH: the H task runs the
 * four phases on this rank, calling xchg(ctx, send_dev, recv_dev, bytes) for
 * the three exchanges while the A/B1/K/G2 MSMs run on other streams; the
 * Z-MSM then uses the local h block.  pk must be the shard with wires of this
 * rank and z_lo = rank*m.  send_dev / recv_dev: gg_hshard_info bytes each. */
int gg_groth16_prove_partial_dist(gg_groth16_pk_t pk, gg_hshard_t hs, const void *wires,
                                  size_t n_wires, const void *sol_a, const void *sol_b,
                                  const void *sol_c, size_t n_cons, int inputs_on_device,
                                  gg_exchange_fn xchg, void *xchg_ctx, void *send_dev,
                                  void *recv_dev, void *partials);

/* ---- one-process multi-GPU Groth16 (SURVEY 8(b) gg_init(ngpu) shape, 8(e)):
 * the caller passes the WHOLE key (arguments as gg_groth16_pk_create) and
 * `world` device ids; shard r (wires [n_wires r/world, n_wires (r+1)/world),
 * Z positions of the distributed computeH) is placed on devices[r].  A proof
 * runs one host thread per shard; the three all-to-alls of the distributed
 * computeH are peer copies between the shards' device buffers (xGMI DMA), done
 * inside the library -- no transport from the caller.  world a power of two
 * <= 16 with n >= world^2 distributes computeH; otherwise every shard computes
 * h itself.  devices may repeat (several shards per GPU).  BN254 (or either
 * curve through _ex); host inputs (gg_groth16_mpk_prove_ex also takes
 * per-device resident solutions).
 * replaces: the per-GPU setupDevicePointers + Prove of icicle.go:31-420 for a
 * node of GPUs driven from one Go process. */
typedef struct gg_groth16_mpk *gg_groth16_mpk_t;
int gg_groth16_mpk_create(int log_n, const void *omega_mont, const void *coset_gen_mont,
                          const void *g1_A, size_t nA, const void *g1_B, size_t nB,
                          const void *g1_Z, size_t nZ, const void *g1_K, size_t nK,
                          const void *alpha1, const void *beta1, const void *delta1,
                          const void *g2_B, const void *beta2, const void *delta2,
                          const uint8_t *inf_A, const uint8_t *inf_B, size_t n_wires,
                          size_t nb_public, const uint32_t *k_wire_index, int world,
                          const int *devices, gg_groth16_mpk_t *out);
/* the same for a chosen curve: GG_CURVE_BN254 (= gg_groth16_mpk_create) or
 * GG_CURVE_BLS12_381 (backend/groth16/bls12-381/prove.go:63-322; points in that
 * curve's layout; computeH distributed over the shards as for BN254) */
int gg_groth16_mpk_create_ex(int curve, int log_n, const void *omega_mont, const void *coset_gen_mont,
                             const void *g1_A, size_t nA, const void *g1_B, size_t nB,
                             const void *g1_Z, size_t nZ, const void *g1_K, size_t nK,
                             const void *alpha1, const void *beta1, const void *delta1,
                             const void *g2_B, const void *beta2, const void *delta2,
                             const uint8_t *inf_A, const uint8_t *inf_B, size_t n_wires,
                             size_t nb_public, const uint32_t *k_wire_index, int world,
                             const int *devices, gg_groth16_mpk_t *out);
int gg_groth16_mpk_release(gg_groth16_mpk_t mpk);
/* gg_groth16_pk_base_info of shard `shard` */
int gg_groth16_mpk_base_info(gg_groth16_mpk_t mpk, int shard, int which, size_t *n_points,
                             int *window_bits, int *n_windows);
/* the device id of every shard (devices[0..world)) */
int gg_groth16_mpk_devices(gg_groth16_mpk_t mpk, int *devices, int cap);
/* world and whether computeH is distributed (1) or replicated per shard (0) */
int gg_groth16_mpk_info(gg_groth16_mpk_t mpk, int *world, int *distributed_h);
/* 1: the shards split the A, B1, K, G2 MSMs by bucket stripes (each device
 * holds the whole wire tables; GG_MPK_SPLIT=stripes at creation, power-of-two
 * worlds); 0: by wire slices (the default, measured faster per GPU) */
int gg_groth16_mpk_split(gg_groth16_mpk_t mpk, int *bucket_stripes);
/* as gg_groth16_prove (host inputs): Ar, Bs, Krs affine */
int gg_groth16_mpk_prove(gg_groth16_mpk_t mpk, const void *wires, size_t n_wires, const void *sol_a,
                         const void *sol_b, const void *sol_c, size_t n_cons, const void *r_mont,
                         const void *s_mont, void *ar_aff, void *bs_aff, void *krs_aff);
/* gg_groth16_mpk_prove with the solution per shard: wires[r], sol_a[r], sol_b[r],
 * sol_c[r] (r < world) are read by shard r -- host memory (inputs_on_device = 0;
 * the entries may all be the same vectors), or, with inputs_on_device = 1, the
 * WHOLE solution resident on devices[r] (e.g. solved there by gg_r1cs_solve:
 * the 2 MB witness is the only per-proof PCIe traffic).  Shards sharing a GPU
 * may share its copy. */
int gg_groth16_mpk_prove_ex(gg_groth16_mpk_t mpk, int inputs_on_device, const void *const *wires,
                            size_t n_wires, const void *const *sol_a, const void *const *sol_b,
                            const void *const *sol_c, size_t n_cons, const void *r_mont,
                            const void *s_mont, void *ar_aff, void *bs_aff, void *krs_aff);
/* ms of the last gg_groth16_mpk_prove: [0] shards (device work + exchanges),
 * [1] partial sum + finalize, [2] total */
int gg_groth16_mpk_last_timings(gg_groth16_mpk_t mpk, double *ms3);
/* where shard `shard`'s time went in the last proof (cap >= GG_MPK_TIMING_SLOTS):
 * [0] the shard's prove ms (its thread: GPU work + exchanges), [1] exchanges
 * recorded (3 with the distributed computeH), then per exchange e
 * [2+4e] ms waiting at the first barrier (peers still computing),
 * [3+4e] ms pushing its chunks to the peers (hipMemcpyPeerAsync over xGMI,
 *        issue to completion), [4+4e] ms waiting at the second barrier (peers'
 *        pushes into this shard still in flight), [5+4e] MB pushed to peers. */
#define GG_MPK_MAX_EXCHANGES 4
#define GG_MPK_TIMING_SLOTS (2 + 4 * GG_MPK_MAX_EXCHANGES)
int gg_groth16_mpk_shard_timings(gg_groth16_mpk_t mpk, int shard, double *out, int cap);
/* xGMI peer access between the parts of a one-process multi-GPU key, as the
 * key's creation left it (hipDeviceEnablePeerAccess, icicle has no such step):
 * codes[i * world + j] for shard i's device reaching shard j's.  A failed pair
 * still copies, staged through host memory by the runtime -- slow, so a first
 * N-GPU run reports it instead of swallowing it. */
#define GG_PEER_SAME_DEVICE 0 /* both parts on one GPU (a rehearsal) */
#define GG_PEER_ENABLED 1     /* peer access on (enabled now or already) */
#define GG_PEER_UNAVAILABLE 2 /* hipDeviceCanAccessPeer says no */
#define GG_PEER_FAILED 3      /* hipDeviceEnablePeerAccess failed */
int gg_groth16_mpk_peer_access(gg_groth16_mpk_t mpk, int *codes, int cap);
/* Timing rehearsal (bench / tests only): solo_shard >= 0 makes every later
 * prove run shard solo_shard ALONE (its exchanges skip the peers, the other
 * shards contribute identity partials), so one GPU times the work one GPU of
 * an N-GPU node does; such proves write an INVALID proof and return
 * GG_REHEARSAL.  -1 (the default) restores real proofs. */
int gg_groth16_mpk_set_rehearsal(gg_groth16_mpk_t mpk, int solo_shard);

/* per-stage timings (ms) of the last gg_groth16_prove on this thread:
 * [0]=upload [1]=computeH [2]=msm_A [3]=msm_B1 [4]=msm_K [5]=msm_Z [6]=msm_G2
 * [7]=epilogue [8]=total */
int gg_groth16_last_timings(double *ms9);
/* the same plus [9] = host staging of the solution's A, B, C (host inputs: done
 * by the computeH task through pinned buffers while the MSMs run; part of [1]).
 * [0] is the staging of the wires (before any MSM starts); [10], [11] = the
 * steady clock (CLOCK_MONOTONIC, ms) at entry to / return from gg_groth16_prove.
 * cap: entries wanted (<= 12). */
int gg_groth16_last_timings_ex(double *ms, int cap);


/* ------------------------------------------------ PlonK BLS12-381 (fr, 32 B)
 * Quotient-path kernels of backend/plonk/bls12-381/prove.go; all buffers are
 * device memory, bls12-381 fr Montgomery.
 *
 * allConstraints of computeNumerator (prove.go:850-935) on coset `coset` of
 * the big domain, written bit-reversed into cres (prove.go:1030-1041):
 *   x_dev[nx]: host array of device pointers, the s.x polynomials in id_ order
 *     (L, R, O, Z, ZS, Ql, Qr, Qm, Qo, Qk, S1, S2, S3, ID, LOne, Qc_i, Pi_i...;
 *     prove.go:60-77), each n evaluations (Lagrange, regular) on this coset;
 *   bcoef: 4 x 4 fr (host), the blinding polynomials Bl, Br, Bo, Bz already
 *     scaled for this coset as prove.go:1003-1011 does; bdeg[4]: their lengths;
 *   twiddles0_dev: s.twiddles0 (omega_small^j, j < n; prove.go:265-277);
 *   beta, gamma, alpha, coset_gen (= pk.Domain[1].FrMultiplicativeGen): host fr;
 *   rho = |Domain[1]| / n; cres_dev: rho * n fr. */
int gg_plonk_numerator_coset(const void *const *x_dev, int nx, const void *bcoef, const int *bdeg,
                             const void *twiddles0_dev, const void *beta, const void *gamma,
                             const void *alpha, const void *coset_gen, size_t n, int rho, int coset,
                             void *cres_dev, void *hip_stream);
/* divideByXMinusOne (prove.go:1223-1276) in place on a LagrangeCoset/BitReverse
 * vector of |big| elements: multiply by (x^n - 1)^-1 on the big coset, then the
 * big coset iFFT (DIT) -> canonical regular.  big: a GG_CURVE_BLS12_381 domain
 * (pk.Domain[1]); n_small = |pk.Domain[0]|. */
int gg_plonk_divide_by_xn_minus_one(gg_domain_t big, size_t n_small, void *data_dev,
                                    void *hip_stream);
/* fr.BatchInvert in place (prove.go:1273; zeros stay zero) */
int gg_bls12_381_fr_batch_invert(void *data_dev, size_t n, void *hip_stream);

/* ---- PlonK BLS12-381 polynomial ops, device buffers,
 * bls12-381 fr Montgomery (32 B).
 *
 * iop.BuildRatioCopyConstraint (prove.go:600-621) into Lagrange/Regular form:
 *   Z[0] = 1, Z[i+1] = Z[i] * prod_j (f_j[i] + beta*ID(j*n+i) + gamma)
 *                           / prod_j (f_j[i] + beta*ID(S[j*n+i]) + gamma),
 *   f = (L, R, O) Lagrange/Regular (n each), perm_dev = pk.trace.S (3n int64),
 *   ID(s) = u^(s div n) * omega^(s mod n) (getSupportPermutation, setup.go:391-407),
 *   omega = pk.Domain[0].Generator, u = pk.Domain[0].FrMultiplicativeGen. */
int gg_plonk_ratio_copy_constraint(const void *l_dev, const void *r_dev, const void *o_dev,
                                   const int64_t *perm_dev, size_t n, const void *beta,
                                   const void *gamma, const void *omega_mont,
                                   const void *coset_shift_mont, void *z_dev, void *hip_stream);
/* out[bitrev(i)] = in[i] (fft.BitReverse out of place; iop ToRegular / ToBitReverse) */
int gg_bls12_381_fr_bit_reverse(const void *in_dev, void *out_dev, size_t n, void *hip_stream);
/* y[i] += a * x[i] (kzg.BatchOpenSinglePoint folding, sum gamma^i p_i) */
int gg_bls12_381_fr_axpy(void *y_dev, const void *x_dev, size_t n, const void *a_mont, void *hip_stream);
/* in place inclusive running product data[i] = data[0] * ... * data[i] */
int gg_bls12_381_fr_prefix_product(void *data_dev, size_t n, void *hip_stream);
/* value_out (host) = f(a) = sum f_i a^i (iop.Polynomial.Evaluate, canonical
 * regular, prove.go:1118-1145, 1313-1320); q_dev (nullable, n - 1 fr) = the
 * KZG opening quotient (f - f(a)) / (X - a) of kzg.Open (prove.go:646, 823-830). */
int gg_bls12_381_fr_horner(const void *f_dev, size_t n, const void *a_mont, void *q_dev,
                           void *value_out, void *hip_stream);
/* values_out[k] (host, count fr) = f_k(a) for count <= 16 device polynomials
 * (canonical regular, lens[k] coefficients, any lengths) at one point: the
 * evaluations of a PlonK proof at zeta that need no quotient (prove.go:640-660
 * the blinded L, R, O and S1, S2, Qcp_i; kzg.BatchOpenSinglePoint's claimed
 * values), batched into one pass; curve: GG_CURVE_BN254 or GG_CURVE_BLS12_381 fr. */
int gg_fr_evaluate_many(int curve, const void *const *polys_dev, const size_t *lens, int count,
                        const void *point_mont, void *values_out, void *hip_stream);
/* foldH (prove.go:670-705): out[i] = (h3[i]*z + h2[i])*z + h1[i], i < n_small + 2,
 * h_dev = h1 | h2 | h3 (3 (n_small + 2) fr), z = zeta^(n_small + 2) (host). */
int gg_plonk_fold_h(const void *h_dev, size_t n_small, const void *zeta_pow_np2, void *out_dev,
                    void *hip_stream);
/* computeLinearizedPolynomial (prove.go:1289-1389), in place on the blinded Z
 * (canonical, nz fr): with i < nz,
 *   t = z[i]*s2 (+ s3[i]*s1 if i < ns3);  t *= alpha;
 *   if i < nq: t += ql[i]*l + qm[i]*rl + qr[i]*r + qo[i]*o + qk[i] + sum_j pi2_j[i]*qcp_j;
 *   z[i] = t + z[i]*lag
 * q_dev[5] = {Ql, Qr, Qm, Qo, Qk} canonical (nq each); pi2_dev[n_cmt] and
 * qcp_zeta (n_cmt fr, host): BSB22 terms; scalars8 (host, 8 fr) =
 * {s1, s2, alpha, l(zeta), r(zeta), l(zeta)r(zeta), o(zeta), alpha^2 L1(zeta)/n}
 * as computed at prove.go:1300-1336. */
int gg_plonk_linearized(void *blinded_z_dev, size_t nz, const void *s3_dev, size_t ns3,
                        const void *const *q_dev, size_t nq, const void *const *pi2_dev,
                        const void *qcp_zeta, int n_cmt, const void *scalars8, void *hip_stream);

/* ---- PlonK BLS12-381 prover (plonk.Prove after the solver; prove.go:116-1079)
 * Device-resident proving key: replaces backend/plonk/bls12-381 ProvingKey
 * (setup.go:88-106) on the GPU.
 *   log_n, log_big: pk.Domain[0] / Domain[1] sizes (|big| / n in {2, 4, 8});
 *   omega_mont, omega_big_mont: their generators; coset_shift_mont:
 *   Domain[0].FrMultiplicativeGen (= vk.CosetShift);
 *   kzg_g1[n_kzg >= n + 3]: pk.Kzg.G1 (affine 96 B); kzg_lagrange_g1[n]: pk.KzgLagrange.G1;
 *   trace[8]: pk.trace Ql, Qr, Qm, Qo, Qk (incomplete), S1, S2, S3 in canonical
 *     regular form (n fr each, host) -- the form Setup leaves them in (setup.go:229-240);
 *   qcp[n_cmt]: pk.trace.Qcp (canonical); perm: pk.trace.S (3n int64);
 *   nb_public: vk.NbPublicVariables; commitment_constraint_indexes[n_cmt]:
 *     vk.CommitmentConstraintIndexes;
 *   vk_digests (nullable): 96-B affine S[0..2], Ql, Qr, Qm, Qo, Qk, Qcp[..] of pk.Vk;
 *     NULL = commit them on the GPU (commitTrace, setup.go:229-272). */
int gg_plonk_pk_create(int log_n, int log_big, const void *omega_mont, const void *omega_big_mont,
                       const void *coset_shift_mont, const void *kzg_g1, size_t n_kzg,
                       const void *kzg_lagrange_g1, const void *const *trace, const void *const *qcp,
                       int n_cmt, const int64_t *perm, size_t nb_public,
                       const uint64_t *commitment_constraint_indexes, const void *vk_digests,
                       gg_plonk_pk_t *out);
int gg_plonk_pk_release(gg_plonk_pk_t pk);
/* Multi-GPU: rank `rank` of `world` keeps the contiguous slice
 * [m rank / world, m (rank + 1) / world) of pk.Kzg.G1 (m = n + 3) and of
 * pk.KzgLagrange.G1 (m = n); every commitment is a partial MSM that
 * reduce(ctx, jac) turns into the sum over all ranks (BLS12-381 G1Jac, 144 B, in
 * place; e.g. an RCCL all-gather + exact adds).  reduce is called from the
 * proving thread in the same order on every rank.  All other work is
 * replicated (the blinding must be the same on all ranks). */
typedef int (*gg_g1_reduce_fn)(void *ctx, void *jac_inout);
int gg_plonk_pk_create_shard(int log_n, int log_big, const void *omega_mont, const void *omega_big_mont,
                             const void *coset_shift_mont, const void *kzg_g1, size_t n_kzg,
                             const void *kzg_lagrange_g1, const void *const *trace, const void *const *qcp,
                             int n_cmt, const int64_t *perm, size_t nb_public,
                             const uint64_t *commitment_constraint_indexes, const void *vk_digests, int rank,
                             int world, gg_g1_reduce_fn reduce, void *reduce_ctx, gg_plonk_pk_t *out);
/* One process, N GPUs (the Go shape of configs[4] "8xMI355X"): the
 * key of gg_plonk_pk_create split over devices[0..n_devices) (ids may repeat:
 * several parts on one GPU).  devices[0] runs the prover DAG; part d holds slice
 * d of pk.Kzg.G1 and pk.KzgLagrange.G1, so every KZG commitment (prove.go:336,
 * 494, 769, 1165-1218) is an MSM split over the parts and summed in the library;
 * the numerator's rho cosets (prove.go:837-1079) go to parts i % min(rho, N),
 * each with its cosets' key evaluations resident (L, R, O, Z, Qk, Pi_i by peer
 * copy per proof, the coset block of the quotient back).  The result is the
 * same proof as the one-GPU key; gg_plonk_prove / commit_lagrange / vk /
 * release take this handle unchanged.  L, R, O inputs on device live on devices[0]. */
int gg_plonk_pk_create_multi(int log_n, int log_big, const void *omega_mont, const void *omega_big_mont,
                             const void *coset_shift_mont, const void *kzg_g1, size_t n_kzg,
                             const void *kzg_lagrange_g1, const void *const *trace, const void *const *qcp,
                             int n_cmt, const int64_t *perm, size_t nb_public,
                             const uint64_t *commitment_constraint_indexes, const void *vk_digests,
                             int n_devices, const int *devices, gg_plonk_pk_t *out);
/* The PlonK key of either curve (backend/plonk/bls12-381 or backend/plonk/bn254:
 * the same prove.go over BN254, whose G1 affine points are 64 B and fr the BN254
 * scalar field); every other argument as gg_plonk_pk_create, with
 * n_devices / devices as gg_plonk_pk_create_multi (n_devices <= 1: one GPU, the
 * calling thread's).  The handle works with every gg_plonk_* call below; point
 * buffers (vk, commit_lagrange, proof) then hold the curve's point size. */
int gg_plonk_pk_create_ex(int curve, int log_n, int log_big, const void *omega_mont, const void *omega_big_mont,
                          const void *coset_shift_mont, const void *kzg_g1, size_t n_kzg,
                          const void *kzg_lagrange_g1, const void *const *trace, const void *const *qcp,
                          int n_cmt, const int64_t *perm, size_t nb_public,
                          const uint64_t *commitment_constraint_indexes, const void *vk_digests,
                          int n_devices, const int *devices, gg_plonk_pk_t *out);
/* gg_plonk_pk_create_shard for either curve */
int gg_plonk_pk_create_shard_ex(int curve, int log_n, int log_big, const void *omega_mont,
                                const void *omega_big_mont, const void *coset_shift_mont, const void *kzg_g1,
                                size_t n_kzg, const void *kzg_lagrange_g1, const void *const *trace,
                                const void *const *qcp, int n_cmt, const int64_t *perm, size_t nb_public,
                                const uint64_t *commitment_constraint_indexes, const void *vk_digests, int rank,
                                int world, gg_g1_reduce_fn reduce, void *reduce_ctx, gg_plonk_pk_t *out);
/* the key's curve, log2 of its domain and its number of BSB22 commitments */
int gg_plonk_pk_info(gg_plonk_pk_t pk, int *curve, int *log_n, int *n_cmt);
/* the key's device parts: *n_devices, devices[0..) (primary first; devices nullable) */
int gg_plonk_pk_devices(gg_plonk_pk_t pk, int *devices, int cap, int *n_devices);
/* Timing rehearsal (bench / tests only): on != 0 makes the peer parts of a
 * multi-part key do nothing in later proves (no MSM slices, no cosets), so one
 * GPU times the primary part's work; such proves write an INVALID proof and
 * return GG_REHEARSAL.  0 (the default) restores real proofs. */
int gg_plonk_pk_set_rehearsal(gg_plonk_pk_t pk, int on);
/* The same for any one device part: part p >= 0 alone does its work (its MSM
 * slices, ratio slice, quotient units, canonical-form tasks; part 0 also the
 * tail stages and the openings), the others skip theirs; -1 ends rehearsals.
 * gg_plonk_pk_set_rehearsal(pk, on) = part 0 / -1. */
int gg_plonk_pk_set_rehearsal_part(gg_plonk_pk_t pk, int part);
/* where device part `part` (0 = primary) spent the last proof (cap >=
 * GG_PLONK_PART_SLOTS): [0] MSM slices, [1] their ms (incl. the scalar copy),
 * [2] ms copying scalar slices from the primary (xGMI), [3] MB copied, [4]
 * quotient units (classes of the big domain), [5] their ms (FFTs, numerator,
 * block inverse DFT, blocks back), [6] 0 (kept for layout: the per-proof
 * polynomials now arrive by the canonical-form pushes of [11..13]), [7] ms
 * copying the units' blocks back, [8] MB moved for the quotient units, [9]
 * part 0 only: ms waiting for the peers' canonical forms, MSM slices and
 * quotient units after finishing its own work, [10] ms of its slice of the
 * copy-constraint ratio (factors, scan, fix-up), [11] canonical-form tasks run
 * (a size-n inverse DFT of L, R, O, Z, Qk or Pi_j: peers only), [12] their ms
 * (input, transform, pushes), [13] MB they pushed over xGMI. */
#define GG_PLONK_PART_SLOTS 14
int gg_plonk_pk_part_timings(gg_plonk_pk_t pk, int part, double *out, int cap);
/* GG_PEER_* codes per ordered pair of device parts (codes[i * parts + j]);
 * codes = NULL only stores the part count in *n_parts */
int gg_plonk_pk_peer_access(gg_plonk_pk_t pk, int *codes, int cap, int *n_parts);
/* the key's vk digests, 96-B affine each: S[0..2], Ql, Qr, Qm, Qo, Qk, Qcp[0..n_cmt) */
int gg_plonk_pk_vk(gg_plonk_pk_t pk, void *out, size_t cap);
/* kzg.Commit(values, pk.KzgLagrange): n Lagrange values (host or device) -> affine 96 B.
 * The BSB22 solver hint (bsb22Hint, prove.go:316-352) commits through this. */
int gg_plonk_commit_lagrange(gg_plonk_pk_t pk, const void *values, int on_device, void *out_aff);
/* bytes of a proof with n_cmt BSB22 commitments (layout below; BLS12-381 points) */
size_t gg_plonk_proof_size(int n_cmt);
/* the same for a curve (BN254: 64-B points) */
size_t gg_plonk_proof_size_ex(int curve, int n_cmt);
/* Prove after Solve (prove.go:116-176; the errgroup DAG as HIP streams):
 *   l, r, o: solution.L, R, O (n fr Lagrange regular, host or device);
 *   public_witness[nb_public]: fullWitness[:len(spr.Public)] (host, completeQk + bindPublicData);
 *   BSB22 (n_cmt as the key): cmt_values[i] = the bsb22Hint's committed-value vector (n fr,
 *     Lagrange, host), cmt_digests = proof.Bsb22Commitments (96 B each), cmt_hashed =
 *     s.commitmentVal (fr each);
 *   blinding (nullable): the 9 coefficients of Bl, Br, Bo (2 each) and Bz (3); NULL = random;
 *   challenge_hash / folding_hash (+ ctx): opts.ChallengeHash / KZGFoldingHash, NULL = SHA-256.
 * proof_out (gg_plonk_proof_size bytes): affine 96 B / fr 32 B, Montgomery:
 *   LRO[3] | Z | H[3] | Bsb22Commitments[n_cmt] | BatchedProof.H |
 *   BatchedProof.ClaimedValues[7 + n_cmt] | ZShiftedOpening.H | ZShiftedOpening.ClaimedValue */
int gg_plonk_prove(gg_plonk_pk_t pk, const void *l, const void *r, const void *o, int inputs_on_device,
                   const void *public_witness, size_t nb_public, const void *const *cmt_values,
                   const void *cmt_digests, const void *cmt_hashed, int n_cmt, const void *blinding,
                   gg_hash_fn challenge_hash, void *challenge_ctx, gg_hash_fn folding_hash,
                   void *folding_ctx, void *proof_out, size_t proof_cap);
/* cumulative stage ends (ms) of the last gg_plonk_prove on this thread: commitToLRO,
 * Z, quotient, H commitments, linearized, batch opening */
int gg_plonk_last_timings(double *ms, int cap);

/* ---- witness / fr.Vector binary format (backend/witness/witness.go:15-36)
 * Field elements are serialised as 32-byte big-endian canonical integers; the
 * prover uses gnark-crypto's in-memory layout (Montgomery, LE limbs).
 * gg_fr_from_canonical_be: in_dev (n x 32 B big-endian) -> out_dev (Montgomery),
 *   may alias; fails (GG_ERR_INVALID_ARG) if any element is >= r, as
 *   fr.Vector.ReadFrom does; *n_invalid (nullable) = their count.
 * gg_fr_to_canonical_be: the inverse (fr.Vector.WriteTo element encoding).
 * curve: GG_CURVE_BN254 or GG_CURVE_BLS12_381 (scalar field). */
int gg_fr_from_canonical_be(int curve, const void *in_dev, void *out_dev, size_t n,
                            uint64_t *n_invalid, void *hip_stream);
int gg_fr_to_canonical_be(int curve, const void *in_dev, void *out_dev, size_t n, void *hip_stream);

/* ---- R1CS solver (constraint/bn254/solver.go:418-608, R1CS without hints)
 * replaces r1cs.Solve(fullWitness) -> R1CSSolution{W, A, B, C} (prove.go:119-126,
 * system.go:64-104) on the GPU, leaving the solution in HBM for gg_groth16_prove
 * (inputs_on_device = 1).  The system in CSR form, as gnark's public API gives it:
 *   term_off[3 c + s] .. term_off[3 c + s + 1]: terms of side s (0 L, 1 R, 2 O) of
 *     constraint c (r1cs.GetR1Cs()); term_wire / term_coeff: wire id and index
 *     into coeffs (r1cs.Coefficients, fr Montgomery);
 *   level_off[l] .. level_off[l + 1]: the constraints of level l (r1cs.Levels).
 * gg_r1cs_solve: witness = public (without ONE_WIRE) then secret values, fr
 *   Montgomery (witness.Vector(), solver.go:65-114); W (n_wires) and A, B, C
 *   (n_constraints) copied to the caller's buffers when non-null (host or device
 *   per out_on_device).  GG_ERR_UNSATISFIED: *unsatisfied = the first failing
 *   constraint (-1 when every constraint holds but wires were left unsolved).
 *   Circuits with hint calls solve on the host (gnark's solver). BN254 only. */
typedef struct gg_r1cs *gg_r1cs_t;
int gg_r1cs_create(size_t n_wires, size_t n_constraints, const uint32_t *term_off,
                   const uint32_t *term_wire, const uint32_t *term_coeff, const void *coeffs,
                   size_t n_coeffs, const uint32_t *level_off, const uint32_t *level_cons,
                   size_t n_levels, gg_r1cs_t *out);
/* the same for curve GG_CURVE_BN254 or GG_CURVE_BLS12_381 (the scalar field of
 * backend/groth16/bls12-381, whose solver is constraint/bls12-381/solver.go) */
int gg_r1cs_create_ex(int curve, size_t n_wires, size_t n_constraints, const uint32_t *term_off,
                      const uint32_t *term_wire, const uint32_t *term_coeff, const void *coeffs,
                      size_t n_coeffs, const uint32_t *level_off, const uint32_t *level_cons,
                      size_t n_levels, gg_r1cs_t *out);
int gg_r1cs_release(gg_r1cs_t r);
int gg_r1cs_info(gg_r1cs_t r, size_t *n_wires, size_t *n_constraints, size_t *n_levels);
int gg_r1cs_solve(gg_r1cs_t r, const void *witness, size_t n_witness, int witness_on_device,
                  void *w_out, void *a_out, void *b_out, void *c_out, int out_on_device,
                  int64_t *unsatisfied);
/* newSolver's witness-size check (solver.go:71-76): afterwards gg_r1cs_solve
 * fails with "invalid witness size, got %d, expected %d" unless
 * n_witness == nb_public - 1 + nb_secret (r1cs.GetNbPublicVariables() counts ONE_WIRE) */
int gg_r1cs_set_inputs(gg_r1cs_t r, size_t nb_public, size_t nb_secret);
/* device pointers of the handle's resident W, A, B, C (valid until the next
 * solve or the release): a prove can read them without a copy */
int gg_r1cs_solution_dev(gg_r1cs_t r, void **w, void **a, void **b, void **c);
/* the schedule the last solve ran (solver.go:418-533 levels, replaced by
 * dependency strands when the levels allow it): *strands = 1 for the strand
 * schedule (one launch per super-level), 0 for one launch per level;
 * *launches = kernel launches per solve, *segments = strand segments (threads) */
int gg_r1cs_schedule(gg_r1cs_t r, int *strands, size_t *launches, size_t *segments);

/* ---- sparse-R1CS (PlonK) solver: the SCS blueprints' Solve
 * (constraint/blueprint_scs.go:53-151) level by level (solver.go:418-533) and
 * evaluateLROSmallDomain (constraint/bls12-381/system.go:221-264): replaces
 * spr.Solve(fullWitness) -> SparseR1CSSolution{L, R, O} (plonk prove.go:180-187)
 * for hint-free systems; L, R, O (domain = next power of two of
 * n_constraints + nb_public) stay in HBM for gg_plonk_prove (inputs_on_device).
 *   wires[3 c + 0..2] = xa, xb, xc; qidx[5 c + 0..4] = qL, qR, qO, qM, qC
 *   (indices into coeffs, fr Montgomery); flags[c] & 1: a BSB22 commitment
 *   constraint (not solved, blueprint_scs.go:56-60), flags nullable;
 *   levels as for gg_r1cs_create.  witness = public then secret values (no
 *   ONE_WIRE).  curve: GG_CURVE_BLS12_381 or GG_CURVE_BN254 (scalar field).
 *   GG_ERR_UNSATISFIED: *failed = the first failing constraint (unsatisfied or
 *   a zero divisor: errDivideByZero). */
typedef struct gg_scs *gg_scs_t;
int gg_scs_create(int curve, size_t n_wires, size_t n_constraints, size_t nb_public, const uint32_t *wires,
                  const uint32_t *qidx, const uint8_t *flags, const void *coeffs, size_t n_coeffs,
                  const uint32_t *level_off, const uint32_t *level_cons, size_t n_levels, gg_scs_t *out);
int gg_scs_release(gg_scs_t h);
int gg_scs_info(gg_scs_t h, size_t *n_wires, size_t *n_constraints, size_t *domain);
int gg_scs_solve(gg_scs_t h, const void *witness, size_t n_witness, int witness_on_device, void *w_out,
                 void *l_out, void *r_out, void *o_out, int out_on_device, int64_t *failed);
int gg_scs_solution_dev(gg_scs_t h, void **w, void **l, void **r, void **o);
/* as gg_r1cs_schedule, for the sparse-R1CS solver */
int gg_scs_schedule(gg_scs_t h, int *strands, size_t *launches, size_t *segments);
/* the same check for a sparse R1CS: n_witness == nb_public + nb_secret */
int gg_scs_set_inputs(gg_scs_t h, size_t nb_public, size_t nb_secret);

/* ------------------------------------------------------------ profiling
 * Kernel-level timing with HIP events recorded on the stream each kernel is
 * launched on (bench.py uses it for the roofline of the dominant kernel).
 * gg_profile_enable(1) clears and enables; names: "msm_accum", "msm_sort",
 * "msm_reduce", "ntt_pass", ... ; totals are summed over launches. */
int gg_profile_enable(int on);
int gg_profile_get(const char *name, double *total_ms, int64_t *launches, double *units);

#ifdef __cplusplus
}
#endif
#endif /* GNARK_AMD_H */
