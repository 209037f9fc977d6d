// PlonK prover behind the C ABI: the device section of gnark's
// backend/plonk/bls12-381 and backend/plonk/bn254 Prove (prove.go:116-1079,
// the same generated code for both curves) after the solver.  PlonkImpl<Cv> is
// the prover over one curve; the C handle dispatches on the key's curve.
//
// Stages (prove.go's errgroup DAG, mapped onto 4 HIP streams and host threads):
//   commitToLRO        3 KZG MSMs on pk.KzgLagrange at once (one MsmWork each),
//                      blinding commitments on the host meanwhile; canonical
//                      L, R, O, completeQk and the BSB22 Pi_i on another stream
//   gamma, beta        Fiat-Shamir (bindPublicData: vk digests, public inputs)
//   ratio Z            BuildRatioCopyConstraint + its commitment
//   alpha              Bsb22Commitments, Z
//   computeNumerator   per coset of the big domain (two cosets in flight):
//                      coset FFTs of L, R, O, Z, Qk, Pi_i (the key's polynomials
//                      are resident coset evaluations), allConstraints kernel
//   divideByXMinusOne  big-coset iFFT, then H1, H2, H3 committed at once
//   zeta               H
//   openZ | linearize  Z opened at zeta*omega (its quotient MSM overlaps the
//                      linearized polynomial and its MSM); foldH
//   batchOpening       kzg.BatchOpenSinglePoint at zeta
// Transcripts: fiat-shamir (challenge = H(name | previous | bindings)),
// points bound with RawBytes (deriveRandomness, verify.go:342-360) or Marshal
// (= RawBytes too: bindPublicData verify.go:296-340, kzg deriveGamma), scalars as
// 32-B big-endian.  The hash is the caller's (gg_hash_fn) or SHA-256.
#include "plonk_ops.h"
#include "curve.cuh"
#include "sha256.h"
#include <atomic>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <cstring>
#include <chrono>
#include <cstdlib>
#include <fstream>
#include <type_traits>

struct gg_msm_base;
namespace gg {
struct MsmWork;
void msm_device_work(gg_msm_base* b, MsmWork* w, const Fr* scalars_dev, void* out_jac, hipStream_t st);
void msm_device_work_batch(gg_msm_base* b, MsmWork* w, const Fr* const* scalars_dev, int nvec, void* const* out_jac,
                           hipStream_t st);
MsmWork* msm_work_new();
void msm_work_delete(MsmWork* w);
bool msm_base_batch_fits(const gg_msm_base* b, int nvec);
}  // namespace gg

using namespace gg;

// curves of the PlonK prover: backend/plonk/bls12-381 and backend/plonk/bn254
// (the same generated prove.go over another curve)
struct PlonkBls12381 {
    using Fr = FrBls;
    using Fp = FpBls;
    static constexpr int curve = GG_CURVE_BLS12_381, group = GG_BLS12_381_G1, fp_u32 = 12;
    static constexpr uint8_t raw_inf = 0x40;             // mUncompressedInfinity (zcash flags)
    static constexpr uint32_t fr_top_mask = 0x7fffffffu;  // r < 2^255
};
struct PlonkBn254 {
    using Fr = gg::Fr;
    using Fp = gg::Fp;
    static constexpr int curve = GG_CURVE_BN254, group = GG_G1, fp_u32 = 8;
    static constexpr uint8_t raw_inf = 0x00;             // mUncompressed: infinity is all zeros
    static constexpr uint32_t fr_top_mask = 0x3fffffffu;  // r < 2^254
};

// key polynomial ids shared by both curves
struct PK {
    enum { QL, QR, QM, QO, QK, S1, S2, S3, NTRACE };
    enum { E_QL, E_QR, E_QM, E_QO, E_S1, E_S2, E_S3, E_X, E_LONE, E_QCP0 };
};

// the C handle: a PlonkImpl<Cv>::Key of its curve
struct gg_plonk_pk {
    int curve = GG_CURVE_BLS12_381;
    virtual ~gg_plonk_pk() {}
};

namespace {

// ------------------------------------------------------------ encodings
// canonical little-endian u32 limbs -> big-endian bytes
template <int N>
void be_bytes(const uint32_t* v, uint8_t* out) {
    for (int i = 0; i < N; i++) {
        const uint32_t w = v[N - 1 - i];
        out[4 * i] = (uint8_t)(w >> 24);
        out[4 * i + 1] = (uint8_t)(w >> 16);
        out[4 * i + 2] = (uint8_t)(w >> 8);
        out[4 * i + 3] = (uint8_t)w;
    }
}

// ------------------------------------------------------------ transcript
struct Hasher {
    gg_hash_fn fn;
    void* ctx;
    std::vector<uint8_t> operator()(const std::vector<uint8_t>& msg) const {
        if (!fn) {
            std::vector<uint8_t> d(32);
            Sha256::hash(msg.data(), msg.size(), d.data());
            return d;
        }
        std::vector<uint8_t> d(128);
        size_t len = d.size();
        GG_CHECK(fn(ctx, msg.data(), msg.size(), d.data(), &len) == 0, GG_ERR_INVALID_ARG, "hash callback failed");
        GG_CHECK(len >= 1 && len <= 128, GG_ERR_INVALID_ARG, "hash callback: digest of 1..128 bytes");
        d.resize(len);
        return d;
    }
};


}  // namespace


// ============================================================== key
// Quotient units (computeNumerator + divideByXMinusOne, prove.go:837-1079,
// 1223-1276, split over device parts).  The big domain u<w_big> (4n points,
// rho = |big| / n cosets) is cut into U = rho S classes K = p (mod U), S >= 1 a
// power of two (S = 1: the cosets; S = 2 on 8 GPUs: half cosets).  Unit p owns
// the m = n / S points u w_big^p <w^S>:
//   * each per-proof polynomial (canonical, bit-reversed) is folded to m
//     coefficients (fold_brev, kappa = s_p^m) and coset-FFTed there (size m,
//     shift s_p = u w_big^p); ZS's points are class p + rho (mod U): for S > 1
//     Z is evaluated there too;
//   * the numerator (allConstraints) is taken on the m points and scaled by
//     1 / (x^n - 1) (constant on a coset);
//   * the values sit in cres at bitrev(U j + p): one contiguous block of m
//     (block bitrev_u(p), u = log2 U), whose first L - u stages of the big
//     coset iFFT (DIT) stay inside the block -- the unit runs them as a size-m
//     inverse DFT; the owner of cres (part 0) runs the last u stages over all
//     blocks (ntt_tail_inverse_coset).
// Unit p runs on part p mod N; on one GPU (N = 1) the four coset units and the
// tail are exactly FFTInverse(DIT, OnCoset) of the whole vector.
struct QUnit {
    int p = 0, device = 0;
    gg_domain_t dom = nullptr;   // size m, root w^S, coset generator s_p
    gg_domain_t zdom = nullptr;  // S > 1: the class (p + rho) mod U (ZS)
    uint32_t kappa[8] = {}, zkappa[8] = {}, inv_den[8] = {};  // s_p^m, s_p'^m, 1 / (s_c^n - 1)
    std::vector<DevBuf> ev;      // the key polynomials on the class (Ql Qr Qm Qo S1 S2 S3 X LOne Qcp_i)
    DevBuf tw0, tw1;             // S > 1: twiddles0 at the class's points and at the next ones
    DevBuf out;                  // on a peer: the class's block of the quotient
    ~QUnit() {
        int cur = 0;
        const bool restore = hipGetDevice(&cur) == hipSuccess;
        (void)hipSetDevice(device);
        if (dom) gg_domain_release(dom);
        if (zdom) gg_domain_release(zdom);
        ev.clear();
        tw0.release();
        tw1.release();
        out.release();
        if (restore) (void)hipSetDevice(cur);
    }
};

// One-process multi-GPU (gg_plonk_pk_create_multi): device parts[p] (p >= 1) of
// a key holds slice p of pk.Kzg.G1 / pk.KzgLagrange.G1 (every commitment is an
// MSM split over the parts, partials summed exactly on the host) and runs its
// quotient units (the key polynomials' evaluations on their classes resident
// there; the per-proof L, R, O, Z, Qk, Pi_i arrive by peer copy, each unit's
// block of the quotient goes back the same way).
struct PlonkPeer {
    int device = 0;
    hipStream_t s[4] = {nullptr, nullptr, nullptr, nullptr};  // 0..2: MSMs (work slot), 3: cosets
    TaskQueue tq[4];                                          // the slots behind s (common.h)
    hipStream_t* act[4] = {&s[0], &s[1], &s[2], &s[3]};
    gg_msm_base_t kzg = nullptr, kzg_lag = nullptr;
    size_t k_lo = 0, k_hi = 0, l_lo = 0, l_hi = 0;
    MsmWork* work[3] = {nullptr, nullptr, nullptr};
    DevBuf scal[3];                     // scalar slice staging per work slot
    std::vector<std::unique_ptr<QUnit>> units;  // quotient units placed here
    DevBuf perm_slice, pz;              // S of its KzgLagrange slice (3 columns), its ratio scan
    Arena ar;                           // ratio scratch
    DevBuf tw0, in[5 + plk::MAX_CMT];   // twiddles0 (S = 1); L R O Z (canonical bit-reversed), Qk, Pi_j
    DevBuf cev[7 + plk::MAX_CMT], zc;   // a unit's evaluation slot; ZS (S > 1)
    hipEvent_t ea[4] = {}, eb[4] = {};  // per stream: around the last peer copy (timing)
    // canonical-form tasks placed here (Key::canon_owner): the size-n domain, the
    // regular form of a task's polynomial, pk's Qk in Lagrange form (Qk's owner),
    // one push stream per destination part
    gg_domain_t d0 = nullptr;
    DevBuf creg, qk_lag;
    std::vector<hipStream_t> xs;
    hipEvent_t reg_ev = nullptr;  // the last regular-form push to part 0 (creg free again)
    bool reg_pending = false;
    hipStream_t cs = nullptr;     // the tasks' transforms (stream 3 belongs to the quotient units)
    // its pushes out of a compute stream's result (its Z slice, its units' blocks):
    // a copy stream of the greatest priority (own hardware queue, common.h) that
    // waits for the producing kernel by event only
    hipStream_t cps = nullptr;
    hipEvent_t cpev = nullptr;
    ~PlonkPeer() {
        int cur = 0;
        const bool restore = hipGetDevice(&cur) == hipSuccess;
        (void)hipSetDevice(device);
        for (auto w : work)
            if (w) msm_work_delete(w);
        if (kzg) gg_msm_base_release(kzg);
        if (kzg_lag) gg_msm_base_release(kzg_lag);
        units.clear();
        for (auto& b : scal) b.release();
        for (auto& b : in) b.release();
        for (auto& b : cev) b.release();
        zc.release();
        tw0.release();
        if (d0) gg_domain_release(d0);
        creg.release();
        qk_lag.release();
        for (hipStream_t x : xs) (void)hipStreamDestroy(x);
        if (reg_ev) (void)hipEventDestroy(reg_ev);
        if (cps) (void)hipStreamDestroy(cps);
        if (cpev) (void)hipEventDestroy(cpev);
        if (cs) (void)hipStreamDestroy(cs);
        perm_slice.release();
        pz.release();
        ar.buf.release();
        task_streams_release(tq, 4, device);
        for (int i = 0; i < 4; i++) {
            if (ea[i]) (void)hipEventDestroy(ea[i]);
            if (eb[i]) (void)hipEventDestroy(eb[i]);
        }
        if (restore) (void)hipSetDevice(cur);
    }
};

// where a device part's time went in the last proof (gg_plonk_pk_part_timings)
struct PlonkPartTimes {
    double msm_count = 0, msm_ms = 0, scalar_copy_ms = 0, scalar_mb = 0;
    double coset_count = 0, coset_ms = 0, coset_in_copy_ms = 0, coset_out_copy_ms = 0, coset_mb = 0;
    double wait_ms = 0;  // part 0: time spent waiting for the peers' MSM slices and cosets
    double ratio_ms = 0;  // its slice of the copy-constraint ratio (factors, scan, fix-up)
    double canon_count = 0, canon_ms = 0, canon_mb = 0;  // canonical-form tasks: count, ms, MB pushed
};

// ============================================================== prover of one curve
template <class Cv>
struct PlonkImpl {
    using FrB = typename Cv::Fr;
    using BAff = Affine<typename Cv::Fp>;
    using BJac = Jac<typename Cv::Fp>;
    static constexpr size_t PT = sizeof(BAff);  // affine G1 bytes: 96 (BLS12-381), 64 (BN254)

// fr.Element.Marshal: 32-B big-endian canonical
static void fr_marshal(const FrB& x, uint8_t out[32]) {
    const FrB c = from_mont(x);
    be_bytes<8>(c.v, out);
}
// fr.Element.SetBytes: big-endian integer mod r
static FrB fr_set_bytes(const uint8_t* b, size_t n) {
    FrB acc = FrB::zero();
    FrB b256 = FrB::zero();
    b256.v[0] = 256;
    b256 = to_mont(b256);
    for (size_t i = 0; i < n; i++) {
        FrB d = FrB::zero();
        d.v[0] = b[i];
        acc = acc * b256 + to_mont(d);
    }
    return acc;
}
// G1Affine.RawBytes = Marshal (uncompressed X | Y, 2 x the fp bytes; infinity:
// BLS12-381 0x40 | zeros, BN254 all zeros -- gnark-crypto's mUncompressedInfinity)
static void g1_raw_bytes(const BAff& p, uint8_t* out) {
    memset(out, 0, PT);
    if (p.is_inf()) {
        out[0] = Cv::raw_inf;
        return;
    }
    be_bytes<Cv::fp_u32>(from_mont(p.x).v, out);
    be_bytes<Cv::fp_u32>(from_mont(p.y).v, out + PT / 2);
}


// gnark-crypto fiat-shamir Transcript: challenge i = H(name_i | value_(i-1) | bindings_i)
struct Transcript {
    std::vector<std::string> names;
    std::vector<std::vector<uint8_t>> bound, value;
    Hasher h;
    Transcript(std::initializer_list<const char*> ns, Hasher hh) : h(hh) {
        for (const char* s : ns) names.emplace_back(s);
        bound.resize(names.size());
        value.resize(names.size());
    }
    size_t idx(const char* n) const {
        for (size_t i = 0; i < names.size(); i++)
            if (names[i] == n) return i;
        throw Error(GG_ERR_INTERNAL, "unknown challenge");
    }
    void bind(const char* n, const uint8_t* b, size_t len) {
        auto& v = bound[idx(n)];
        v.insert(v.end(), b, b + len);
    }
    FrB compute(const char* n) {
        const size_t i = idx(n);
        std::vector<uint8_t> msg(names[i].begin(), names[i].end());
        if (i) msg.insert(msg.end(), value[i - 1].begin(), value[i - 1].end());
        msg.insert(msg.end(), bound[i].begin(), bound[i].end());
        value[i] = h(msg);
        return fr_set_bytes(value[i].data(), value[i].size());
    }
};
// deriveRandomness (verify.go:342-360): RawBytes of each point, then the challenge
static FrB derive(Transcript& fs, const char* n, std::initializer_list<const BAff*> pts) {
    uint8_t b[96];
    for (const BAff* p : pts) {
        g1_raw_bytes(*p, b);
        fs.bind(n, b, PT);
    }
    return fs.compute(n);
}

// ------------------------------------------------------------ host G1 helpers
static BJac jmul(const BAff& p, const FrB& k) {
    const FrB c = from_mont(k);
    return jac_mul(BJac::from_affine(p), c.v);
}
static BAff to_aff(const BJac& j) { return jac_to_affine(j); }
// k <= 4 points with one field inversion (Montgomery's trick): the commitments
// of a stage come out together, and each host inversion is ~25 us on the
// critical path of the stage's hand-over (r06p HIP trace)
static void to_aff_batch(const BJac* j, int k, BAff* out) {
    using Fq = decltype(j[0].z);
    Fq pre[4];
    Fq acc = Fq::one();
    for (int i = 0; i < k; i++) {
        pre[i] = acc;
        if (!j[i].is_inf()) acc = acc * j[i].z;
    }
    Fq inv = inverse(acc);
    for (int i = k - 1; i >= 0; i--) {
        if (j[i].is_inf()) {
            out[i] = BAff::inf();
            continue;
        }
        const Fq zi = inv * pre[i];
        inv = inv * j[i].z;
        const Fq zi2 = sqr(zi);
        out[i] = BAff{j[i].x * zi2, j[i].y * zi2 * zi};
    }
}
static FrB frv(uint64_t x) {
    FrB r = FrB::zero();
    r.v[0] = (uint32_t)x;
    r.v[1] = (uint32_t)(x >> 32);
    return to_mont(r);
}
static FrB horner_host(const std::vector<FrB>& c, const FrB& x) {
    FrB r = FrB::zero();
    for (size_t k = c.size(); k-- > 0;) r = r * x + c[k];
    return r;
}
// random fr (rejection sampled, SetRandom of gnark-crypto)
static FrB fr_random() {
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    static std::ifstream ur("/dev/urandom", std::ios::binary);
    GG_CHECK(ur.good(), GG_ERR_INTERNAL, "no /dev/urandom");
    const FrB p = FrB::modulus();
    for (;;) {
        FrB x;
        ur.read((char*)x.v, 32);
        x.v[7] &= Cv::fr_top_mask;  // r < 2^255 (BLS12-381), < 2^254 (BN254)
        bool lt = false;
        for (int i = 7; i >= 0; i--)
            if (x.v[i] != p.v[i]) { lt = x.v[i] < p.v[i]; break; }
        if (lt) return to_mont(x);
    }
}

struct Key : gg_plonk_pk {
    using CvT = Cv;
    int log_n = 0, log_big = 0;
    size_t n = 0, big = 0, rho = 0;
    FrB omega, omega_big, u, n_inv;
    gg_domain_t d0 = nullptr, d1 = nullptr;
    std::vector<FrB> coset_shift;  // u w_big^i, i < rho
    // trace, canonical regular (reg) and bit-reversed (brev); Qk incomplete
    enum { QL = PK::QL, QR, QM, QO, QK, S1, S2, S3, NTRACE };
    DevBuf reg[NTRACE], brev[NTRACE], qk_lag;
    std::vector<DevBuf> qcp_reg, qcp_brev;
    // resident evaluations of Ql Qr Qm Qo S1 S2 S3 X LOne Qcp_i on every quotient unit's class
    enum { E_QL = PK::E_QL, E_QR, E_QM, E_QO, E_S1, E_S2, E_S3, E_X, E_LONE, E_QCP0 };
    int U = 1, S = 1, log_u = 0;  // quotient units: U = rho S classes of the big domain
    bool split_idft = false;      // units run the first L - log_u stages of the big coset iFFT
    std::vector<std::unique_ptr<QUnit>> units;  // units of part 0
    DevBuf perm, tw0;
    gg_msm_base_t kzg = nullptr, kzg_lag = nullptr;
    BAff blind_lo[3], blind_hi[3];  // G1[0..3), G1[n..n+3)
    BAff vkS[3], vkQ[5];            // S1 S2 S3, Ql Qr Qm Qo Qk
    std::vector<BAff> vkQcp;
    size_t nb_public = 0;
    std::vector<uint64_t> cmt_idx;
    // multi-GPU: this rank keeps pk.Kzg.G1[k_lo, k_hi) and pk.KzgLagrange.G1[l_lo, l_hi);
    // every commitment is a partial MSM completed by `reduce` (sum over ranks)
    int rank = 0, world = 1;
    size_t k_lo = 0, k_hi = 0, l_lo = 0, l_hi = 0;
    gg_g1_reduce_fn reduce = nullptr;
    void* reduce_ctx = nullptr;
    // one-process multi-GPU: this key is part 0 of 1 + peers.size() device parts
    std::vector<std::unique_ptr<PlonkPeer>> peers;
    int n_parts = 1;  // device parts (unit p -> part p mod n_parts)
    // gg_plonk_pk_set_rehearsal / _part (timing only): only part solo_part does
    // its work, the proof is not valid and gg_plonk_prove returns GG_REHEARSAL
    bool solo = false;
    int solo_part = 0;
    // device parts' task streams on hardware queues of their own (task_streams_init):
    // creation layout = part order while the device's GG_TASK_QUEUES last; a
    // rehearsal of part p gives p's device's queues to p (restream), -1 restores
    // the creation layout (GG_PLONK_PART_QUEUES=1)
    bool part_queues = false;
    int queue_owner = -1;  // part holding its device's dedicated queues (-1: creation layout)
    std::mutex tmu;
    std::vector<PlonkPartTimes> ptimes;  // [part], last proof
    std::vector<int> peer_codes;         // GG_PEER_* per ordered part pair (one-process parts)
    int n_cmt = 0;
    hipStream_t s[4] = {nullptr, nullptr, nullptr, nullptr};
    TaskQueue tq[4];  // the slots behind s (common.h: own stream + borrowed dedicated queue)
    hipStream_t* act[4] = {&s[0], &s[1], &s[2], &s[3]};
    MsmWork* work[3] = {nullptr, nullptr, nullptr};
    hipEvent_t msm_ready[3] = {nullptr, nullptr, nullptr};  // per work slot: its scalars are complete
    Arena ar[4];
    // per-proof buffers
    DevBuf lag[3], can[4], cbrev[4], zlag, pz, qkc, pi_reg[plk::MAX_CMT], pi_brev[plk::MAX_CMT];
    DevBuf cev[2][7 + plk::MAX_CMT], zc[2];  // unit evaluation slots (two units in flight), ZS (S > 1)
    DevBuf cres, hpad[3], bz, bl[3], fold, lin, q1, q2, vals, pad;
    int device = 0;
    std::vector<hipEvent_t> evs;  // cross-stream ordering events, reused by every prove
    size_t ev_next = 0;
    std::mutex mu;
    Key() { curve = Cv::curve; }
    ~Key() override {
        peers.clear();
        for (hipEvent_t e : evs) (void)hipEventDestroy(e);
        for (hipEvent_t e : msm_ready)
            if (e) (void)hipEventDestroy(e);
        for (auto w : work)
            if (w) msm_work_delete(w);
        if (kzg) gg_msm_base_release(kzg);
        if (kzg_lag) gg_msm_base_release(kzg_lag);
        if (d0) gg_domain_release(d0);
        if (d1) gg_domain_release(d1);
        units.clear();
        task_streams_release(tq, 4, device);
    }
};


static FrB* F(const DevBuf& b) { return b.as<FrB>(); }
static void dcopy(void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (bytes) GG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
}
static void zero(void* dst, size_t bytes, hipStream_t st) {
    if (bytes) GG_HIP(hipMemsetAsync(dst, 0, bytes, st));
}
static void up(void* dst, const void* src, size_t bytes, bool on_dev, hipStream_t st) {
    if (bytes) GG_HIP(hipMemcpyAsync(dst, src, bytes, on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
}
// canonical regular -> canonical bit-reversed copy
static void to_brev(Key* pk, const FrB* reg, FrB* brev, hipStream_t st) { plk::bit_reverse(reg, brev, pk->n, st); }
// Lagrange regular (n) -> canonical bit-reversed (out) + canonical regular (reg)
static void lag_to_canonical(Key* pk, const FrB* lag, FrB* brev, FrB* reg, hipStream_t st) {
    dcopy(brev, lag, pk->n * 32, st);
    plk::ntt(pk->d0, brev, 1, 0, 0, st);  // FFTInverse DIF: natural in -> bit-reversed out
    if (reg) plk::bit_reverse(brev, reg, pk->n, st);
}
// evaluations (natural order, m = n / S) of a canonical bit-reversed polynomial on
// a quotient unit's class: fold to m coefficients, then the coset FFT there
static void unit_eval(Key* pk, gg_domain_t dom, const uint32_t* kappa, const FrB* brev, FrB* out, hipStream_t st) {
    if (pk->S == 1) dcopy(out, brev, pk->n * 32, st);
    else {
        FrB k;
        memcpy(k.v, kappa, 32);
        plk::fold_brev(brev, pk->n, pk->S, k, out, st);
    }
    plk::ntt(dom, out, 0, 1, 1, st);  // FFT DIT on the coset: bit-reversed in -> natural out
}
// an event marking the work enqueued on `from` so far (events live as long as the key)
static hipEvent_t record(Key* pk, hipStream_t from) {
    if (pk->ev_next == pk->evs.size()) {
        hipEvent_t e;
        GG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        pk->evs.push_back(e);
    }
    hipEvent_t e = pk->evs[pk->ev_next++];
    GG_HIP(hipEventRecord(e, from));
    return e;
}
// `to` waits for the work enqueued on `from` so far
static void record_wait(Key* pk, hipStream_t from, hipStream_t to) {
    if (from == to) return;
    GG_HIP(hipStreamWaitEvent(to, record(pk, from), 0));
}
// a peer part's share of an MSM: its scalar slice copied from the primary GPU
// (xGMI peer copy), its resident base slice
static double ms_since(std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
}
// (resident: the slice is already in the peer's slot, e.g. its slice of Z)
static BJac peer_msm(Key* pk, int part, PlonkPeer* p, bool kzg, int wi, const FrB* scal, bool resident = false) {
    GG_HIP(hipSetDevice(p->device));
    const size_t lo = kzg ? p->k_lo : p->l_lo, hi = kzg ? p->k_hi : p->l_hi;
    BJac j = BJac::inf();
    if (hi == lo) return j;
    const auto a = std::chrono::steady_clock::now();
    GG_HIP(hipEventRecord(p->ea[wi], p->s[wi]));
    if (!resident)
        GG_HIP(hipMemcpyPeerAsync(p->scal[wi].p, p->device, scal + lo, pk->device, 32 * (hi - lo), p->s[wi]));
    GG_HIP(hipEventRecord(p->eb[wi], p->s[wi]));
    msm_device_work(kzg ? p->kzg : p->kzg_lag, p->work[wi], p->scal[wi].as<Fr>(), &j, p->s[wi]);
    float cp = 0;
    GG_HIP(hipEventElapsedTime(&cp, p->ea[wi], p->eb[wi]));  // the MSM synchronised the stream
    std::lock_guard<std::mutex> lk(pk->tmu);
    if ((size_t)part >= pk->ptimes.size()) return j;  // outside a proof (key setup)
    PlonkPartTimes& T = pk->ptimes[part];
    T.msm_count += 1;
    T.msm_ms += ms_since(a);
    T.scalar_copy_ms += cp;
    if (!resident) T.scalar_mb += 32.0 * (hi - lo) / 1e6;
    return j;
}
static bool plonk_solo(Key* pk) { return pk->solo; }
// does device part `part` (0 = primary) do its work in this proof (a rehearsal
// keeps only one part busy)
static bool part_runs(const Key* pk, int part) { return !pk->solo || pk->solo_part == part; }
// the multi-part protocol: peers exist and at least one of them works
static bool peers_active(const Key* pk) { return !pk->peers.empty() && (!pk->solo || pk->solo_part > 0); }
// this rank's partial MSM (the whole MSM on one GPU, or split over the key's
// device parts and summed here); red() completes a process shard's partial
static BJac msm_jac(Key* pk, gg_msm_base_t base, int wi, const FrB* scal, hipStream_t st,
                    bool peer_resident = false) {
    BJac j = BJac::inf();
    const bool kz = base == pk->kzg;
    const size_t lo = kz ? pk->k_lo : pk->l_lo;
    std::vector<gg::Task<BJac>> fs;
    if (peers_active(pk)) {
        // the peers' threads start at once; each waits for the scalars (complete
        // at this point of st) before its copy -- not for a resident slice
        hipEvent_t ready = pk->msm_ready[wi];
        GG_HIP(hipEventRecord(ready, st));
        for (size_t q = 0; q < pk->peers.size(); q++)
            if (part_runs(pk, (int)q + 1))
                fs.push_back(gg::run_task([pk, q, pp = pk->peers[q].get(), kz, wi, scal, peer_resident,
                                                             ready] {
                    if (!peer_resident) GG_WAIT_EVENT(ready);
                    return peer_msm(pk, (int)q + 1, pp, kz, wi, scal, peer_resident);
                }));
    }
    const auto a = std::chrono::steady_clock::now();
    if (part_runs(pk, 0)) msm_device_work(base, pk->work[wi], (const Fr*)(scal + lo), &j, st);
    const double own = ms_since(a);
    const auto w = std::chrono::steady_clock::now();
    for (auto& f : fs) j = jac_add(j, f.get());
    const double waited = ms_since(w);
    if (!pk->ptimes.empty()) {
        std::lock_guard<std::mutex> lk(pk->tmu);
        PlonkPartTimes& T = pk->ptimes[0];
        if (part_runs(pk, 0)) {
            T.msm_count += 1;
            T.msm_ms += own;
        }
        T.wait_ms += waited;
    }
    return j;
}
// kzg.Commit(p, pk.Kzg) of a buffer of n + 3 scalars (zero beyond the polynomial)
static BJac commit_kzg(Key* pk, int wi, const FrB* scal, hipStream_t st) { return msm_jac(pk, pk->kzg, wi, scal, st); }

// Same-base commitments batched (commitToLRO on pk.KzgLagrange, prove.go:425-502;
// commitToQuotient on pk.Kzg, :1199-1218): every part runs ONE MSM over its
// base slice for all nv scalar vectors (gg_msm_batch: one sort, accumulation,
// level 2 and reduction) in work slot 0; the scalars are complete on st.
// GG_PLONK_BATCH=0 keeps three MSMs on three streams.
static bool plonk_batch() {
    static const bool on = !(getenv("GG_PLONK_BATCH") && atoi(getenv("GG_PLONK_BATCH")) == 0);
    return on;
}
// the batch on every part's slice of the base fits the sort's 32-bit words
// (gg_msm_batch_shape); else the three MSMs run one per stream
static bool batch_ok(Key* pk, bool kzg, int nv) {
    if (!plonk_batch()) return false;
    if (!msm_base_batch_fits(kzg ? pk->kzg : pk->kzg_lag, nv)) return false;
    for (auto& p : pk->peers)
        if (!msm_base_batch_fits(kzg ? p->kzg : p->kzg_lag, nv)) return false;
    return true;
}
static void peer_msm_batch(Key* pk, int part, PlonkPeer* p, bool kzg, const FrB* const* scal, int nv, BJac* out) {
    GG_HIP(hipSetDevice(p->device));
    const size_t lo = kzg ? p->k_lo : p->l_lo, hi = kzg ? p->k_hi : p->l_hi;
    for (int v = 0; v < nv; v++) out[v] = BJac::inf();
    if (hi == lo) return;
    const auto a = std::chrono::steady_clock::now();
    hipStream_t q = p->s[0];
    GG_HIP(hipEventRecord(p->ea[0], q));
    const Fr* sv[4];
    void* ov[4];
    for (int v = 0; v < nv; v++) {
        GG_HIP(hipMemcpyPeerAsync(p->scal[v].p, p->device, scal[v] + lo, pk->device, 32 * (hi - lo), q));
        sv[v] = p->scal[v].as<Fr>();
        ov[v] = &out[v];
    }
    GG_HIP(hipEventRecord(p->eb[0], q));
    msm_device_work_batch(kzg ? p->kzg : p->kzg_lag, p->work[0], sv, nv, ov, q);
    float cp = 0;
    GG_HIP(hipEventElapsedTime(&cp, p->ea[0], p->eb[0]));  // the MSM synchronised the stream
    std::lock_guard<std::mutex> lk(pk->tmu);
    if ((size_t)part >= pk->ptimes.size()) return;
    PlonkPartTimes& T = pk->ptimes[part];
    T.msm_count += nv;
    T.msm_ms += ms_since(a);
    T.scalar_copy_ms += cp;
    T.scalar_mb += 32.0 * (hi - lo) * nv / 1e6;
}
static void msm_jac_batch(Key* pk, gg_msm_base_t base, const FrB* const* scal, int nv, hipStream_t st, BJac* out) {
    const bool kz = base == pk->kzg;
    const size_t lo = kz ? pk->k_lo : pk->l_lo;
    for (int v = 0; v < nv; v++) out[v] = BJac::inf();
    std::vector<gg::Task<std::vector<BJac>>> fs;
    if (peers_active(pk)) {
        hipEvent_t ready = pk->msm_ready[0];
        GG_HIP(hipEventRecord(ready, st));
        std::vector<const FrB*> sc(scal, scal + nv);
        for (size_t q = 0; q < pk->peers.size(); q++)
            if (part_runs(pk, (int)q + 1))
                fs.push_back(gg::run_task([pk, q, pp = pk->peers[q].get(), kz, sc, nv, ready] {
                    GG_WAIT_EVENT(ready);
                    std::vector<BJac> r(nv);
                    peer_msm_batch(pk, (int)q + 1, pp, kz, sc.data(), nv, r.data());
                    return r;
                }));
    }
    const auto a = std::chrono::steady_clock::now();
    if (part_runs(pk, 0)) {
        const Fr* sv[4];
        void* ov[4];
        for (int v = 0; v < nv; v++) {
            sv[v] = (const Fr*)(scal[v] + lo);
            ov[v] = &out[v];
        }
        msm_device_work_batch(base, pk->work[0], sv, nv, ov, st);
    }
    const double own = ms_since(a);
    const auto w = std::chrono::steady_clock::now();
    for (auto& f : fs) {
        const std::vector<BJac> r = f.get();
        for (int v = 0; v < nv; v++) out[v] = jac_add(out[v], r[v]);
    }
    const double waited = ms_since(w);
    if (!pk->ptimes.empty()) {
        std::lock_guard<std::mutex> lk(pk->tmu);
        PlonkPartTimes& T = pk->ptimes[0];
        if (part_runs(pk, 0)) {
            T.msm_count += nv;
            T.msm_ms += own;
        }
        T.wait_ms += waited;
    }
}
// sum of the ranks' partials (called in one fixed order on every rank)
static BJac red(Key* pk, BJac j) {
    if (pk->world == 1) return j;
    GG_CHECK(pk->reduce(pk->reduce_ctx, &j) == 0, GG_ERR_DEVICE, "commitment reduce callback failed");
    return j;
}
// commitBlindingFactor (prove.go:1159-1172): sum_j b_j (G1[n + j] - G1[j])
static BJac blind_commit(Key* pk, const std::vector<FrB>& b) {
    BJac acc = BJac::inf();
    for (size_t j = 0; j < b.size(); j++) {
        acc = jac_add(acc, jmul(pk->blind_hi[j], b[j]));
        acc = jac_add(acc, jmul(pk->blind_lo[j], -b[j]));
    }
    return acc;
}
static FrB fetch(const FrB* dev, hipStream_t st) {
    FrB v;
    GG_HIP(hipMemcpyAsync(v.v, dev, 32, hipMemcpyDeviceToHost, st));
    GG_WAIT_STREAM(st);
    return v;
}
static FrB eval_dev(Key* pk, const FrB* f, size_t len, const FrB& a, FrB* q, FrB* slot, int ai, hipStream_t st) {
    pk->ar[ai].reset();
    plk::horner(f, len, a, q, slot, st, pk->ar[ai]);
    return fetch(slot, st);
}

// evaluations of `count` polynomials at a (plk::eval_many) read back at once
static std::vector<FrB> eval_batch(Key* pk, const FrB* const* f, const size_t* len, int count, const FrB& a,
                                   FrB* slot, int ai, hipStream_t st) {
    pk->ar[ai].reset();
    plk::eval_many(f, len, count, a, slot, st, pk->ar[ai]);
    std::vector<FrB> v(count);
    GG_HIP(hipMemcpyAsync(v.data(), slot, 32 * (size_t)count, hipMemcpyDeviceToHost, st));
    GG_WAIT_STREAM(st);
    return v;
}

// The canonical forms of a multi-part key's per-proof polynomials are taken on
// the peers: task i (PlonkPeer::in index: 0..2 L R O, 4 Qk, 5 + j Pi_j, then 3 Z,
// which is complete only after the ratio) runs on peer i mod (N - 1); its owner
// pushes the bit-reversed form to every peer with quotient units and both forms
// to part 0, so part 0 runs no size-n transform of its own and no polynomial
// leaves it whole.
static std::vector<int> canon_tasks(const Key* pk) {
    std::vector<int> t = {0, 1, 2, 4};
    for (int j = 0; j < pk->n_cmt; j++) t.push_back(5 + j);
    t.push_back(3);
    return t;
}
static PlonkPeer* canon_owner(const Key* pk, size_t i) { return pk->peers[i % pk->peers.size()].get(); }

// one canonical-form task on peer pi: `fill` leaves the polynomial's Lagrange
// form in p->in[b] (ordered on p->cs); the size-n inverse DIF there (canonical
// bit-reversed, in place), the regular form in creg when part 0 needs it, then the
// pushes, each on its own stream (one xGMI link each): bit-reversed to every other
// peer with quotient units and to brev0 on part 0, regular to reg0.  Returns once
// the bit-reversed form is everywhere (the quotient units need it next); the
// regular push (the openings need it, much later) stays in flight behind
// p->reg_ev, which canon_wait_regular and the owner's next task wait for.
static void canon_run(Key* pk, size_t pi, int b, FrB* brev0, FrB* reg0, const std::function<void(hipStream_t)>& fill) {
    PlonkPeer* p = pk->peers[pi].get();
    const size_t n = pk->n, nb = 32 * n;
    GG_HIP(hipSetDevice(p->device));
    const auto a = std::chrono::steady_clock::now();
    hipStream_t q = p->cs;
    if (p->reg_pending) {  // creg is read by the previous task's regular push
        GG_WAIT_EVENT(p->reg_ev);
        p->reg_pending = false;
    }
    fill(q);
    plk::ntt(p->d0, p->in[b].p, 1, 0, 0, q);  // FFTInverse DIF: natural in -> bit-reversed out
    if (reg0) plk::bit_reverse(F(p->in[b]), F(p->creg), n, q);
    GG_WAIT_STREAM(q);
    size_t x = 0;
    double mb = 0;
    for (auto& o : pk->peers)
        if (o.get() != p && !o->units.empty()) {
            GG_HIP(hipMemcpyPeerAsync(o->in[b].p, o->device, p->in[b].p, p->device, nb, p->xs[x++]));
            mb += nb / 1e6;
        }
    GG_HIP(hipMemcpyPeerAsync(brev0, pk->device, p->in[b].p, p->device, nb, p->xs[x++]));
    if (reg0) {
        hipStream_t r = p->xs[x];
        GG_HIP(hipMemcpyPeerAsync(reg0, pk->device, p->creg.p, p->device, nb, r));
        GG_HIP(hipEventRecord(p->reg_ev, r));
        p->reg_pending = true;
    }
    mb += (reg0 ? 2.0 : 1.0) * nb / 1e6;
    for (size_t i = 0; i < x; i++) GG_WAIT_STREAM(p->xs[i]);
    std::lock_guard<std::mutex> lk(pk->tmu);
    PlonkPartTimes& T = pk->ptimes[pi + 1];
    T.canon_count += 1;
    T.canon_ms += ms_since(a);
    T.canon_mb += mb;
}

// every owner's last regular-form push to part 0 has landed (before the openings)
static void canon_wait_regular(Key* pk) {
    for (auto& pp : pk->peers) {
        PlonkPeer* p = pp.get();
        if (!p->reg_pending) continue;
        GG_WAIT_EVENT(p->reg_ev);
        p->reg_pending = false;
    }
}

// Each device part's share of the KZG slices (both bases, the ratio, Z's
// slices).  Beside its MSM slices part 0 runs the quotient's tail stages and
// the openings, a peer its canonical-form tasks (canon_tasks; Z's transform and
// pushes sit between the ratio and the quotient units).  With E_p that extra
// work as a fraction of the one-GPU MSM work, the shares f_p = (1 + sum E) / N
// - E_p equalise f_p + E_p.  E from the parts rehearsed alone at 2^22 x 8
// (profiles/r04_l_bench_driver_command.json: parts without tasks 23.1 ms, with
// L / R / O / Qk +0.0-0.7, Z's owner +0.9, part 0 +2.3 at equal-MSM terms;
// MSM work ~120 ms): part 0 0.019, a task 0.0033, Z's 0.0075.
// GG_PLONK_PART0_WEIGHT=w instead: part 0 weight w, every peer 1.
static std::vector<double> plonk_part_shares(int n_devices, int n_cmt) {
    std::vector<double> f(std::max(1, n_devices), 1.0);
    if (n_devices > 1) {
        if (const char* e = getenv("GG_PLONK_PART0_WEIGHT")) {  // tuning / A/B
            const double w = atof(e);
            if (w > 0.05 && w <= 4.0) f[0] = w;
        } else {
            std::vector<double> E(n_devices, 0.0);
            E[0] = 0.019;
            const int T = 5 + n_cmt;  // canon_tasks order: L R O Qk Pi_j..., Z last
            for (int i = 0; i < T; i++) E[1 + i % (n_devices - 1)] += (i == T - 1) ? 0.0075 : 0.0033;
            double sum = 0;
            for (double x : E) sum += x;
            for (int p = 0; p < n_devices; p++) f[p] = std::max(0.3 / n_devices, (1.0 + sum) / n_devices - E[p]);
        }
    }
    double tot = 0;
    for (double x : f) tot += x;
    for (double& x : f) x /= tot;
    return f;
}

// GG_PLONK_PART_QUEUES=1: device parts' task streams on dedicated hardware queues
static bool part_queues_enabled() {
    const char* e = getenv("GG_PLONK_PART_QUEUES");
    return e && atoi(e) == 1;
}
// part q's four task slots on dedicated queues or their own streams (between
// proofs; no stream is created or destroyed: common.h TaskQueue)
static void restream_part(Key* pk, int q, bool dedicated) {
    if (q == 0) task_streams_switch(pk->act, pk->tq, 4, pk->device, dedicated);
    else task_streams_switch(pk->peers[q - 1]->act, pk->peers[q - 1]->tq, 4, pk->peers[q - 1]->device, dedicated);
}
// the queue layout for a rehearsal of `part` (-1: none): its device's dedicated
// queues go to it, as on a node where it is alone on its GPU; -1 restores the
// creation layout (every part released first, then re-created in part order)
static void queue_layout(Key* pk, int part) {
    if (!pk->part_queues || part == pk->queue_owner) return;
    int cur = 0;
    GG_HIP(hipGetDevice(&cur));
    const int np = 1 + (int)pk->peers.size();
    auto dev_of = [&](int q) { return q == 0 ? pk->device : pk->peers[q - 1]->device; };
    if (part >= 0) {
        for (int q = 0; q < np; q++)
            if (q != part && dev_of(q) == dev_of(part)) restream_part(pk, q, false);
        restream_part(pk, part, true);
    } else {  // the creation layout: dedicated queues in part order while they last
        for (int q = 0; q < np; q++) restream_part(pk, q, false);
        for (int q = 0; q < np; q++) restream_part(pk, q, true);
    }
    pk->queue_owner = part;
    GG_HIP(hipSetDevice(cur));
}

static void plonk_pk_build(Key* pk, int log_n, int log_big, const void* omega, const void* omega_big,
                           const void* coset_shift, const void* kzg_g1, size_t n_kzg,
                           const void* kzg_lagrange_g1, const void* const* trace, const void* const* qcp,
                           int n_cmt, const int64_t* perm, size_t nb_public, const uint64_t* cmt_idx,
                           const void* vk_digests, int rank, int world, gg_g1_reduce_fn reduce, void* rctx,
                           const int* devices = nullptr, int n_devices = 1) {
    GG_CHECK(world >= 1 && rank >= 0 && rank < world && (world == 1 || reduce), GG_ERR_INVALID_ARG,
             "bad shard (rank, world) or missing reduce callback");
    GG_CHECK(n_devices >= 1 && n_devices <= 64 && (n_devices == 1 || (devices && world == 1)), GG_ERR_INVALID_ARG,
             "device parts: 1..64 devices, not combined with process shards");
    pk->rank = rank;
    pk->world = world;
    pk->reduce = reduce;
    pk->reduce_ctx = rctx;
    GG_CHECK(log_n >= 1 && log_n <= 27 && log_big > log_n && log_big - log_n <= 3 && log_big <= 30,
             GG_ERR_INVALID_ARG, "need 2 <= n, |big| / n in {2, 4, 8}");
    GG_CHECK(omega && omega_big && coset_shift && kzg_g1 && kzg_lagrange_g1 && trace && perm, GG_ERR_INVALID_ARG,
             "null argument");
    GG_CHECK(n_cmt >= 0 && n_cmt <= plk::MAX_CMT && (n_cmt == 0 || (qcp && cmt_idx)), GG_ERR_INVALID_ARG,
             "0..8 BSB22 commitments with their Qcp polynomials and constraint indexes");
    pk->log_n = log_n;
    pk->log_big = log_big;
    pk->n = (size_t)1 << log_n;
    pk->big = (size_t)1 << log_big;
    pk->rho = pk->big / pk->n;
    const size_t n = pk->n, nb = 32 * n;
    GG_CHECK(n_kzg >= n + 3, GG_ERR_INVALID_ARG, "len(pk.Kzg.G1) < n + 3 (setup.go:150)");
    GG_CHECK(nb_public < n, GG_ERR_INVALID_ARG, "nb_public >= n");
    pk->nb_public = nb_public;
    pk->n_cmt = n_cmt;
    for (int i = 0; i < n_cmt; i++) {
        GG_CHECK(nb_public + cmt_idx[i] < n, GG_ERR_INVALID_ARG, "commitment constraint index out of range");
        pk->cmt_idx.push_back(cmt_idx[i]);
    }
    if (n_devices > 1) {
        int ndev = 0;
        GG_HIP(hipGetDeviceCount(&ndev));
        for (int d = 0; d < n_devices; d++)
            GG_CHECK(devices[d] >= 0 && devices[d] < ndev, GG_ERR_INVALID_ARG, "device id out of range");
        GG_HIP(hipSetDevice(devices[0]));
        // xGMI peer access between the distinct devices (copies work without it,
        // staged through host memory: kept per pair, gg_plonk_pk_peer_access)
        pk->peer_codes = gg::enable_peer_access(std::vector<int>(devices, devices + n_devices));
        GG_HIP(hipSetDevice(devices[0]));
    }
    GG_HIP(hipGetDevice(&pk->device));
    memcpy(pk->omega.v, omega, 32);
    memcpy(pk->omega_big.v, omega_big, 32);
    memcpy(pk->u.v, coset_shift, 32);
    pk->n_inv = inverse(frv(n));
    GG_CHECK(pow_u64(pk->omega_big, pk->rho) == pk->omega, GG_ERR_INVALID_ARG, "omega_big^(|big|/n) != omega");
    auto dom = [&](int lg, const FrB& w, const FrB& g) {
        gg_domain_t d;
        int rc = gg_domain_create_ex(Cv::curve, lg, w.v, g.v, &d);
        GG_CHECK(rc == GG_OK, rc, gg_last_error());
        return d;
    };
    pk->d0 = dom(log_n, pk->omega, pk->u);
    pk->d1 = dom(log_big, pk->omega_big, pk->u);
    FrB sh = pk->u;
    for (size_t i = 0; i < pk->rho; i++) {  // coset i of the big domain: shift u w_big^i
        pk->coset_shift.push_back(sh);
        sh = sh * pk->omega_big;
    }
    // quotient units: U = rho S classes, S the largest power of two with U <= the
    // device parts (and <= 16, m = n / S >= 16); unit p runs on part p mod N
    pk->n_parts = n_devices > 1 ? n_devices : 1;
    pk->S = 1;
    while ((size_t)pk->rho * pk->S * 2 <= (size_t)pk->n_parts && pk->rho * pk->S * 2 <= 16 && n / (pk->S * 2) >= 16)
        pk->S *= 2;
    pk->U = (int)pk->rho * pk->S;
    pk->log_u = 0;
    while ((1 << pk->log_u) < pk->U) pk->log_u++;
    pk->split_idft = log_big >= 12;
    // a one-device key's four streams on hardware queues of their own (common.h
    // TaskQueue: 125.9 vs 127.5-128.1 ms at 2^22, profiles/r05_l_*); a key with
    // device parts on them only with GG_PLONK_PART_QUEUES=1 (r05k's stall, in the
    // stream re-creation its rehearsal did then: DESIGN.md §5)
    pk->part_queues = n_devices > 1 && part_queues_enabled();
    task_streams_init(pk->act, pk->tq, 4, pk->device, n_devices <= 1 || pk->part_queues);
    for (auto& w : pk->work) w = msm_work_new();
    for (hipEvent_t& e : pk->msm_ready) GG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipStream_t st = pk->s[0];
    // KZG bases (resident, fixed-base precomputation): pk.Kzg.G1[:n+3], pk.KzgLagrange.G1
    {
        auto range = [&](size_t m, size_t& lo, size_t& hi) {  // dist.shard_range
            lo = m * (size_t)pk->rank / (size_t)pk->world;
            hi = m * (size_t)(pk->rank + 1) / (size_t)pk->world;
        };
        // device parts: slice boundaries by share (plonk_part_shares)
        const std::vector<double> share = plonk_part_shares(n_devices, n_cmt);
        // the window of the parts' KZG slices (0 = the cost model's choose_c);
        // GG_PLONK_PART_WINDOW forces one (A/B of the per-part bucket reductions)
        const int part_c = [&] {
            const char* e = getenv("GG_PLONK_PART_WINDOW");
            return n_devices > 1 && e ? std::max(0, std::min(atoi(e), 23)) : 0;
        }();
        auto bound = [&](size_t m, int d) -> size_t {
            if (d <= 0) return 0;
            if (d >= n_devices) return m;
            long double cum = 0;
            for (int q = 0; q < d; q++) cum += share[q];
            return std::min(m, (size_t)((long double)m * cum));
        };
        if (n_devices > 1) {  // part 0 here, parts 1.. on the peers
            for (int d = 1; d < n_devices; d++) {
                pk->peers.emplace_back(new PlonkPeer());
                PlonkPeer* p = pk->peers.back().get();
                p->device = devices[d];
                p->k_lo = bound(n + 3, d);
                p->k_hi = bound(n + 3, d + 1);
                p->l_lo = bound(n, d);
                p->l_hi = bound(n, d + 1);
                GG_HIP(hipSetDevice(p->device));
                task_streams_init(p->act, p->tq, 4, p->device, pk->part_queues);
                gg::create_copy_stream(&p->cps);
                GG_HIP(hipEventCreateWithFlags(&p->cpev, hipEventDisableTiming));
                for (int e = 0; e < 4; e++) {
                    GG_HIP(hipEventCreate(&p->ea[e]));
                    GG_HIP(hipEventCreate(&p->eb[e]));
                }
                for (auto& w : p->work) w = msm_work_new();
                for (auto& b : p->scal) b.alloc(32 * std::max<size_t>(1, std::max(p->k_hi - p->k_lo, p->l_hi - p->l_lo)));
                int rc = gg_msm_base_create(Cv::group, (const uint8_t*)kzg_g1 + PT * p->k_lo, p->k_hi - p->k_lo,
                                            0, nullptr, part_c, &p->kzg);
                GG_CHECK(rc == GG_OK, rc, gg_last_error());
                rc = gg_msm_base_create(Cv::group, (const uint8_t*)kzg_lagrange_g1 + PT * p->l_lo,
                                        p->l_hi - p->l_lo, 0, nullptr, part_c, &p->kzg_lag);
                GG_CHECK(rc == GG_OK, rc, gg_last_error());
            }
            GG_HIP(hipSetDevice(pk->device));
            pk->k_lo = 0;
            pk->k_hi = bound(n + 3, 1);
            pk->l_lo = 0;
            pk->l_hi = bound(n, 1);
        } else {
            range(n + 3, pk->k_lo, pk->k_hi);
            range(n, pk->l_lo, pk->l_hi);
        }
        int rc = gg_msm_base_create(Cv::group, (const uint8_t*)kzg_g1 + PT * pk->k_lo, pk->k_hi - pk->k_lo, 0,
                                    nullptr, part_c, &pk->kzg);
        GG_CHECK(rc == GG_OK, rc, gg_last_error());
        rc = gg_msm_base_create(Cv::group, (const uint8_t*)kzg_lagrange_g1 + PT * pk->l_lo,
                                pk->l_hi - pk->l_lo, 0, nullptr, part_c, &pk->kzg_lag);
        GG_CHECK(rc == GG_OK, rc, gg_last_error());
        const uint8_t* g = (const uint8_t*)kzg_g1;
        for (int j = 0; j < 3; j++) {
            memcpy(&pk->blind_lo[j], g + PT * j, PT);
            memcpy(&pk->blind_hi[j], g + PT * (n + j), PT);
        }
    }
    // trace polynomials
    for (int k = 0; k < Key::NTRACE; k++) {
        GG_CHECK(trace[k], GG_ERR_INVALID_ARG, "null trace polynomial");
        pk->reg[k].alloc(nb);
        pk->brev[k].alloc(nb);
        up(pk->reg[k].p, trace[k], nb, false, st);
        to_brev(pk, F(pk->reg[k]), F(pk->brev[k]), st);
    }
    pk->qcp_reg.resize(n_cmt);
    pk->qcp_brev.resize(n_cmt);
    for (int i = 0; i < n_cmt; i++) {
        GG_CHECK(qcp[i], GG_ERR_INVALID_ARG, "null Qcp polynomial");
        pk->qcp_reg[i].alloc(nb);
        pk->qcp_brev[i].alloc(nb);
        up(pk->qcp_reg[i].p, qcp[i], nb, false, st);
        to_brev(pk, F(pk->qcp_reg[i]), F(pk->qcp_brev[i]), st);
    }
    // Qk in Lagrange regular form (completeQk: trace.Qk.Clone().ToLagrange().ToRegular())
    {
        DevBuf t(nb);
        dcopy(t.p, pk->reg[Key::QK].p, nb, st);
        plk::ntt(pk->d0, t.p, 0, 0, 0, st);  // FFT DIF: natural in -> bit-reversed out
        pk->qk_lag.alloc(nb);
        plk::bit_reverse(F(t), F(pk->qk_lag), n, st);
        GG_WAIT_STREAM(st);
    }
    // s.twiddles0 = w^j: DIT FFT of the coefficients of X (bit-reversed layout)
    // (every upload below is ordered on st and waited for: a plain hipMemcpy runs
    // on the null stream, which does not order against the non-blocking st)
    pk->tw0.alloc(nb);
    zero(pk->tw0.p, nb, st);
    const FrB one = FrB::one();
    GG_HIP(hipMemcpyAsync(F(pk->tw0) + n / 2, one.v, 32, hipMemcpyHostToDevice, st));
    GG_WAIT_STREAM(st);
    plk::ntt(pk->d0, pk->tw0.p, 0, 1, 0, st);
    // resident coset evaluations of the key's polynomials (the reference redoes
    // these 2 rho FFTs per polynomial per proof, prove.go:995-1017)
    DevBuf xb(nb), lone(nb);
    zero(xb.p, nb, st);
    GG_HIP(hipMemcpyAsync(F(xb) + n / 2, one.v, 32, hipMemcpyHostToDevice, st));  // X, bit-reversed
    {
        std::vector<FrB> v(n, pk->n_inv);  // LOne canonical: 1/n everywhere
        GG_HIP(hipMemcpyAsync(lone.p, v.data(), nb, hipMemcpyHostToDevice, st));
        GG_WAIT_STREAM(st);
    }
    std::vector<const FrB*> srcs = {F(pk->brev[Key::QL]), F(pk->brev[Key::QR]),
                                    F(pk->brev[Key::QM]), F(pk->brev[Key::QO]),
                                    F(pk->brev[Key::S1]), F(pk->brev[Key::S2]),
                                    F(pk->brev[Key::S3]), F(xb), F(lone)};
    for (int i = 0; i < n_cmt; i++) srcs.push_back(F(pk->qcp_brev[i]));
    GG_WAIT_STREAM(st);
    // quotient units: domains, resident key evaluations on the class, twiddles0 there
    const size_t m = n / pk->S, mb = 32 * m;
    const FrB wS = pow_u64(pk->omega, (uint64_t)pk->S);
    for (int p = 0; p < pk->U; p++) {
        const int part = p % pk->n_parts;
        PlonkPeer* peer = part ? pk->peers[part - 1].get() : nullptr;
        std::unique_ptr<QUnit> up_(new QUnit());
        QUnit* q = up_.get();
        q->p = p;
        q->device = peer ? peer->device : pk->device;
        GG_HIP(hipSetDevice(q->device));
        hipStream_t qs = peer ? peer->s[3] : st;
        const FrB sp = pk->u * pow_u64(pk->omega_big, (uint64_t)p);
        const FrB spz = pk->u * pow_u64(pk->omega_big, (uint64_t)((p + (int)pk->rho) % pk->U));
        const FrB kap = pow_u64(sp, m), zkap = pow_u64(spz, m);
        const FrB den = inverse(pow_u64(pk->coset_shift[p % pk->rho], n) - FrB::one());
        GG_CHECK(!(pow_u64(pk->coset_shift[p % pk->rho], n) == FrB::one()), GG_ERR_INVALID_ARG,
                 "x^n - 1 vanishes on the big coset");
        memcpy(q->kappa, kap.v, 32);
        memcpy(q->zkappa, zkap.v, 32);
        memcpy(q->inv_den, den.v, 32);
        q->dom = dom(log_n - (pk->log_u - (int)(pk->log_big - pk->log_n)), wS, sp);
        if (pk->S > 1) q->zdom = dom(log_n - (pk->log_u - (int)(pk->log_big - pk->log_n)), wS, spz);
        if (peer && !peer->tw0.p) {  // the peer's per-proof buffers, once
            peer->tw0.alloc(nb);
            GG_HIP(hipMemcpyPeerAsync(peer->tw0.p, peer->device, pk->tw0.p, pk->device, nb, qs));
            for (int k = 0; k < 5 + n_cmt; k++) peer->in[k].alloc(nb);
            for (int k = 0; k < 7 + n_cmt; k++)
                if (k != 4 && k != 5) peer->cev[k].alloc(mb);
            if (pk->S > 1) peer->zc.alloc(mb);
        }
        for (size_t k = 0; k < srcs.size(); k++) {
            q->ev.emplace_back(mb);
            const FrB* src = srcs[k];
            if (peer) {  // the key polynomial to the peer (staged in its input buffer), evaluated there
                GG_HIP(hipMemcpyPeerAsync(peer->in[0].p, peer->device, src, pk->device, nb, qs));
                src = F(peer->in[0]);
            }
            unit_eval(pk, q->dom, q->kappa, src, F(q->ev.back()), qs);
        }
        if (pk->S > 1) {  // twiddles0 at the class's points w^(s + S j) and the next ones (ZS)
            const FrB* t0 = peer ? F(peer->tw0) : F(pk->tw0);
            q->tw0.alloc(mb);
            q->tw1.alloc(mb);
            plk::gather_strided(t0, n, pk->S, p / (int)pk->rho, F(q->tw0), qs);
            plk::gather_strided(t0, n, pk->S, p / (int)pk->rho + 1, F(q->tw1), qs);
        }
        if (peer) q->out.alloc(mb);
        GG_WAIT_STREAM(qs);
        (peer ? peer->units : pk->units).push_back(std::move(up_));
    }
    // peers: the permutation's columns over their KzgLagrange slice, for their share of the ratio
    for (auto& pp : pk->peers) {
        PlonkPeer* p = pp.get();
        const size_t cnt = p->l_hi - p->l_lo;
        if (!cnt) continue;
        GG_HIP(hipSetDevice(p->device));
        p->perm_slice.alloc(3 * cnt * 8);
        for (int j = 0; j < 3; j++)
            up(p->perm_slice.as<int64_t>() + j * cnt, perm + (size_t)j * n + p->l_lo, cnt * 8, false, p->s[0]);
        p->pz.alloc(32 * cnt);
        p->ar.reserve(plk::ratio_range_arena_bytes(n, cnt) + 65536);
        GG_WAIT_STREAM(p->s[0]);
    }
    // peers: the canonical-form tasks (canon_tasks) -- a size-n domain, the regular
    // form's buffer and push streams on each owner, Qk in Lagrange form on Qk's
    if (!pk->peers.empty()) {
        const std::vector<int> tasks = canon_tasks(pk);
        for (size_t i = 0; i < tasks.size(); i++) {
            PlonkPeer* p = canon_owner(pk, i);
            GG_HIP(hipSetDevice(p->device));
            if (!p->in[0].p)
                for (int k = 0; k < 5 + n_cmt; k++) p->in[k].alloc(nb);
            if (!p->d0) {
                p->d0 = dom(log_n, pk->omega, pk->u);
                p->creg.alloc(nb);
                p->xs.resize(pk->peers.size() + 2);
                for (hipStream_t& x : p->xs) gg::create_copy_stream(&x);  // pushes: own hardware queues
                GG_HIP(hipEventCreateWithFlags(&p->reg_ev, hipEventDisableTiming));
                GG_HIP(hipStreamCreateWithFlags(&p->cs, hipStreamNonBlocking));
            }
            if (tasks[i] == 4) {
                p->qk_lag.alloc(nb);
                GG_HIP(hipMemcpyPeerAsync(p->qk_lag.p, p->device, pk->qk_lag.p, pk->device, nb, p->s[3]));
                GG_WAIT_STREAM(p->s[3]);
            }
        }
    }
    GG_HIP(hipSetDevice(pk->device));
    pk->perm.alloc(3 * n * 8);
    up(pk->perm.p, perm, 3 * n * 8, false, st);
    // per-proof buffers
    for (auto& b : pk->lag) b.alloc(nb);
    for (auto& b : pk->can) b.alloc(nb);
    for (auto& b : pk->cbrev) b.alloc(nb);
    pk->zlag.alloc(nb);
    pk->pz.alloc(nb);
    pk->qkc.alloc(nb);
    for (int i = 0; i < n_cmt; i++) {
        pk->pi_reg[i].alloc(nb);
        pk->pi_brev[i].alloc(nb);
    }
    for (auto& slot : pk->cev)
        for (int k = 0; k < 7 + n_cmt; k++)
            if (k != 4 && k != 5) slot[k].alloc(mb);  // 4 (ZS), 5 (beta X): formed in the numerator kernel
    if (pk->S > 1)
        for (auto& z : pk->zc) z.alloc(mb);
    pk->cres.alloc(32 * pk->big);
    const size_t nb3 = 32 * (n + 3);
    for (auto& b : pk->hpad) b.alloc(nb3);
    pk->bz.alloc(nb3);
    for (auto& b : pk->bl) b.alloc(nb3);
    pk->fold.alloc(nb3);
    pk->lin.alloc(nb3);
    pk->q1.alloc(nb3);
    pk->q2.alloc(nb3);
    pk->pad.alloc(nb3);
    pk->vals.alloc(32 * 64);
    const size_t ab = std::max(std::max(plk::ratio_arena_bytes(n), plk::horner_arena_bytes(n + 3)),
                               plk::eval_many_arena_bytes(n + 3, plk::EVAL_MAX)) + 65536;
    for (auto& a : pk->ar) a.reserve(ab);
    GG_WAIT_STREAM(st);
    // vk digests (commitTrace, setup.go:229-272) unless the caller has them
    pk->vkQcp.resize(n_cmt);
    if (vk_digests) {
        const uint8_t* d = (const uint8_t*)vk_digests;
        for (int k = 0; k < 3; k++) memcpy(&pk->vkS[k], d + PT * k, PT);
        for (int k = 0; k < 5; k++) memcpy(&pk->vkQ[k], d + PT * (3 + k), PT);
        for (int i = 0; i < n_cmt; i++) memcpy(&pk->vkQcp[i], d + PT * (8 + i), PT);
    } else {
        auto cm = [&](const DevBuf& reg) {
            zero(pk->pad.p, nb3, st);
            dcopy(pk->pad.p, reg.p, nb, st);
            return to_aff(red(pk, commit_kzg(pk, 0, F(pk->pad), st)));
        };
        for (int k = 0; k < 3; k++) pk->vkS[k] = cm(pk->reg[Key::S1 + k]);
        for (int k = 0; k < 5; k++) pk->vkQ[k] = cm(pk->reg[Key::QL + k]);
        for (int i = 0; i < n_cmt; i++) pk->vkQcp[i] = cm(pk->qcp_reg[i]);
    }
}

// ============================================================== prove

struct PlonkProof {
    BAff lro[3], z, h[3], batched_h, zs_h;
    std::vector<BAff> bsb22;
    std::vector<FrB> claimed;
    FrB zs_value;
};

// GG_PLONK_SERIAL=1: the concurrent MSM groups run one after another (A/B timing)
static std::launch msm_policy() {
    static const bool serial = getenv("GG_PLONK_SERIAL") && atoi(getenv("GG_PLONK_SERIAL"));
    return serial ? std::launch::deferred : std::launch::async;
}
// a commitment's MSM task: on a kept worker, or deferred to its get() (GG_PLONK_SERIAL)
template <class Fn>
static auto msm_task(Fn fn) {
    return gg::run_task(std::move(fn), msm_policy() == std::launch::deferred);
}

static void prove(Key* pk, const void* const lro_in[3], bool on_dev, const FrB* pub, size_t nb_pub,
           const void* const* cmt_values, const BAff* cmt_digests, const FrB* cmt_hashed, int n_cmt,
           const FrB* blinding, Hasher ch, Hasher fh, PlonkProof& P, double* tms) {
    const size_t n = pk->n, nb = 32 * n, nb3 = 32 * (n + 3);
    hipStream_t* s = pk->s;
    pk->ev_next = 0;
    pk->ptimes.assign(1 + pk->peers.size(), PlonkPartTimes());
    auto t0 = std::chrono::steady_clock::now();
    int tk = 0;
    auto mark = [&]() {
        if (!tms) return;
        auto t = std::chrono::steady_clock::now();
        tms[tk++] = std::chrono::duration<double, std::milli>(t - t0).count();
    };
    // blinding polynomials (initBlindingPolynomials, prove.go:295-302): orders 1, 1, 1, 2
    std::vector<FrB> bp[4];
    const int ord[4] = {1, 1, 1, 2};
    for (int q = 0, k = 0; q < 4; q++)
        for (int j = 0; j <= ord[q]; j++) bp[q].push_back(blinding ? blinding[k++] : fr_random());
    // ---- inputs: L, R, O (Lagrange regular) on streams 0..2
    hipEvent_t uploaded[3];
    for (int k = 0; k < 3; k++) {
        up(pk->lag[k].p, lro_in[k], nb, on_dev, s[k]);
        uploaded[k] = record(pk, s[k]);
    }
    const bool dz = !pk->peers.empty();
    const bool peers_on = peers_active(pk);
    const bool run0 = part_runs(pk, 0);  // part 0's own kernels (a peer's rehearsal skips them)
    // multi-part keys: the canonical forms on the peers (canon_tasks), L R O as
    // soon as uploaded, Qk and Pi_j at once; Z after the ratio
    const std::vector<int> ctasks = dz ? canon_tasks(pk) : std::vector<int>();
    std::vector<gg::Task<void>> cfut(pk->peers.size());  // per owner: its tasks before Z, in order
    if (peers_on) {
        for (size_t pi = 0; pi < pk->peers.size(); pi++) {
            std::vector<int> mine;
            for (size_t i = 0; i + 1 < ctasks.size(); i++)
                if (i % pk->peers.size() == pi) mine.push_back(ctasks[i]);
            if (mine.empty() || !part_runs(pk, (int)pi + 1)) continue;
            cfut[pi] = gg::run_task([&, pi, mine] {
                PlonkPeer* p = pk->peers[pi].get();
                for (int b : mine) {
                    if (b < 3)
                        canon_run(pk, pi, b, F(pk->cbrev[b]), F(pk->can[b]), [&](hipStream_t q) {
                            GG_WAIT_EVENT(uploaded[b]);
                            GG_HIP(hipMemcpyPeerAsync(p->in[b].p, p->device, pk->lag[b].p, pk->device, nb, q));
                        });
                    else if (b == 4)  // completeQk (prove.go:397-423) on its owner
                        canon_run(pk, pi, 4, F(pk->qkc), nullptr, [&](hipStream_t q) {
                            dcopy(p->in[4].p, p->qk_lag.p, nb, q);
                            if (nb_pub) GG_HIP(hipMemcpyAsync(p->in[4].p, pub, 32 * nb_pub, hipMemcpyHostToDevice, q));
                            for (int i = 0; i < n_cmt; i++)
                                GG_HIP(hipMemcpyAsync(F(p->in[4]) + pk->nb_public + pk->cmt_idx[i], cmt_hashed[i].v, 32,
                                                      hipMemcpyHostToDevice, q));
                        });
                    else
                        canon_run(pk, pi, b, F(pk->pi_brev[b - 5]), F(pk->pi_reg[b - 5]),
                                  [&](hipStream_t q) { up(p->in[b].p, cmt_values[b - 5], nb, false, q); });
                }
            }).share();
        }
    }
    // blinding commitments of L, R, O, Z on host threads while the GPU works
    gg::Task<BJac> fblind[4];
    for (int q = 0; q < 4; q++) fblind[q] = gg::run_task([pk, &bp, q] { return blind_commit(pk, bp[q]); });
    // ---- commitToLRO: three KZG MSMs on pk.KzgLagrange at once
    BJac lroj[3];
    {
        std::vector<gg::Task<void>> fs;
        if (batch_ok(pk, false, 3)) {
            // one batched MSM on s[0] once L, R, O are uploaded
            for (int k = 1; k < 3; k++) GG_HIP(hipStreamWaitEvent(s[0], uploaded[k], 0));
            fs.push_back(msm_task([&] {
                GG_HIP(hipSetDevice(pk->device));
                const FrB* sc[3] = {F(pk->lag[0]), F(pk->lag[1]), F(pk->lag[2])};
                msm_jac_batch(pk, pk->kzg_lag, sc, 3, s[0], lroj);
            }));
        } else {
            for (int k = 0; k < 3; k++)
                fs.push_back(msm_task([&, k] {
                    GG_HIP(hipSetDevice(pk->device));
                    lroj[k] = msm_jac(pk, pk->kzg_lag, k, F(pk->lag[k]), s[k]);
                }));
        }
        // meanwhile on stream 3 (one part; with peers: canon_tasks): completeQk
        // (prove.go:397-423) and the BSB22 Pi_i
        if (!dz) {
            hipStream_t q = s[3];
            dcopy(pk->qkc.p, pk->qk_lag.p, nb, q);
            if (nb_pub) GG_HIP(hipMemcpyAsync(pk->qkc.p, pub, 32 * nb_pub, hipMemcpyHostToDevice, q));
            for (int i = 0; i < n_cmt; i++)
                GG_HIP(hipMemcpyAsync(F(pk->qkc) + pk->nb_public + pk->cmt_idx[i], cmt_hashed[i].v, 32,
                                      hipMemcpyHostToDevice, q));
            plk::ntt(pk->d0, pk->qkc.p, 1, 0, 0, q);  // -> canonical bit-reversed
            for (int i = 0; i < n_cmt; i++) {
                up(pk->pi_reg[i].p, cmt_values[i], nb, false, q);
                lag_to_canonical(pk, F(pk->pi_reg[i]), F(pk->pi_brev[i]), nullptr, q);
                plk::bit_reverse(F(pk->pi_brev[i]), F(pk->pi_reg[i]), n, q);
            }
            // canonical L, R, O (bit-reversed for the coset FFTs, regular for the
            // openings) while the commitments run: they only read lag[k]
            for (int k = 0; k < 3; k++) {
                GG_HIP(hipStreamWaitEvent(q, uploaded[k], 0));
                lag_to_canonical(pk, F(pk->lag[k]), F(pk->cbrev[k]), F(pk->can[k]), q);
            }
            GG_WAIT_STREAM(q);
        }
        for (auto& f : fs) f.get();
    }
    {
        BJac t[3];
        for (int k = 0; k < 3; k++) t[k] = jac_add(red(pk, lroj[k]), fblind[k].get());
        to_aff_batch(t, 3, P.lro);
    }
    mark();
    // ---- gamma, beta (deriveGammaAndBeta, prove.go:454-489; bindPublicData, verify.go:296-340).
    // G1Affine.Marshal is the UNCOMPRESSED encoding (RawBytes): groth16/bls12-381/verify.go:80-82
    // writes Marshal() into a buffer and continues at SizeOfG1AffineUncompressed, and the BN254
    // Solidity verifier of the same transcript binds X | Y (plonk/bn254/solidity.go:407-460)
    Transcript fs({"gamma", "beta", "alpha", "zeta"}, ch);
    {
        uint8_t b[96];
        for (int k = 0; k < 3; k++) { g1_raw_bytes(pk->vkS[k], b); fs.bind("gamma", b, PT); }
        for (int k = 0; k < 5; k++) { g1_raw_bytes(pk->vkQ[k], b); fs.bind("gamma", b, PT); }
        for (int i = 0; i < pk->n_cmt; i++) { g1_raw_bytes(pk->vkQcp[i], b); fs.bind("gamma", b, PT); }
        uint8_t f32[32];
        for (size_t i = 0; i < nb_pub; i++) { fr_marshal(pub[i], f32); fs.bind("gamma", f32, 32); }
    }
    const FrB gamma = derive(fs, "gamma", {&P.lro[0], &P.lro[1], &P.lro[2]});
    const FrB beta = fs.compute("beta");
    // ---- ratio Z (buildRatioCopyConstraint, prove.go:600-632) + its commitment.
    // With device parts every part takes the factors of its KzgLagrange slice
    // [l_lo, l_hi) (its L, R, O slices are still in its scalar slots from
    // commitToLRO) and scans them; the slice products are chained here and each
    // part writes its slice of Z where its share of the Z commitment reads it
    // (and into the primary's Z for the rest of the proof).
    for (int k = 0; k < 3; k++) record_wait(pk, s[k], s[0]);
    // the owner of Z's canonical form: every part pushes its slice of Z there
    PlonkPeer* zown = peers_on ? canon_owner(pk, ctasks.size() - 1) : nullptr;
    {
        const size_t zlo = dz ? pk->l_lo : 0, zcnt = dz ? pk->l_hi - pk->l_lo : n;
        const auto ta = std::chrono::steady_clock::now();
        const int64_t* pm = pk->perm.template as<int64_t>();
        pk->ar[0].reset();
        if (run0)
            plk::ratio_range(F(pk->lag[0]) + zlo, F(pk->lag[1]) + zlo, F(pk->lag[2]) + zlo, pm + zlo, pm + n + zlo,
                             pm + 2 * n + zlo, zlo, zcnt, n, beta, gamma, pk->omega, pk->u, F(pk->pz), s[0], pk->ar[0]);
        std::vector<FrB> agg(1 + pk->peers.size(), FrB::one());
        std::vector<FrB> pre(agg.size(), FrB::one());
        // one thread per peer: factors + scan of its slice, hand its slice product
        // over, wait for the chained prefixes, fix its slice of Z up and push it
        // to Z's owner (a failing peer releases the others through `stop`)
        std::vector<std::promise<void>> agg_done(pk->peers.size());
        std::promise<void> pre_ready;
        std::shared_future<void> pre_f = pre_ready.get_future().share();
        std::atomic<bool> stop{false};
        std::vector<gg::Task<void>> pf;
        if (peers_on)
            for (size_t q = 0; q < pk->peers.size(); q++)
                pf.push_back(gg::run_task([&, q] {
                    PlonkPeer* p = pk->peers[q].get();
                    const size_t cnt = p->l_hi - p->l_lo;
                    const bool mine = cnt && part_runs(pk, (int)q + 1);
                    double ms = 0;
                    try {
                        if (mine) {
                            GG_HIP(hipSetDevice(p->device));
                            const auto a = std::chrono::steady_clock::now();
                            p->ar.reset();
                            const int64_t* ps = p->perm_slice.as<int64_t>();
                            plk::ratio_range(F(p->scal[0]), F(p->scal[1]), F(p->scal[2]), ps, ps + cnt, ps + 2 * cnt,
                                             p->l_lo, cnt, n, beta, gamma, pk->omega, pk->u, F(p->pz), p->s[0], p->ar);
                            agg[q + 1] = fetch(F(p->pz) + cnt - 1, p->s[0]);
                            ms += ms_since(a);
                        }
                        agg_done[q].set_value();
                    } catch (...) {
                        agg_done[q].set_exception(std::current_exception());
                        return;
                    }
                    pre_f.wait();
                    if (!mine || stop) return;
                    const auto b = std::chrono::steady_clock::now();
                    plk::ratio_fixup(F(p->pz), cnt, pre[q + 1], F(p->scal[0]), p->s[0]);  // the Z slot of its MSM
                    // pushed to Z's owner from the copy stream (waits for the fixup only)
                    GG_HIP(hipEventRecord(p->cpev, p->s[0]));
                    GG_HIP(hipStreamWaitEvent(p->cps, p->cpev, 0));
                    GG_HIP(hipMemcpyPeerAsync(F(zown->in[3]) + p->l_lo, zown->device, p->scal[0].p, p->device, 32 * cnt,
                                              p->cps));
                    GG_WAIT_STREAM(p->cps);
                    std::lock_guard<std::mutex> lk(pk->tmu);
                    pk->ptimes[q + 1].ratio_ms += ms + ms_since(b);
                }));
        try {
            agg[0] = zcnt && run0 ? fetch(F(pk->pz) + zcnt - 1, s[0]) : FrB::one();
            for (size_t q = 0; q < pf.size(); q++) agg_done[q].get_future().get();
        } catch (...) {
            stop = true;
            pre_ready.set_value();
            for (auto& f : pf) f.wait();
            throw;
        }
        // prefix of part r = the product of the factors of the slices before it
        for (size_t r = 1; r < agg.size(); r++) pre[r] = pre[r - 1] * agg[r - 1];
        pre_ready.set_value();
        if (run0) plk::ratio_fixup(F(pk->pz), zcnt, pre[0], F(pk->zlag) + zlo, s[0]);
        if (zown && zcnt && run0)
            GG_HIP(hipMemcpyPeerAsync(F(zown->in[3]) + zlo, zown->device, F(pk->zlag) + zlo, pk->device, 32 * zcnt, s[0]));
        for (auto& f : pf) f.get();
        std::lock_guard<std::mutex> lk(pk->tmu);
        pk->ptimes[0].ratio_ms += ms_since(ta);
    }
    record_wait(pk, s[0], s[1]);
    gg::Task<void> zfut;
    if (peers_on) {  // Z's canonical forms on its owner, once every slice has landed there
        GG_WAIT_STREAM(s[0]);
        const size_t zi = (ctasks.size() - 1) % pk->peers.size();
        if (part_runs(pk, (int)zi + 1))
            zfut = gg::run_task([&, zi] {
            if (cfut[zi].valid()) cfut[zi].wait();  // its earlier tasks (creg, stream cs) first
            canon_run(pk, zi, 3, F(pk->cbrev[3]), F(pk->can[3]), [](hipStream_t) {});
        }).share();
    } else if (!dz) {
        lag_to_canonical(pk, F(pk->zlag), F(pk->cbrev[3]), F(pk->can[3]), s[1]);  // overlaps the Z commitment
    }
    // the Z commitment in flight; meanwhile each part's first quotient unit takes
    // its evaluations of L, R, O, Qk, Pi_j (only Z's wait for Z)
    gg::Task<BJac> fzc = msm_task([&] {
        GG_HIP(hipSetDevice(pk->device));
        return msm_jac(pk, pk->kzg_lag, 0, F(pk->zlag), s[0], peers_on);
    });
    auto unit_pre = [&](const QUnit* q, const FrB* const* src, FrB* const* e, hipStream_t st) {
        for (int k = 0; k < 3; k++) unit_eval(pk, q->dom, q->kappa, src[k], e[k], st);
        unit_eval(pk, q->dom, q->kappa, src[4], e[6], st);
        for (int j = 0; j < n_cmt; j++) unit_eval(pk, q->dom, q->kappa, src[5 + j], e[7 + j], st);
    };
    if (peers_on) {  // L R O Qk Pi_j have reached every part
        const auto w = std::chrono::steady_clock::now();
        for (auto& f : cfut)
            if (f.valid()) f.get();
        {
            std::lock_guard<std::mutex> lk(pk->tmu);
            pk->ptimes[0].wait_ms += ms_since(w);
        }
        for (size_t pi = 0; pi < pk->peers.size(); pi++) {
            PlonkPeer* p = pk->peers[pi].get();
            if (p->units.empty() || !part_runs(pk, (int)pi + 1)) continue;
            GG_HIP(hipSetDevice(p->device));
            const FrB* ins[5 + plk::MAX_CMT] = {};
            for (int k = 0; k < 5 + n_cmt; k++) ins[k] = F(p->in[k]);
            FrB* e[7 + plk::MAX_CMT] = {};
            for (int k = 0; k < 7 + n_cmt; k++) e[k] = F(p->cev[k]);
            unit_pre(p->units[0].get(), ins, e, p->s[3]);
        }
        GG_HIP(hipSetDevice(pk->device));
    }
    if (run0 && !pk->units.empty()) {  // part 0's first unit: slot 0, stream 2
        const FrB* src[5 + plk::MAX_CMT] = {F(pk->cbrev[0]), F(pk->cbrev[1]), F(pk->cbrev[2]), F(pk->cbrev[3]),
                                            F(pk->qkc)};
        for (int j = 0; j < n_cmt; j++) src[5 + j] = F(pk->pi_brev[j]);
        FrB* e[7 + plk::MAX_CMT] = {};
        for (int k = 0; k < 7 + n_cmt; k++) e[k] = F(pk->cev[0][k]);
        unit_pre(pk->units[0].get(), src, e, s[2]);
    }
    P.z = to_aff(jac_add(red(pk, fzc.get()), fblind[3].get()));
    mark();
    // ---- alpha (deriveAlpha, prove.go:504-512)
    P.bsb22.assign(cmt_digests, cmt_digests + n_cmt);
    {
        uint8_t b[96];
        for (int i = 0; i < n_cmt; i++) { g1_raw_bytes(P.bsb22[i], b); fs.bind("alpha", b, PT); }
    }
    const FrB alpha = derive(fs, "alpha", {&P.z});
    // ---- computeNumerator + divideByXMinusOne (prove.go:837-1079, 1223-1276) as
    // quotient units (QUnit): this part's units two in flight on s[2], s[3], the
    // other parts' units on their devices concurrently; then the tail stages of
    // the big coset iFFT here
    for (int k = 0; k < 4; k++) record_wait(pk, s[k == 3 ? 1 : k], s[2]), record_wait(pk, s[k == 3 ? 1 : k], s[3]);
    const size_t m = n / pk->S, mb = 32 * m;
    // the parameters of unit q: e[] = its evaluations of L R O Z (0..3), Qk (6),
    // Pi_j (7 + j); zc = Z on class p + rho (S > 1); the key's evaluations in q->ev
    auto unit_params = [&](const QUnit* q, FrB* const* e, const FrB* zc, FrB* cres, bool local) {
        const FrB cs = pk->u, css = pk->u * pk->u;
        plk::NumParamsT<FrB> NP{};
        auto kev = [&](int k) { return (const FrB*)F(q->ev[k]); };
        NP.x[plk::ID_L] = e[0];
        NP.x[plk::ID_R] = e[1];
        NP.x[plk::ID_O] = e[2];
        NP.x[plk::ID_Z] = e[3];
        NP.x[plk::ID_ZS] = zc;  // nullptr (S = 1): Z[(j + 1) % m]
        NP.zs_shift = (zc && q->p + (int)pk->rho >= pk->U) ? 1u : 0u;
        NP.x[plk::ID_QL] = kev(Key::E_QL);
        NP.x[plk::ID_QR] = kev(Key::E_QR);
        NP.x[plk::ID_QM] = kev(Key::E_QM);
        NP.x[plk::ID_QO] = kev(Key::E_QO);
        NP.x[plk::ID_QK] = e[6];
        NP.x[plk::ID_S1] = kev(Key::E_S1);
        NP.x[plk::ID_S2] = kev(Key::E_S2);
        NP.x[plk::ID_S3] = kev(Key::E_S3);
        NP.x[plk::ID_ID] = kev(Key::E_X);  // X; beta folded into ka, kb, kc
        NP.x[plk::ID_LONE] = kev(Key::E_LONE);
        for (int j = 0; j < n_cmt; j++) {
            NP.x[plk::ID_QCI + 2 * j] = kev(Key::E_QCP0 + j);
            NP.x[plk::ID_QCI + 2 * j + 1] = e[7 + j];
        }
        NP.nx = plk::ID_QCI + 2 * n_cmt;
        // blinding polynomials scaled for the unit's coset c: b_j s^j (s^n - 1) (prove.go:985-993)
        const FrB sc = pk->coset_shift[q->p % pk->rho];
        const FrB sn1 = pow_u64(sc, n) - FrB::one();
        for (int q4 = 0; q4 < 4; q4++) {
            FrB acc = sn1;
            NP.bdeg[q4] = (int)bp[q4].size();
            for (size_t j = 0; j < bp[q4].size(); j++) {
                NP.bcoef[q4][j] = bp[q4][j] * acc;
                acc = acc * sc;
            }
        }
        // twiddles0 at the class's points (S = 1: the small domain itself)
        NP.tw0 = pk->S > 1 ? (const FrB*)F(q->tw0) : nullptr;
        NP.tw1 = pk->S > 1 ? (const FrB*)F(q->tw1) : nullptr;
        NP.beta = beta;
        NP.gamma = gamma;
        NP.alpha = alpha;
        NP.cs = cs;
        NP.css = css;
        NP.ka = beta;
        NP.kb = beta * cs;
        NP.kc = beta * css;
        NP.n = (uint32_t)m;
        NP.rho = (uint32_t)pk->U;
        NP.coset = (uint32_t)q->p;
        NP.log_big = (uint32_t)pk->log_big;
        NP.cres = cres;
        NP.local_block = local ? 1u : 0u;
        NP.has_out_scale = 1;  // divideByXMinusOne: 1 / (x^n - 1), constant on the coset
        memcpy(NP.out_scale.v, q->inv_den, 32);
        return NP;
    };
    // one unit: its polynomials' evaluations (L R O Qk Pi_j already taken for a
    // part's first unit: pre), the numerator (scaled), and the first L - u stages
    // of the big coset iFFT on its block
    auto run_unit = [&](const QUnit* q, const FrB* const* src, FrB* const* e, FrB* zc, const FrB* tw0, FrB* cres,
                        bool local, bool pre, hipStream_t st) {
        if (!pre) unit_pre(q, src, e, st);
        unit_eval(pk, q->dom, q->kappa, src[3], e[3], st);
        if (pk->S > 1) unit_eval(pk, q->zdom, q->zkappa, src[3], zc, st);
        plk::NumParamsT<FrB> NP = unit_params(q, e, pk->S > 1 ? zc : nullptr, cres, local);
        if (pk->S == 1) NP.tw0 = tw0;
        plk::numerator(NP, st);
        if (pk->split_idft) {
            const size_t blk = (size_t)(__builtin_bitreverse32((uint32_t)q->p) >> (32 - pk->log_u));
            ntt_inverse_dit_noscale(q->dom, local ? (void*)cres : (void*)(cres + blk * m), st);
        }
    };
    std::vector<gg::Task<void>> peer_work;
    if (peers_on) {  // Z's canonical form pushed by its owner
        const auto w = std::chrono::steady_clock::now();
        if (zfut.valid()) zfut.get();
        std::lock_guard<std::mutex> lk(pk->tmu);
        pk->ptimes[0].wait_ms += ms_since(w);
    }
    if (peers_on) {
        for (size_t pi = 0; pi < pk->peers.size(); pi++) {
            PlonkPeer* p = pk->peers[pi].get();
            if (p->units.empty() || !part_runs(pk, (int)pi + 1)) continue;
            peer_work.push_back(gg::run_task([&, p, pi] {
                GG_HIP(hipSetDevice(p->device));
                const auto ta = std::chrono::steady_clock::now();
                hipStream_t q = p->s[3];
                const FrB* ins[5 + plk::MAX_CMT] = {};
                for (int k = 0; k < 5 + n_cmt; k++) ins[k] = F(p->in[k]);
                FrB* e[7 + plk::MAX_CMT] = {};
                for (int k = 0; k < 7 + n_cmt; k++) e[k] = F(p->cev[k]);
                for (size_t u = 0; u < p->units.size(); u++)
                    run_unit(p->units[u].get(), ins, e, F(p->zc), F(p->tw0), F(p->units[u]->out), true, u == 0, q);
                // the units' blocks back to the primary's cres (timed separately),
                // from the copy stream: it waits for the units' kernels only
                GG_HIP(hipEventRecord(p->cpev, q));
                GG_HIP(hipStreamWaitEvent(p->cps, p->cpev, 0));
                GG_HIP(hipEventRecord(p->ea[3], p->cps));
                for (auto& qu : p->units) {
                    const size_t blk = (size_t)(__builtin_bitreverse32((uint32_t)qu->p) >> (32 - pk->log_u));
                    GG_HIP(hipMemcpyPeerAsync(F(pk->cres) + blk * m, pk->device, qu->out.p, p->device, mb, p->cps));
                }
                GG_HIP(hipEventRecord(p->eb[3], p->cps));
                GG_WAIT_STREAM(p->cps);
                float cout = 0;
                GG_HIP(hipEventElapsedTime(&cout, p->ea[3], p->eb[3]));
                std::lock_guard<std::mutex> lk(pk->tmu);
                PlonkPartTimes& T = pk->ptimes[pi + 1];
                T.coset_count += (double)p->units.size();
                T.coset_ms += ms_since(ta);
                T.coset_out_copy_ms += cout;
                T.coset_mb += (double)mb * p->units.size() / 1e6;
            }));
        }
    }
    {
        int slot = 0;
        const FrB* src[5 + plk::MAX_CMT] = {F(pk->cbrev[0]), F(pk->cbrev[1]), F(pk->cbrev[2]), F(pk->cbrev[3]),
                                            F(pk->qkc)};
        for (int j = 0; j < n_cmt; j++) src[5 + j] = F(pk->pi_brev[j]);
        for (size_t u = 0; run0 && u < pk->units.size(); u++) {
            hipStream_t q = s[2 + slot];
            FrB* e[7 + plk::MAX_CMT] = {};
            for (int k = 0; k < 7 + n_cmt; k++) e[k] = F(pk->cev[slot][k]);
            run_unit(pk->units[u].get(), src, e, F(pk->zc[slot]), F(pk->tw0), F(pk->cres), false, u == 0, q);
            slot ^= 1;
        }
        std::lock_guard<std::mutex> lk(pk->tmu);
        if (run0) pk->ptimes[0].coset_count += (double)pk->units.size();
    }
    {
        const auto w = std::chrono::steady_clock::now();
        for (auto& f : peer_work) f.get();  // their blocks of cres have landed
        std::lock_guard<std::mutex> lk(pk->tmu);
        pk->ptimes[0].wait_ms += ms_since(w);
    }
    record_wait(pk, s[3], s[2]);
    // h, canonical regular: the last log2(U) stages of FFTInverse(DIT, OnCoset) over
    // the units' blocks (or, for domains below 2^12, the whole inverse here)
    if (run0) {
        if (pk->split_idft) ntt_tail_inverse_coset(pk->d1, F(pk->cres), pk->log_u, s[2]);
        else plk::ntt(pk->d1, F(pk->cres), 1, 1, 1, s[2]);
        for (int k = 0; k < 3; k++) {  // n + 2 coefficients, the (n + 3)-th MSM scalar zero
            dcopy(pk->hpad[k].p, F(pk->cres) + (n + 2) * k, 32 * (n + 2), s[2]);
            zero(F(pk->hpad[k]) + n + 2, 32, s[2]);
        }
    }
    for (int k = 0; k < 3; k++) record_wait(pk, s[2], s[k]);
    mark();
    // ---- commitToQuotient: H1, H2, H3 at once (prove.go:1199-1218)
    {
        BJac hj[3];
        if (batch_ok(pk, true, 3)) {
            // hpad[k] are complete on s[2] (recorded just above into s[0..2])
            const FrB* sc[3] = {F(pk->hpad[0]), F(pk->hpad[1]), F(pk->hpad[2])};
            msm_jac_batch(pk, pk->kzg, sc, 3, s[0], hj);
        } else {
            std::vector<gg::Task<void>> fs3;
            for (int k = 0; k < 3; k++)
                fs3.push_back(msm_task([&, k] {
                    GG_HIP(hipSetDevice(pk->device));
                    hj[k] = commit_kzg(pk, k, F(pk->hpad[k]), s[k]);
                }));
            for (auto& f : fs3) f.get();
        }
        BJac t[3];
        for (int k = 0; k < 3; k++) t[k] = red(pk, hj[k]);
        to_aff_batch(t, 3, P.h);
    }
    mark();
    const FrB zeta = derive(fs, "zeta", {&P.h[0], &P.h[1], &P.h[2]});
    const FrB zn = pow_u64(zeta, n), zn1 = zn - FrB::one();
    if (peers_on) canon_wait_regular(pk);  // the regular L, R, O, Z, Pi_j for the openings
    // ---- openZ (prove.go:635-652): blinded Z = Z - bz + bz X^n, opened at zeta * omega
    auto blinded = [&](const DevBuf& canon, const std::vector<FrB>& b, DevBuf& out, hipStream_t q) {
        if (!run0) return;
        dcopy(out.p, canon.p, nb, q);
        zero(F(out) + n, nb3 - nb, q);
        std::vector<FrB> head(b.size()), tail(b);
        for (size_t j = 0; j < b.size(); j++) head[j] = -b[j];
        GG_HIP(hipMemcpyAsync(F(pk->pad), head.data(), 32 * b.size(), hipMemcpyHostToDevice, q));
        plk::axpy(F(out), F(pk->pad), b.size(), FrB::one(), q);
        GG_HIP(hipMemcpyAsync(F(out) + n, tail.data(), 32 * b.size(), hipMemcpyHostToDevice, q));
        GG_WAIT_STREAM(q);  // host vectors
    };
    blinded(pk->can[3], bp[3], pk->bz, s[0]);
    if (run0) zero(F(pk->q1) + n + 2, 32, s[0]);  // Horner writes the n + 2 quotient coefficients
    const FrB zu = run0 ? eval_dev(pk, F(pk->bz), n + 3, zeta * pk->omega, F(pk->q1), F(pk->vals), 0, s[0]) : FrB::zero();
    P.zs_value = zu;
    // openZ's quotient and the linearized polynomial are both committed on
    // pk.Kzg.  GG_PLONK_BATCH_OPEN=1: one batched MSM once the linearized
    // polynomial is formed (one sort and one bucket reduction fewer per part) --
    // measured slower (r06i: one GPU 126.8 vs 125.5 ms, slowest of 8 parts 25.0
    // vs 24.1 ms): openZ's MSM no longer overlaps the linearized polynomial's
    // evaluations and kernel.  Default: openZ's MSM at once on s[0]
    static const bool open_batch_env = getenv("GG_PLONK_BATCH_OPEN") && atoi(getenv("GG_PLONK_BATCH_OPEN")) == 1;
    const bool open_batch = open_batch_env && batch_ok(pk, true, 2);
    gg::Task<BJac> fzs;
    if (!open_batch)
        fzs = msm_task([&] {
            GG_HIP(hipSetDevice(pk->device));
            return commit_kzg(pk, 0, F(pk->q1), s[0]);
        });
    // ---- foldH (prove.go:670-705) on s[2]
    const FrB zp = pow_u64(zeta, n + 2);
    if (run0) {
        zero(F(pk->fold) + n + 2, 32, s[2]);  // fold_h writes n + 2 coefficients
        plk::fold_h(F(pk->cres), n, zp, F(pk->fold), s[2]);
    }
    BJac fhd = jac_add(jac_add(BJac::from_affine(P.h[0]), jmul(P.h[1], zp)), jmul(P.h[2], zp * zp));
    const BAff folded_digest = to_aff(fhd);
    // ---- evaluations at zeta (blinded L, R, O; S1, S2; Qcp_i) on s[1]: one
    // batched pass over the 5 + n_cmt polynomials, one read-back
    for (int k = 0; k < 3; k++) blinded(pk->can[k], bp[k], pk->bl[k], s[1]);
    FrB lz[3], s1z, s2z;
    std::vector<FrB> qcpz(n_cmt);
    {
        const FrB* fz[plk::EVAL_MAX] = {F(pk->bl[0]), F(pk->bl[1]), F(pk->bl[2]), F(pk->reg[Key::S1]),
                                        F(pk->reg[Key::S2])};
        size_t lz_len[plk::EVAL_MAX] = {n + 2, n + 2, n + 2, n, n};
        for (int j = 0; j < n_cmt; j++) {
            fz[5 + j] = F(pk->qcp_reg[j]);
            lz_len[5 + j] = n;
        }
        std::vector<FrB> v = run0 ? eval_batch(pk, fz, lz_len, 5 + n_cmt, zeta, F(pk->vals) + 1, 1, s[1])
                                  : std::vector<FrB>(5 + n_cmt, FrB::zero());
        for (int k = 0; k < 3; k++) lz[k] = v[k];
        s1z = v[3];
        s2z = v[4];
        for (int j = 0; j < n_cmt; j++) qcpz[j] = v[5 + j];
    }
    // ---- computeLinearizedPolynomial (prove.go:1289-1389) on s[1]
    {
        const FrB l = lz[0], r = lz[1], o = lz[2];
        FrB sa = (s1z * beta + l + gamma) * (s2z * beta + r + gamma) * zu * beta;
        const FrB uz = zeta * pk->u, uuz = uz * pk->u;
        FrB sb = (beta * zeta + l + gamma) * (beta * uz + r + gamma) * (beta * uuz + o + gamma);
        sb = -sb;
        const FrB lag = zn1 * inverse(zeta - FrB::one()) * alpha * alpha * pk->n_inv;
        if (run0) dcopy(pk->lin.p, pk->bz.p, nb3, s[1]);  // bz is complete: openZ's Horner synchronised s[0]
        plk::LinParamsT<FrB> LP{};
        LP.z = F(pk->lin);
        LP.nz = n + 3;
        LP.s3 = F(pk->reg[Key::S3]);
        LP.ns3 = n;
        LP.ql = F(pk->reg[Key::QL]);
        LP.qr = F(pk->reg[Key::QR]);
        LP.qm = F(pk->reg[Key::QM]);
        LP.qo = F(pk->reg[Key::QO]);
        LP.qk = F(pk->reg[Key::QK]);
        LP.nq = n;
        LP.ncmt = n_cmt;
        for (int j = 0; j < n_cmt; j++) {
            LP.pi2[j] = F(pk->pi_reg[j]);
            LP.qcp[j] = qcpz[j];
        }
        LP.s1 = sa;
        LP.s2 = sb;
        LP.alpha = alpha;
        LP.l = l;
        LP.r = r;
        LP.rl = l * r;
        LP.o = o;
        LP.lag = lag;
        if (run0) plk::linearized(LP, s[1]);
    }
    mark();
    BAff lin_digest;
    BJac zs_jac = BJac::inf();
    if (open_batch) {
        record_wait(pk, s[0], s[1]);  // q1 (openZ's Horner on s[0]) and lin (s[1]) complete on s[1]
        const FrB* sc[2] = {F(pk->q1), F(pk->lin)};
        BJac oj[2];
        msm_jac_batch(pk, pk->kzg, sc, 2, s[1], oj);
        zs_jac = oj[0];
        lin_digest = to_aff(red(pk, oj[1]));
    } else {
        lin_digest = to_aff(red(pk, commit_kzg(pk, 1, F(pk->lin), s[1])));
    }
    mark();
    // ---- batchOpening: kzg.BatchOpenSinglePoint at zeta (prove.go:777-835)
    GG_WAIT_STREAM(s[2]);  // folded H
    std::vector<std::pair<const FrB*, size_t>> polys = {
        {F(pk->fold), n + 2}, {F(pk->lin), n + 3}, {F(pk->bl[0]), n + 2}, {F(pk->bl[1]), n + 2},
        {F(pk->bl[2]), n + 2}, {F(pk->reg[Key::S1]), n}, {F(pk->reg[Key::S2]), n}};
    for (int j = 0; j < n_cmt; j++) polys.push_back({F(pk->qcp_reg[j]), n});
    std::vector<BAff> digests = {folded_digest, lin_digest, P.lro[0], P.lro[1], P.lro[2], pk->vkS[0], pk->vkS[1]};
    for (int j = 0; j < n_cmt; j++) digests.push_back(pk->vkQcp[j]);
    P.claimed.resize(polys.size());
    {
        const FrB* fz[plk::EVAL_MAX] = {polys[0].first, polys[1].first};
        const size_t fl[plk::EVAL_MAX] = {polys[0].second, polys[1].second};
        std::vector<FrB> v = run0 ? eval_batch(pk, fz, fl, 2, zeta, F(pk->vals) + 16, 2, s[2])
                                  : std::vector<FrB>(2, FrB::zero());
        P.claimed[0] = v[0];
        P.claimed[1] = v[1];
    }
    for (int k = 0; k < 3; k++) P.claimed[2 + k] = lz[k];
    P.claimed[5] = s1z;
    P.claimed[6] = s2z;
    for (int j = 0; j < n_cmt; j++) P.claimed[7 + j] = qcpz[j];
    // deriveGamma of kzg (gnark-crypto [ext]): point, digests (Marshal = uncompressed), claimed
    // values, Z(w zeta) -- the order of compute_gamma_kzg, plonk/bn254/solidity.go:961-1024
    Transcript fg({"gamma"}, fh);
    {
        uint8_t b[96];
        fr_marshal(zeta, b);
        fg.bind("gamma", b, 32);
        for (auto& d : digests) { g1_raw_bytes(d, b); fg.bind("gamma", b, PT); }
        for (auto& c : P.claimed) { fr_marshal(c, b); fg.bind("gamma", b, 32); }
        fr_marshal(zu, b);
        fg.bind("gamma", b, 32);
    }
    const FrB gf = fg.compute("gamma");
    FrB fe = P.claimed.back();
    for (size_t i = P.claimed.size() - 1; i-- > 0;) fe = fe * gf + P.claimed[i];
    // folded polynomial sum_i gamma^i p_i (one pass), then the quotient (f - f(zeta)) / (X - zeta)
    {
        const FrB* fp[plk::EVAL_MAX];
        size_t fl[plk::EVAL_MAX];
        FrB cf[plk::EVAL_MAX];
        FrB gp = FrB::one();
        for (size_t i = 0; i < polys.size(); i++) {
            fp[i] = polys[i].first;
            fl[i] = polys[i].second;
            cf[i] = gp;
            gp = gp * gf;
        }
        if (run0) plk::lincomb(F(pk->q2), n + 3, fp, fl, cf, (int)polys.size(), s[2]);
    }
    if (run0) {
        zero(F(pk->fold) + n + 2, 32, s[2]);  // reuse as the batch quotient (n + 2 of n + 3)
        const FrB fv = eval_dev(pk, F(pk->q2), n + 3, zeta, F(pk->fold), F(pk->vals) + 18, 2, s[2]);
        GG_CHECK(fv == fe, GG_ERR_INTERNAL, "batch opening: folded evaluation mismatch");
    }
    P.batched_h = to_aff(red(pk, commit_kzg(pk, 2, F(pk->fold), s[2])));
    P.zs_h = to_aff(red(pk, open_batch ? zs_jac : fzs.get()));
    mark();
    for (hipStream_t q : pk->s) GG_WAIT_STREAM(q);
}

};

// ============================================================== C ABI
// cumulative stage ends (ms) of the last gg_plonk_prove on this thread
static thread_local double g_plonk_ms[8];

namespace {

template <class Cv>
gg_plonk_pk* plonk_create(int log_n, int log_big, const void* omega, const void* omega_big, const void* coset_shift,
                          const void* kzg_g1, size_t n_kzg, const void* kzg_lagrange_g1, const void* const* trace,
                          const void* const* qcp, int n_cmt, const int64_t* perm, size_t nb_public,
                          const uint64_t* cmt_idx, const void* vk_digests, int rank, int world, gg_g1_reduce_fn reduce,
                          void* rctx, const int* devices, int n_devices) {
    using Impl = PlonkImpl<Cv>;
    std::unique_ptr<typename Impl::Key> pk(new typename Impl::Key());
    Impl::plonk_pk_build(pk.get(), log_n, log_big, omega, omega_big, coset_shift, kzg_g1, n_kzg, kzg_lagrange_g1,
                         trace, qcp, n_cmt, perm, nb_public, cmt_idx, vk_digests, rank, world, reduce, rctx, devices,
                         n_devices);
    return pk.release();
}

gg_plonk_pk* create_any(int curve, int log_n, int log_big, const void* omega, const void* omega_big,
                        const void* coset_shift, const void* kzg_g1, size_t n_kzg, const void* kzg_lagrange_g1,
                        const void* const* trace, const void* const* qcp, int n_cmt, const int64_t* perm,
                        size_t nb_public, const uint64_t* cmt_idx, const void* vk_digests, int rank, int world,
                        gg_g1_reduce_fn reduce, void* rctx, const int* devices, int n_devices) {
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "bad curve");
    if (curve == GG_CURVE_BN254)
        return plonk_create<PlonkBn254>(log_n, log_big, omega, omega_big, coset_shift, kzg_g1, n_kzg,
                                        kzg_lagrange_g1, trace, qcp, n_cmt, perm, nb_public, cmt_idx, vk_digests,
                                        rank, world, reduce, rctx, devices, n_devices);
    return plonk_create<PlonkBls12381>(log_n, log_big, omega, omega_big, coset_shift, kzg_g1, n_kzg,
                                       kzg_lagrange_g1, trace, qcp, n_cmt, perm, nb_public, cmt_idx, vk_digests, rank,
                                       world, reduce, rctx, devices, n_devices);
}

// fn(typed key) on the handle's curve
template <class Fn>
auto with_key(gg_plonk_pk* pk, Fn fn) {
    if (pk->curve == GG_CURVE_BN254) return fn(static_cast<typename PlonkImpl<PlonkBn254>::Key*>(pk));
    return fn(static_cast<typename PlonkImpl<PlonkBls12381>::Key*>(pk));
}

size_t proof_size(int curve, int n_cmt) {
    const size_t pt = curve == GG_CURVE_BN254 ? 64 : 96;
    return pt * (3 + 1 + 3 + (size_t)n_cmt + 1 + 1) + 32 * (7 + (size_t)n_cmt) + 32;
}

}  // namespace

extern "C" int gg_plonk_pk_create_ex(int curve, int log_n, int log_big, const void* omega_mont,
                                     const void* omega_big_mont, const void* coset_shift_mont, const void* kzg_g1,
                                     size_t n_kzg, const void* kzg_lagrange_g1, const void* const* trace,
                                     const void* const* qcp, int n_cmt, const int64_t* perm, size_t nb_public,
                                     const uint64_t* commitment_constraint_indexes, const void* vk_digests,
                                     int n_devices, const int* devices, gg_plonk_pk_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out && (n_devices <= 1 || devices), GG_ERR_INVALID_ARG, "null argument");
    *out = create_any(curve, log_n, log_big, omega_mont, omega_big_mont, coset_shift_mont, kzg_g1, n_kzg,
                      kzg_lagrange_g1, trace, qcp, n_cmt, perm, nb_public, commitment_constraint_indexes, vk_digests,
                      0, 1, nullptr, nullptr, n_devices > 1 ? devices : nullptr, n_devices > 1 ? n_devices : 1);
    GG_CAPI_END
}

extern "C" int gg_plonk_pk_create(int log_n, int log_big, const void* omega_mont, const void* omega_big_mont,
                                  const void* coset_shift_mont, const void* kzg_g1, size_t n_kzg,
                                  const void* kzg_lagrange_g1, const void* const* trace, const void* const* qcp,
                                  int n_cmt, const int64_t* perm, size_t nb_public,
                                  const uint64_t* commitment_constraint_indexes, const void* vk_digests,
                                  gg_plonk_pk_t* out) {
    return gg_plonk_pk_create_ex(GG_CURVE_BLS12_381, log_n, log_big, omega_mont, omega_big_mont, coset_shift_mont,
                                 kzg_g1, n_kzg, kzg_lagrange_g1, trace, qcp, n_cmt, perm, nb_public,
                                 commitment_constraint_indexes, vk_digests, 1, nullptr, out);
}

extern "C" int gg_plonk_pk_create_shard_ex(int curve, int log_n, int log_big, const void* omega_mont,
                                           const void* omega_big_mont, const void* coset_shift_mont,
                                           const void* kzg_g1, size_t n_kzg, const void* kzg_lagrange_g1,
                                           const void* const* trace, const void* const* qcp, int n_cmt,
                                           const int64_t* perm, size_t nb_public,
                                           const uint64_t* commitment_constraint_indexes, const void* vk_digests,
                                           int rank, int world, gg_g1_reduce_fn reduce, void* reduce_ctx,
                                           gg_plonk_pk_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out, GG_ERR_INVALID_ARG, "null out");
    *out = create_any(curve, log_n, log_big, omega_mont, omega_big_mont, coset_shift_mont, kzg_g1, n_kzg,
                      kzg_lagrange_g1, trace, qcp, n_cmt, perm, nb_public, commitment_constraint_indexes, vk_digests,
                      rank, world, reduce, reduce_ctx, nullptr, 1);
    GG_CAPI_END
}

extern "C" int gg_plonk_pk_create_shard(int log_n, int log_big, const void* omega_mont, const void* omega_big_mont,
                                        const void* coset_shift_mont, const void* kzg_g1, size_t n_kzg,
                                        const void* kzg_lagrange_g1, const void* const* trace,
                                        const void* const* qcp, int n_cmt, const int64_t* perm, size_t nb_public,
                                        const uint64_t* commitment_constraint_indexes, const void* vk_digests,
                                        int rank, int world, gg_g1_reduce_fn reduce, void* reduce_ctx,
                                        gg_plonk_pk_t* out) {
    return gg_plonk_pk_create_shard_ex(GG_CURVE_BLS12_381, log_n, log_big, omega_mont, omega_big_mont,
                                       coset_shift_mont, kzg_g1, n_kzg, kzg_lagrange_g1, trace, qcp, n_cmt, perm,
                                       nb_public, commitment_constraint_indexes, vk_digests, rank, world, reduce,
                                       reduce_ctx, out);
}

extern "C" int gg_plonk_pk_create_multi(int log_n, int log_big, const void* omega_mont, const void* omega_big_mont,
                                        const void* coset_shift_mont, const void* kzg_g1, size_t n_kzg,
                                        const void* kzg_lagrange_g1, const void* const* trace,
                                        const void* const* qcp, int n_cmt, const int64_t* perm, size_t nb_public,
                                        const uint64_t* commitment_constraint_indexes, const void* vk_digests,
                                        int n_devices, const int* devices, gg_plonk_pk_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out && devices, GG_ERR_INVALID_ARG, "null argument");
    *out = create_any(GG_CURVE_BLS12_381, log_n, log_big, omega_mont, omega_big_mont, coset_shift_mont, kzg_g1,
                      n_kzg, kzg_lagrange_g1, trace, qcp, n_cmt, perm, nb_public, commitment_constraint_indexes,
                      vk_digests, 0, 1, nullptr, nullptr, devices, n_devices);
    GG_CAPI_END
}

extern "C" int gg_plonk_pk_info(gg_plonk_pk_t pk, int* curve, int* log_n, int* n_cmt) {
    GG_CAPI_BEGIN
    GG_CHECK(pk, GG_ERR_INVALID_ARG, "null key");
    with_key(pk, [&](auto* k) {
        if (curve) *curve = k->curve;
        if (log_n) *log_n = k->log_n;
        if (n_cmt) *n_cmt = k->n_cmt;
        return 0;
    });
    GG_CAPI_END
}

extern "C" int gg_plonk_pk_devices(gg_plonk_pk_t pk, int* devices, int cap, int* n_devices) {
    GG_CAPI_BEGIN
    GG_CHECK(pk && n_devices, GG_ERR_INVALID_ARG, "null argument");
    with_key(pk, [&](auto* k) {
        *n_devices = 1 + (int)k->peers.size();
        GG_CHECK(!devices || cap >= *n_devices, GG_ERR_INVALID_ARG, "cap < number of device parts");
        if (devices) {
            devices[0] = k->device;
            for (size_t i = 0; i < k->peers.size(); i++) devices[1 + i] = k->peers[i]->device;
        }
        return 0;
    });
    GG_CAPI_END
}

extern "C" int gg_plonk_pk_release(gg_plonk_pk_t pk) {
    GG_CAPI_BEGIN
    delete pk;
    GG_CAPI_END
}

extern "C" int gg_plonk_pk_vk(gg_plonk_pk_t pk, void* out, size_t cap) {
    GG_CAPI_BEGIN
    GG_CHECK(pk && out, GG_ERR_INVALID_ARG, "null argument");
    with_key(pk, [&](auto* k) {
        const size_t pt = sizeof(k->vkS[0]);
        GG_CHECK(cap >= pt * (size_t)(8 + k->n_cmt), GG_ERR_INVALID_ARG, "vk buffer too small");
        uint8_t* o = (uint8_t*)out;
        for (int j = 0; j < 3; j++) memcpy(o + pt * j, &k->vkS[j], pt);
        for (int j = 0; j < 5; j++) memcpy(o + pt * (3 + j), &k->vkQ[j], pt);
        for (int i = 0; i < k->n_cmt; i++) memcpy(o + pt * (8 + i), &k->vkQcp[i], pt);
        return 0;
    });
    GG_CAPI_END
}

extern "C" int gg_plonk_commit_lagrange(gg_plonk_pk_t pk, const void* values, int on_device, void* out_aff) {
    GG_CAPI_BEGIN
    GG_CHECK(pk && values && out_aff, GG_ERR_INVALID_ARG, "null argument");
    with_key(pk, [&](auto* k) {
        using Impl = PlonkImpl<typename std::remove_pointer<decltype(k)>::type::CvT>;
        std::lock_guard<std::mutex> lk(k->mu);
        GG_HIP(hipSetDevice(k->device));
        hipStream_t st = k->s[3];
        Impl::up(k->pad.p, values, 32 * k->n, on_device != 0, st);
        // a hint commitment is a value the circuit consumes: every part works on
        // it even while the key rehearses one part (gg_plonk_pk_set_rehearsal_part)
        struct SoloGuard {
            bool& f;
            bool saved;
            ~SoloGuard() { f = saved; }
        } solo_guard{k->solo, k->solo};
        k->solo = false;
        const auto a = Impl::to_aff(Impl::red(k, Impl::msm_jac(k, k->kzg_lag, 2, Impl::F(k->pad), st)));
        if (gg::kAccumProbe) throw gg::Error(GG_REHEARSAL, "traffic-probe build (GG_ACCUM_PROBE): wrong MSM sums");
        memcpy(out_aff, &a, sizeof(a));
        return 0;
    });
    GG_CAPI_END
}

extern "C" size_t gg_plonk_proof_size(int n_cmt) { return proof_size(GG_CURVE_BLS12_381, n_cmt); }

extern "C" size_t gg_plonk_proof_size_ex(int curve, int n_cmt) { return proof_size(curve, n_cmt); }

extern "C" int gg_plonk_prove(gg_plonk_pk_t pk, const void* l, const void* r, const void* o, int inputs_on_device,
                              const void* public_witness, size_t nb_public, const void* const* cmt_values,
                              const void* cmt_digests, const void* cmt_hashed, int n_cmt, const void* blinding,
                              gg_hash_fn challenge_hash, void* challenge_ctx, gg_hash_fn folding_hash,
                              void* folding_ctx, void* proof_out, size_t proof_cap) {
    GG_CAPI_BEGIN
    GG_CHECK(pk && l && r && o && proof_out, GG_ERR_INVALID_ARG, "null argument");
    with_key(pk, [&](auto* k) {
        using Impl = PlonkImpl<typename std::remove_pointer<decltype(k)>::type::CvT>;
        using FrT = typename Impl::FrB;
        using AffT = typename Impl::BAff;
        const size_t pt = sizeof(AffT);
        GG_CHECK(nb_public == k->nb_public, GG_ERR_INVALID_ARG, "len(public witness) != vk.NbPublicVariables");
        GG_CHECK(nb_public == 0 || public_witness, GG_ERR_INVALID_ARG, "null public witness");
        GG_CHECK(n_cmt == k->n_cmt, GG_ERR_INVALID_ARG, "BSB22 commitment count differs from the key's");
        GG_CHECK(n_cmt == 0 || (cmt_values && cmt_digests && cmt_hashed), GG_ERR_INVALID_ARG,
                 "null BSB22 commitment data");
        GG_CHECK(proof_cap >= proof_size(k->curve, n_cmt), GG_ERR_INVALID_ARG, "proof buffer too small");
        std::lock_guard<std::mutex> lk(k->mu);
        GG_HIP(hipSetDevice(k->device));
        std::vector<FrT> pub(nb_public), hashed(n_cmt), blind;
        if (nb_public) memcpy(pub.data(), public_witness, 32 * nb_public);
        if (n_cmt) memcpy(hashed.data(), cmt_hashed, 32 * (size_t)n_cmt);
        std::vector<AffT> dg(n_cmt);
        if (n_cmt) memcpy(dg.data(), cmt_digests, pt * (size_t)n_cmt);
        if (blinding) {
            blind.resize(9);
            memcpy(blind.data(), blinding, 9 * 32);
        }
        const void* lro[3] = {l, r, o};
        typename Impl::PlonkProof P;
        double tms[8] = {0};
        Impl::prove(k, lro, inputs_on_device != 0, pub.data(), nb_public, cmt_values, dg.data(), hashed.data(), n_cmt,
                    blinding ? blind.data() : nullptr, Hasher{challenge_hash, challenge_ctx},
                    Hasher{folding_hash, folding_ctx}, P, tms);
        uint8_t* w = (uint8_t*)proof_out;
        auto put = [&](const void* src, size_t b) {
            memcpy(w, src, b);
            w += b;
        };
        for (auto& p : P.lro) put(&p, pt);
        put(&P.z, pt);
        for (auto& p : P.h) put(&p, pt);
        for (auto& p : P.bsb22) put(&p, pt);
        put(&P.batched_h, pt);
        for (auto& c : P.claimed) put(c.v, 32);
        put(&P.zs_h, pt);
        put(P.zs_value.v, 32);
        memcpy(g_plonk_ms, tms, sizeof(tms));
        return 0;
    });
    const bool rehearsal = with_key(pk, [](auto* k) { return k->solo && !k->peers.empty(); });
    if (gg::kAccumProbe) {
        gg::set_last_error("traffic-probe build (GG_ACCUM_PROBE): the MSM sums are wrong, the proof is NOT valid");
        return GG_REHEARSAL;
    }
    if (rehearsal) {
        gg::set_last_error("timing rehearsal (gg_plonk_pk_set_rehearsal): only one device part worked, the proof "
                           "is NOT valid");
        return GG_REHEARSAL;
    }
    GG_CAPI_END
}

extern "C" int gg_plonk_pk_set_rehearsal_part(gg_plonk_pk_t pk, int part) {
    GG_CAPI_BEGIN
    GG_CHECK(pk, GG_ERR_INVALID_ARG, "null key");
    with_key(pk, [&](auto* k) {
        std::lock_guard<std::mutex> lk(k->mu);
        GG_CHECK(part >= -1 && part <= (int)k->peers.size(), GG_ERR_INVALID_ARG, "rehearsal part out of range");
        using Impl = PlonkImpl<typename std::remove_pointer<decltype(k)>::type::CvT>;
        Impl::queue_layout(k, part);
        k->solo = part >= 0;
        k->solo_part = part >= 0 ? part : 0;
        return 0;
    });
    GG_CAPI_END
}

extern "C" int gg_plonk_pk_set_rehearsal(gg_plonk_pk_t pk, int on) { return gg_plonk_pk_set_rehearsal_part(pk, on ? 0 : -1); }

extern "C" int gg_plonk_pk_part_timings(gg_plonk_pk_t pk, int part, double* out, int cap) {
    GG_CAPI_BEGIN
    GG_CHECK(pk && out, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(cap >= GG_PLONK_PART_SLOTS, GG_ERR_INVALID_ARG, "cap < GG_PLONK_PART_SLOTS");
    with_key(pk, [&](auto* k) {
        std::lock_guard<std::mutex> lk(k->mu);
        GG_CHECK(part >= 0 && part <= (int)k->peers.size(), GG_ERR_INVALID_ARG, "part out of range");
        for (int i = 0; i < GG_PLONK_PART_SLOTS; i++) out[i] = 0;
        if (part >= (int)k->ptimes.size()) return 0;  // no proof yet
        std::lock_guard<std::mutex> lt(k->tmu);
        const PlonkPartTimes& T = k->ptimes[part];
        const double v[GG_PLONK_PART_SLOTS] = {T.msm_count,   T.msm_ms,    T.scalar_copy_ms,    T.scalar_mb,
                                               T.coset_count, T.coset_ms,  T.coset_in_copy_ms, T.coset_out_copy_ms,
                                               T.coset_mb,    T.wait_ms,   T.ratio_ms,        T.canon_count,
                                               T.canon_ms,    T.canon_mb};
        for (int i = 0; i < GG_PLONK_PART_SLOTS; i++) out[i] = v[i];
        return 0;
    });
    GG_CAPI_END
}

extern "C" int gg_plonk_pk_peer_access(gg_plonk_pk_t pk, int* codes, int cap, int* n_parts) {
    GG_CAPI_BEGIN
    GG_CHECK(pk && n_parts, GG_ERR_INVALID_ARG, "null argument");
    with_key(pk, [&](auto* k) {
        const int np = 1 + (int)k->peers.size();
        *n_parts = np;
        if (!codes) return 0;  // size query
        GG_CHECK(cap >= np * np, GG_ERR_INVALID_ARG, "cap < parts * parts");
        for (int i = 0; i < np * np; i++)
            codes[i] = i < (int)k->peer_codes.size() ? k->peer_codes[i] : GG_PEER_SAME_DEVICE;
        return 0;
    });
    GG_CAPI_END
}

extern "C" int gg_plonk_last_timings(double* ms, int cap) {
    GG_CAPI_BEGIN
    GG_CHECK(ms && cap >= 0, GG_ERR_INVALID_ARG, "null argument");
    memcpy(ms, g_plonk_ms, sizeof(double) * (size_t)std::min(cap, 8));
    GG_CAPI_END
}
