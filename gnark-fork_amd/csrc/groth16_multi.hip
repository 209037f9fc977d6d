// One-process multi-GPU Groth16 (SURVEY.md 8(b) "gg_init(ngpu)" shape, 8(e)):
// a Go (or any single-process) caller hands over the whole proving key once and
// gets proofs computed on `world` GPUs, with no transport of its own.
//
// This is the runtime layer a cgo caller would otherwise have to write around
// the per-shard entry points: it places key shard r on devices[r]
// (gg_groth16_pk_create_shard, slices cut as groth16.slice_key does), runs one
// host thread per shard through gg_groth16_prove_partial_dist, and performs the
// three all-to-alls of the distributed computeH itself -- peer copies
// (hipMemcpyPeerAsync, xGMI DMA between MI355X GPUs) between the shards' device
// buffers, fenced by an in-process barrier.  The 576-B partials are added with
// the exact group law and combined by gg_groth16_finalize (prove.go:206-299).
//
// devices[] may repeat a GPU: several shards on one device rehearse the
// N-GPU layout (the peer copy degenerates to a device-local copy), which is how
// the one-GPU tests check it bit-exact against the single-key prover.
#include "common.h"
#include <chrono>
#include <condition_variable>
#include <memory>
#include <cstring>
#include <mutex>
#include <algorithm>
#include <string>
#include <thread>
#include <vector>

struct gg_groth16_pk;
struct WireBases;
namespace gg {
std::shared_ptr<WireBases> g16_wire_bases(int curve, int log_n, const void* g1_A, size_t nA, const void* g1_B,
                                          size_t nB, const void* g1_K, size_t nK, const void* g2_B,
                                          const uint8_t* inf_A, const uint8_t* inf_B, size_t n_wires,
                                          size_t nb_public, const uint32_t* k_wire_index, size_t nZ);
gg_groth16_pk* g16_stripe_shard(std::shared_ptr<WireBases> wb, int curve, int log_n, const void* omega_mont,
                                const void* coset_gen_mont, const void* g1_Z, size_t z_lo, size_t nZ,
                                const void* alpha1, const void* beta1, const void* delta1, const void* beta2,
                                const void* delta2, size_t n_wires, size_t nb_public, int slog, uint32_t spart);
int g16_wire_window(int curve, size_t n_wires, size_t nB);
void g16_restream(gg_groth16_pk* pk, bool dedicated);
}  // namespace gg

namespace {

bool dist_h_ok(size_t n, int world) {
    return world >= 1 && world <= 16 && (world & (world - 1)) == 0 && n >= 2 && n >= (size_t)world * world;
}

}  // namespace

struct gg_groth16_mpk {
    int world = 0, curve = GG_CURVE_BN254;
    // how the A, B1, K and G2 MSMs are split: bucket stripes (every device holds
    // the whole wire tables, shard r takes the buckets b = r mod world) or wire
    // slices (shard r holds wires [r W / world, (r + 1) W / world))
    bool stripes = false;
    // gg_groth16_mpk_set_rehearsal(m, r) (timing rehearsal only): a prove runs
    // shard r ALONE -- its exchanges skip the peers, the other shards do
    // nothing -- so one GPU times the work one GPU of an N-GPU node does (less
    // the xGMI transfers); such a prove returns GG_REHEARSAL, never GG_OK
    int solo = -1;
    size_t n = 0, n_wires = 0;
    size_t g1a = 64, g2a = 128, g1j = 96, g2j = 192;  // the curve's point sizes
    bool dist = false;
    std::vector<int> dev;
    std::vector<gg_groth16_pk_t> pk;
    std::vector<gg_hshard_t> hs;
    std::vector<void*> send, recv;
    // per shard: one copy stream per destination, of the greatest priority
    // (common.h create_copy_stream: their own hardware queues)
    std::vector<std::vector<hipStream_t>> xst;
    uint8_t alpha1[96], beta1[96], delta1[96], beta2[192], delta2[192];
    gg::PartBarrier bar;  // the exchanges' meeting point (bounded: gg_set_wait_timeout)
    std::mutex mu;  // one proof at a time per key
    double last_ms[4] = {0, 0, 0, 0};
    // per shard, last proof: where its time went (gg_groth16_mpk_shard_timings)
    struct ShardTimes {
        double prove_ms = 0;
        int nx = 0;
        double wait_in[GG_MPK_MAX_EXCHANGES] = {}, copy[GG_MPK_MAX_EXCHANGES] = {},
               wait_out[GG_MPK_MAX_EXCHANGES] = {}, mbytes[GG_MPK_MAX_EXCHANGES] = {};
    };
    std::vector<ShardTimes> times;
    // peer access of shard i's device to shard j's (gg_groth16_mpk_peer_access):
    // GG_PEER_* codes, world x world
    std::vector<int> peer;
};

namespace {

struct XCtx {
    gg_groth16_mpk* m;
    int rank;
};

// gg_exchange_fn of shard `rank`: chunk k of its send buffer -> chunk rank of
// shard k's recv buffer.  First barrier: every shard's send is written and its
// recv no longer read (the caller synchronised its stream); second: every push
// into this shard's recv has landed.  The world pushes go out on one stream
// each, so the copies to the N-1 peers run at once over their own xGMI links
// (on one stream they would take the links one after another: at 2^24 over 8
// GPUs, 392 MB per shard per proof).
// Per exchange the shard records: the wait at the first barrier (peers still
// computing: load imbalance), the push time (its N-1 copies issued until all
// have landed: xGMI), and the wait at the second barrier (peers' pushes into
// it still in flight).
int mpk_exchange(void* ctx, const void* send_dev, void* recv_dev, size_t bytes) {
    XCtx* x = (XCtx*)ctx;
    gg_groth16_mpk* m = x->m;
    const int r = x->rank;
    (void)recv_dev;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    int rc = m->bar.wait("the shards' sends written (exchange, first barrier)");
    if (rc == GG_ERR_INTERNAL) gg::set_last_error("exchange aborted: another shard failed");
    if (rc) return rc;
    const auto t1 = clk::now();
    bool ok = hipSetDevice(m->dev[r]) == hipSuccess;
    size_t pushed = 0;
    for (int j = 0; ok && j < m->world; j++) {
        const int k = (r + j) % m->world;  // staggered: shard r starts with its own chunk, then r+1, ...
        if (m->solo >= 0 && k != r) continue;  // timing rehearsal: no peers
        ok = hipMemcpyPeerAsync((char*)m->recv[k] + (size_t)r * bytes, m->dev[k],
                                (const char*)send_dev + (size_t)k * bytes, m->dev[r], bytes,
                                m->xst[r][j]) == hipSuccess;
        if (k != r) pushed += bytes;
    }
    if (!ok) {
        (void)hipGetLastError();
        m->bar.abort();
        return GG_ERR_DEVICE;
    }
    try {
        gg::WaitScope ws("shard " + std::to_string(r) + " exchange " + std::to_string(m->times[r].nx + 1));
        for (int j = 0; j < m->world; j++) GG_WAIT_STREAM(m->xst[r][j]);  // its pushes have landed
    } catch (const gg::Error& e) {
        gg::set_last_error(e.what());
        m->bar.abort();
        return e.code;
    }
    const auto t2 = clk::now();
    const int rc2 = m->bar.wait("the peers' pushes into this shard (exchange, second barrier)");
    if (rc2 == GG_ERR_INTERNAL) gg::set_last_error("exchange aborted: another shard failed");
    const auto t3 = clk::now();
    auto& T = m->times[r];
    if (T.nx < GG_MPK_MAX_EXCHANGES) {
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        T.wait_in[T.nx] = ms(t0, t1);
        T.copy[T.nx] = ms(t1, t2);
        T.wait_out[T.nx] = ms(t2, t3);
        T.mbytes[T.nx] = pushed / 1e6;
    }
    T.nx++;
    return rc2;
}

// identity partials (Jacobian infinity: x = y = 1, z = 0 in Montgomery form --
// gg_g1_jac_add treats z = 0 as the identity whatever x, y hold)
void G16PartialsInf(int curve, uint8_t* p, size_t g1j, size_t g2j) {
    (void)curve;
    memset(p, 0, 4 * g1j + g2j);
}

void mpk_free(gg_groth16_mpk* m) {
    for (int r = 0; r < (int)m->dev.size(); r++) {
        if (hipSetDevice(m->dev[r]) != hipSuccess) continue;
        if (r < (int)m->pk.size() && m->pk[r]) gg_groth16_pk_release(m->pk[r]);
        if (r < (int)m->hs.size() && m->hs[r]) gg_hshard_release(m->hs[r]);
        if (r < (int)m->send.size() && m->send[r]) (void)hipFree(m->send[r]);
        if (r < (int)m->recv.size() && m->recv[r]) (void)hipFree(m->recv[r]);
        if (r < (int)m->xst.size())
            for (hipStream_t s : m->xst[r])
                if (s) (void)hipStreamDestroy(s);
    }
    delete m;
}

// run fn(r) on one host thread per shard (bound to its device); first error wins
template <class Fn>
void on_shards(gg_groth16_mpk* m, Fn fn) {
    std::mutex emu;
    std::string err;
    int code = GG_OK;
    bool echo_only = false;
    std::vector<gg::Task<void>> th;  // kept worker threads (common.h run_task); all shards run at once
    for (int r = 0; r < m->world; r++)
        th.push_back(gg::run_task([&, r] {
            int rc = gg_set_device(m->dev[r]);
            std::string msg = rc ? gg_last_error() : "";
            if (!rc) {
                rc = fn(r);
                if (rc) msg = gg_last_error();
            }
            if (rc) {
                m->bar.abort();
                std::lock_guard<std::mutex> g(emu);
                // the failing shard's own error wins over its peers' "another shard failed"
                const bool echo = msg.find("another shard failed") != std::string::npos;
                if (code == GG_OK || (echo_only && !echo)) {
                    code = rc;
                    echo_only = echo;
                    err = "shard " + std::to_string(r) + " (device " + std::to_string(m->dev[r]) + "): " + msg;
                }
            }
        }));
    for (auto& t : th) t.wait();
    if (code != GG_OK) throw gg::Error(code, err);
}

}  // namespace

extern "C" int gg_groth16_mpk_create_ex(int curve, int log_n, const void* omega_mont,
                                        const void* coset_gen_mont, const void* g1_A, size_t nA,
                                        const void* g1_B, size_t nB, const void* g1_Z, size_t nZ,
                                        const void* g1_K, size_t nK, const void* alpha1, const void* beta1,
                                        const void* delta1, const void* g2_B, const void* beta2,
                                        const void* delta2, const uint8_t* inf_A, const uint8_t* inf_B,
                                        size_t n_wires, size_t nb_public, const uint32_t* k_wire_index,
                                        int world, const int* devices, gg_groth16_mpk_t* out) {
    GG_CAPI_BEGIN
    GG_CHECK(out && alpha1 && beta1 && delta1 && beta2 && delta2 && inf_A && inf_B && devices, GG_ERR_INVALID_ARG,
             "null argument");
    GG_CHECK(curve == GG_CURVE_BN254 || curve == GG_CURVE_BLS12_381, GG_ERR_INVALID_ARG, "bad curve");
    GG_CHECK(world >= 1 && world <= 64, GG_ERR_INVALID_ARG, "world must be in [1, 64]");
    GG_CHECK(log_n >= 0 && log_n <= 28, GG_ERR_INVALID_ARG, "log_n out of range");
    const size_t n = (size_t)1 << log_n;
    GG_CHECK(nZ <= n, GG_ERR_INVALID_ARG, "more Z points than the domain");
    int ndev = 0;
    GG_HIP(hipGetDeviceCount(&ndev));
    for (int r = 0; r < world; r++)
        GG_CHECK(devices[r] >= 0 && devices[r] < ndev, GG_ERR_INVALID_ARG, "device id out of range");
    std::unique_ptr<gg_groth16_mpk, void (*)(gg_groth16_mpk*)> m(new gg_groth16_mpk, mpk_free);
    m->world = world;
    m->curve = curve;
    if (curve == GG_CURVE_BLS12_381) {
        m->g1a = 96;
        m->g2a = 192;
        m->g1j = 144;
        m->g2j = 288;
    }
    m->n = n;
    m->n_wires = n_wires;
    // the four-step distributed computeH (either curve's fr); a world it does
    // not support (not a power of two, n < world^2) replicates H on every shard
    m->dist = dist_h_ok(n, world);
    m->dev.assign(devices, devices + world);
    m->pk.assign(world, nullptr);
    m->hs.assign(world, nullptr);
    m->send.assign(world, nullptr);
    m->recv.assign(world, nullptr);
    m->xst.assign(world, {});
    m->bar.n = world;
    memcpy(m->alpha1, alpha1, m->g1a);
    memcpy(m->beta1, beta1, m->g1a);
    memcpy(m->delta1, delta1, m->g1a);
    memcpy(m->beta2, beta2, m->g2a);
    memcpy(m->delta2, delta2, m->g2a);
    // xGMI peer access between the distinct devices (copies work without it,
    // staged through host memory by the runtime -- which would look like slow
    // xGMI, so the outcome is kept per pair: gg_groth16_mpk_peer_access)
    m->peer = gg::enable_peer_access(m->dev);
    // prefix counts of the non-infinity A / B points (key order = wire order)
    std::vector<size_t> pa(n_wires + 1, 0), pb(n_wires + 1, 0);
    for (size_t w = 0; w < n_wires; w++) {
        pa[w + 1] = pa[w] + (inf_A[w] == 0);
        pb[w + 1] = pb[w] + (inf_B[w] == 0);
    }
    GG_CHECK(pa[n_wires] == nA && pb[n_wires] == nB, GG_ERR_INVALID_ARG,
             "point counts disagree with the infinity masks");
    const uint8_t* A = (const uint8_t*)g1_A;
    const uint8_t* B = (const uint8_t*)g1_B;
    const uint8_t* B2 = (const uint8_t*)g2_B;
    const uint8_t* K = (const uint8_t*)g1_K;
    const uint8_t* Z = (const uint8_t*)g1_Z;
    const size_t g1a = m->g1a, g2a = m->g2a;
    // Z positions of shard r: the slice the distributed computeH leaves on rank r
    auto zrange = [&](int r, size_t& zl, size_t& zh) {
        if (m->dist) {
            const size_t mm = n / world;
            zl = std::min(r * mm, n - 1);
            zh = std::min((r + 1) * mm, n - 1);
        } else {
            zl = (n - 1) * r / world;
            zh = (n - 1) * (r + 1) / world;
        }
        zl = std::min(zl, nZ);
        zh = std::min(zh, nZ);
    };
    // bucket stripes (GG_MPK_SPLIT=stripes, a power-of-two world whose windows
    // allow it): the whole wire tables once per device, each shard's A, B1, K,
    // G2 MSMs over its 2^-log2(world) of the buckets.  Wire slices are the
    // default: measured one shard at a time (GG_MPK_SOLO), a stripe shard of
    // the 2^24 key takes 21.1 ms against 19.3 for a wire shard at N = 8 (37.4 /
    // 35.9 at N = 4, 64.9 / 62.5 at N = 2): its digit pass and sort read all
    // n W entries, and its gathers span the whole 12.9-GB tables
    int slog = 0;
    while ((1 << slog) < world) slog++;
    {
        const char* e = getenv("GG_MPK_SPLIT");
        const bool want = e && strcmp(e, "stripes") == 0;
        m->stripes = want && world > 1 && (1 << slog) == world &&
                     slog <= gg::g16_wire_window(curve, n_wires, nB) - 2;
    }
    if (m->stripes) {
        std::vector<int> uniq;
        for (int d : m->dev)
            if (std::find(uniq.begin(), uniq.end(), d) == uniq.end()) uniq.push_back(d);
        std::vector<std::shared_ptr<WireBases>> wbs(uniq.size());
        std::vector<std::thread> th;
        std::mutex emu;
        std::string err;
        int code = GG_OK;
        for (size_t u = 0; u < uniq.size(); u++)
            th.emplace_back([&, u] {
                int rc = gg_set_device(uniq[u]);
                try {
                    if (rc) throw gg::Error(rc, gg_last_error());
                    size_t zdev = 0;  // Z points of the shards placed on this device
                    for (int r = 0; r < world; r++)
                        if (m->dev[r] == uniq[u]) {
                            size_t zl, zh;
                            zrange(r, zl, zh);
                            zdev += zh - zl;
                        }
                    wbs[u] = gg::g16_wire_bases(curve, log_n, g1_A, nA, g1_B, nB, g1_K, nK, g2_B, inf_A, inf_B,
                                                n_wires, nb_public, k_wire_index, zdev);
                } catch (const gg::Error& ex) {
                    std::lock_guard<std::mutex> g(emu);
                    if (code == GG_OK) { code = ex.code; err = ex.what(); }
                } catch (const std::exception& ex) {
                    std::lock_guard<std::mutex> g(emu);
                    if (code == GG_OK) { code = GG_ERR_INTERNAL; err = ex.what(); }
                }
            });
        for (auto& t : th) t.join();
        if (code != GG_OK) throw gg::Error(code, "wire tables (device): " + err);
        on_shards(m.get(), [&](int r) -> int {
            size_t zl, zh;
            zrange(r, zl, zh);
            const size_t u = std::find(uniq.begin(), uniq.end(), m->dev[r]) - uniq.begin();
            try {
                m->pk[r] = gg::g16_stripe_shard(wbs[u], curve, log_n, omega_mont, coset_gen_mont, Z + zl * g1a, zl,
                                                zh - zl, alpha1, beta1, delta1, beta2, delta2, n_wires, nb_public,
                                                slog, (uint32_t)r);
            } catch (const gg::Error& ex) {
                gg::set_last_error(ex.what());
                return ex.code;
            }
            if (!m->dist) return 0;
            m->xst[r].assign(world, nullptr);
            for (auto& x : m->xst[r]) gg::create_copy_stream(&x);  // own queues: pushes never wait behind MSMs
            int rc = gg_hshard_create_ex(curve, log_n, omega_mont, coset_gen_mont, r, world, &m->hs[r]);
            if (rc) return rc;
            size_t mm = 0, xb = 0;
            rc = gg_hshard_info(m->hs[r], &mm, &xb);
            if (rc) return rc;
            if (hipMalloc(&m->send[r], std::max<size_t>(xb, 256)) != hipSuccess ||
                hipMalloc(&m->recv[r], std::max<size_t>(xb, 256)) != hipSuccess)
                return GG_ERR_OOM;
            return 0;
        });
        *out = m.release();
        return GG_OK;
    }
    on_shards(m.get(), [&](int r) -> int {
        const size_t lo = n_wires * r / world, hi = n_wires * (r + 1) / world;
        size_t zl, zh;
        zrange(r, zl, zh);
        // K points of this shard's wires, with absolute wire ids
        std::vector<uint8_t> kp;
        std::vector<uint32_t> kidx;
        const uint8_t* kptr;
        size_t kcnt;
        const uint32_t* kix = nullptr;
        if (k_wire_index) {
            for (size_t j = 0; j < nK; j++)
                if (k_wire_index[j] >= lo && k_wire_index[j] < hi) {
                    kp.insert(kp.end(), K + j * g1a, K + (j + 1) * g1a);
                    kidx.push_back(k_wire_index[j]);
                }
            kptr = kp.data();
            kcnt = kidx.size();
            kix = kidx.data();
        } else {
            size_t k1 = std::max(hi, nb_public) - nb_public, k0 = std::max(lo, nb_public) - nb_public;
            k1 = std::min(k1, nK);
            k0 = std::min(k0, k1);
            kptr = K + k0 * g1a;
            kcnt = k1 - k0;
        }
        int rc = gg_groth16_pk_create_shard_ex(curve, log_n, omega_mont, coset_gen_mont, A + pa[lo] * g1a,
                                               pa[hi] - pa[lo], B + pb[lo] * g1a, pb[hi] - pb[lo], Z + zl * g1a, zl,
                                               zh - zl, kptr, kcnt, alpha1, beta1, delta1, B2 + pb[lo] * g2a, beta2,
                                               delta2, inf_A, inf_B, n_wires, nb_public, kix, lo, hi, &m->pk[r]);
        if (rc) return rc;
        if (!m->dist) return 0;
        m->xst[r].assign(world, nullptr);
        for (auto& x : m->xst[r]) gg::create_copy_stream(&x);  // own queues: pushes never wait behind MSMs
        rc = gg_hshard_create_ex(curve, log_n, omega_mont, coset_gen_mont, r, world, &m->hs[r]);
        if (rc) return rc;
        size_t mm = 0, xb = 0;
        rc = gg_hshard_info(m->hs[r], &mm, &xb);
        if (rc) return rc;
        if (hipMalloc(&m->send[r], std::max<size_t>(xb, 256)) != hipSuccess ||
            hipMalloc(&m->recv[r], std::max<size_t>(xb, 256)) != hipSuccess)
            return GG_ERR_OOM;
        return 0;
    });
    *out = m.release();
    GG_CAPI_END
}

extern "C" int gg_groth16_mpk_create(int log_n, const void* omega_mont, const void* coset_gen_mont,
                                     const void* g1_A, size_t nA, const void* g1_B, size_t nB,
                                     const void* g1_Z, size_t nZ, const void* g1_K, size_t nK,
                                     const void* alpha1, const void* beta1, const void* delta1,
                                     const void* g2_B, const void* beta2, const void* delta2,
                                     const uint8_t* inf_A, const uint8_t* inf_B, size_t n_wires,
                                     size_t nb_public, const uint32_t* k_wire_index, int world,
                                     const int* devices, gg_groth16_mpk_t* out) {
    return gg_groth16_mpk_create_ex(GG_CURVE_BN254, log_n, omega_mont, coset_gen_mont, g1_A, nA, g1_B, nB, g1_Z, nZ,
                                    g1_K, nK, alpha1, beta1, delta1, g2_B, beta2, delta2, inf_A, inf_B, n_wires,
                                    nb_public, k_wire_index, world, devices, out);
}

extern "C" int gg_groth16_mpk_release(gg_groth16_mpk_t m) {
    GG_CAPI_BEGIN
    if (m) mpk_free(m);
    GG_CAPI_END
}

extern "C" int gg_groth16_mpk_info(gg_groth16_mpk_t m, int* world, int* distributed_h) {
    GG_CAPI_BEGIN
    GG_CHECK(m, GG_ERR_INVALID_ARG, "null key");
    if (world) *world = m->world;
    if (distributed_h) *distributed_h = m->dist ? 1 : 0;
    GG_CAPI_END
}

extern "C" int gg_groth16_mpk_split(gg_groth16_mpk_t m, int* bucket_stripes) {
    GG_CAPI_BEGIN
    GG_CHECK(m && bucket_stripes, GG_ERR_INVALID_ARG, "null argument");
    *bucket_stripes = m->stripes ? 1 : 0;
    GG_CAPI_END
}

extern "C" int gg_groth16_mpk_base_info(gg_groth16_mpk_t m, int shard, int which, size_t* n_points,
                                        int* window_bits, int* n_windows) {
    GG_CAPI_BEGIN
    GG_CHECK(m && shard >= 0 && shard < m->world, GG_ERR_INVALID_ARG, "bad shard");
    return gg_groth16_pk_base_info(m->pk[shard], which, n_points, window_bits, n_windows);
    GG_CAPI_END
}

extern "C" int gg_groth16_mpk_devices(gg_groth16_mpk_t m, int* devices, int cap) {
    GG_CAPI_BEGIN
    GG_CHECK(m && devices && cap >= m->world, GG_ERR_INVALID_ARG, "null argument or cap < world");
    for (int r = 0; r < m->world; r++) devices[r] = m->dev[r];
    GG_CAPI_END
}

extern "C" int gg_groth16_mpk_prove_ex(gg_groth16_mpk_t m, int inputs_on_device, const void* const* wires,
                                       size_t n_wires, const void* const* sol_a, const void* const* sol_b,
                                       const void* const* sol_c, size_t n_cons, const void* r_mont,
                                       const void* s_mont, void* ar_aff, void* bs_aff, void* krs_aff) {
    GG_CAPI_BEGIN
    GG_CHECK(m && wires && sol_a && sol_b && sol_c && r_mont && s_mont && ar_aff && bs_aff && krs_aff,
             GG_ERR_INVALID_ARG, "null argument");
    for (int r = 0; r < m->world; r++)
        GG_CHECK(wires[r] && sol_a[r] && sol_b[r] && sol_c[r], GG_ERR_INVALID_ARG, "null solution pointer");
    GG_CHECK(n_wires == m->n_wires, GG_ERR_INVALID_ARG, "wire count differs from the key's");
    GG_CHECK(n_cons <= m->n, GG_ERR_INVALID_ARG, "more constraints than the domain");
    std::lock_guard<std::mutex> lk(m->mu);
    const auto t0 = std::chrono::steady_clock::now();
    // the fixed-point terms (r.delta, s.delta, kr.delta, s.delta2) on host
    // threads while the shards prove
    gg_g16_fixed_t fx = nullptr;
    {
        const int rc = gg_groth16_finalize_begin(m->curve, m->delta1, m->delta2, r_mont, s_mont, &fx);
        GG_CHECK(rc == GG_OK, rc, gg_last_error());
    }
    struct FxGuard {
        gg_g16_fixed_t& h;
        ~FxGuard() { if (h) gg_groth16_finalize_end(h, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr); }
    } fx_guard{fx};
    m->bar.n = m->solo >= 0 ? 1 : m->world;
    m->bar.reset();
    const size_t pbytes = 4 * m->g1j + m->g2j;  // a | b1 | k | z | b2 (gg_groth16_prove_partial)
    std::vector<std::vector<uint8_t>> parts(m->world, std::vector<uint8_t>(pbytes));
    std::vector<XCtx> ctx(m->world);
    m->times.assign(m->world, gg_groth16_mpk::ShardTimes());
    on_shards(m, [&](int r) -> int {
        ctx[r] = XCtx{m, r};
        if (m->solo >= 0 && r != m->solo) {  // timing rehearsal: identity partials
            G16PartialsInf(m->curve, parts[r].data(), m->g1j, m->g2j);
            return 0;
        }
        const auto a = std::chrono::steady_clock::now();
        int rc;
        if (m->dist)
            rc = gg_groth16_prove_partial_dist(m->pk[r], m->hs[r], wires[r], n_wires, sol_a[r], sol_b[r], sol_c[r],
                                               n_cons, inputs_on_device, mpk_exchange, &ctx[r], m->send[r],
                                               m->recv[r], parts[r].data());
        else
            rc = gg_groth16_prove_partial(m->pk[r], wires[r], n_wires, sol_a[r], sol_b[r], sol_c[r], n_cons,
                                          inputs_on_device, parts[r].data(), nullptr);
        m->times[r].prove_ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
        return rc;
    });
    const auto t1 = std::chrono::steady_clock::now();
    // exact sum of the partials: 4 G1Jac then one G2Jac
    const bool bn = m->curve == GG_CURVE_BN254;
    auto g1add = bn ? gg_g1_jac_add : gg_bls12_381_g1_jac_add;
    auto g2add = bn ? gg_g2_jac_add : gg_bls12_381_g2_jac_add;
    std::vector<uint8_t> sum = parts[0];
    for (int r = 1; r < m->world; r++) {
        uint8_t tmp[288];
        for (int i = 0; i < 4; i++) {
            uint8_t* acc = sum.data() + m->g1j * i;
            GG_CHECK(g1add(acc, parts[r].data() + m->g1j * i, tmp) == GG_OK, GG_ERR_INTERNAL, "partial sum");
            memcpy(acc, tmp, m->g1j);
        }
        uint8_t* acc2 = sum.data() + 4 * m->g1j;
        GG_CHECK(g2add(acc2, parts[r].data() + 4 * m->g1j, tmp) == GG_OK, GG_ERR_INTERNAL, "partial sum");
        memcpy(acc2, tmp, m->g2j);
    }
    gg_g16_fixed_t h = fx;
    fx = nullptr;  // end releases it
    const int rc = gg_groth16_finalize_end(h, m->alpha1, m->beta1, m->beta2, sum.data(), ar_aff, bs_aff, krs_aff);
    GG_CHECK(rc == GG_OK, rc, gg_last_error());
    const auto t2 = std::chrono::steady_clock::now();
    m->last_ms[0] = std::chrono::duration<double, std::milli>(t1 - t0).count();
    m->last_ms[1] = std::chrono::duration<double, std::milli>(t2 - t1).count();
    m->last_ms[2] = std::chrono::duration<double, std::milli>(t2 - t0).count();
    if (gg::kAccumProbe || m->solo >= 0) {
        if (gg::kAccumProbe) {
            gg::set_last_error("traffic-probe build (GG_ACCUM_PROBE): the MSM sums are wrong, the proof is NOT valid");
            return GG_REHEARSAL;
        }
        gg::set_last_error("timing rehearsal (gg_groth16_mpk_set_rehearsal): shard " + std::to_string(m->solo) +
                           " proved alone, the proof is NOT valid");
        return GG_REHEARSAL;
    }
    GG_CAPI_END
}

extern "C" int gg_groth16_mpk_prove(gg_groth16_mpk_t m, const void* wires, size_t n_wires, const void* sol_a,
                                    const void* sol_b, const void* sol_c, size_t n_cons, const void* r_mont,
                                    const void* s_mont, void* ar_aff, void* bs_aff, void* krs_aff) {
    GG_CAPI_BEGIN
    GG_CHECK(m, GG_ERR_INVALID_ARG, "null key");
    // host inputs: every shard reads the same host vectors
    const std::vector<const void*> w(m->world, wires), a(m->world, sol_a), b(m->world, sol_b), c(m->world, sol_c);
    return gg_groth16_mpk_prove_ex(m, 0, w.data(), n_wires, a.data(), b.data(), c.data(), n_cons, r_mont, s_mont,
                                   ar_aff, bs_aff, krs_aff);
    GG_CAPI_END
}

extern "C" int gg_groth16_mpk_last_timings(gg_groth16_mpk_t m, double* ms3) {
    GG_CAPI_BEGIN
    GG_CHECK(m && ms3, GG_ERR_INVALID_ARG, "null argument");
    for (int i = 0; i < 3; i++) ms3[i] = m->last_ms[i];
    GG_CAPI_END
}

extern "C" int gg_groth16_mpk_set_rehearsal(gg_groth16_mpk_t m, int solo_shard) {
    GG_CAPI_BEGIN
    GG_CHECK(m, GG_ERR_INVALID_ARG, "null key");
    GG_CHECK(solo_shard >= -1 && solo_shard < m->world, GG_ERR_INVALID_ARG, "solo shard out of range");
    std::lock_guard<std::mutex> lk(m->mu);
    // shards sharing a device share its dedicated hardware queues (common.h
    // task_streams_switch): the solo shard gets them, as on a node
    if (solo_shard >= 0 && solo_shard != m->solo) {
        for (int r = 0; r < m->world; r++)
            if (r != solo_shard && m->dev[r] == m->dev[solo_shard]) gg::g16_restream(m->pk[r], false);
        gg::g16_restream(m->pk[solo_shard], true);
    } else if (solo_shard < 0 && m->solo >= 0) {
        // back to the creation layout: every shard released, then
        // re-created in shard order, as gg_groth16_mpk_create placed them
        for (int r = 0; r < m->world; r++) gg::g16_restream(m->pk[r], false);
        for (int r = 0; r < m->world; r++) gg::g16_restream(m->pk[r], true);
    }
    m->solo = solo_shard;
    GG_CAPI_END
}

extern "C" int gg_groth16_mpk_peer_access(gg_groth16_mpk_t m, int* codes, int cap) {
    GG_CAPI_BEGIN
    GG_CHECK(m && codes, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(cap >= m->world * m->world, GG_ERR_INVALID_ARG, "cap < world * world");
    for (int i = 0; i < m->world * m->world; i++) codes[i] = m->peer[i];
    GG_CAPI_END
}

extern "C" int gg_groth16_mpk_shard_timings(gg_groth16_mpk_t m, int shard, double* out, int cap) {
    GG_CAPI_BEGIN
    GG_CHECK(m && out, GG_ERR_INVALID_ARG, "null argument");
    GG_CHECK(shard >= 0 && shard < m->world, GG_ERR_INVALID_ARG, "shard out of range");
    GG_CHECK(cap >= GG_MPK_TIMING_SLOTS, GG_ERR_INVALID_ARG, "cap < GG_MPK_TIMING_SLOTS");
    std::lock_guard<std::mutex> lk(m->mu);
    for (int i = 0; i < GG_MPK_TIMING_SLOTS; i++) out[i] = 0;
    if (shard >= (int)m->times.size()) return GG_OK;  // no proof yet
    const auto& T = m->times[shard];
    out[0] = T.prove_ms;
    const int nx = std::min(T.nx, GG_MPK_MAX_EXCHANGES);
    out[1] = nx;
    for (int e = 0; e < nx; e++) {
        out[2 + 4 * e] = T.wait_in[e];
        out[3 + 4 * e] = T.copy[e];
        out[4 + 4 * e] = T.wait_out[e];
        out[5 + 4 * e] = T.mbytes[e];
    }
    GG_CAPI_END
}
