// Pinned, multi-threaded host -> HBM staging (stage.h).
#include "stage.h"
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <thread>

namespace gg {

Stager::Stager(int device) : device_(device) {
    if (const char* e = getenv("GG_STAGE_NT")) nt_ = std::max(1, std::min(NT, atoi(e)));  // tuning
    if (const char* e = getenv("GG_STAGE_STREAMS")) nst_ = std::max(1, std::min(nt_, atoi(e)));
    for (int t = 0; t < nt_; t++) {
        for (int b = 0; b < 2; b++) {
            GG_HIP(hipHostMalloc(&pin_[t][b], CHUNK, hipHostMallocDefault));
            GG_HIP(hipEventCreateWithFlags(&ev_[t][b], hipEventDisableTiming));
        }
        GG_HIP(hipEventCreateWithFlags(&end_[t], hipEventDisableTiming));
        // one DMA stream shared by the copy threads (GG_STAGE_STREAMS=1, default),
        // of the greatest priority: its own hardware queue, so the H2D copies
        // never queue behind an MSM kernel of the prove's streams (common.h)
        if (t < nst_) create_copy_stream(&st_[t]);
        else st_[t] = st_[t % nst_];
    }
}

Stager::~Stager() {
    for (int t = 0; t < NT; t++) {
        if (st_[t]) (void)hipStreamSynchronize(st_[t]);
        for (int b = 0; b < 2; b++) {
            if (pin_[t][b]) (void)hipHostFree(pin_[t][b]);
            if (ev_[t][b]) (void)hipEventDestroy(ev_[t][b]);
        }
        if (end_[t]) (void)hipEventDestroy(end_[t]);
        if (st_[t] && t < nst_) (void)hipStreamDestroy(st_[t]);
    }
}

void Stager::run(void* dst, const void* src, size_t elem, size_t first, size_t stride, size_t count) {
    if (!count) return;
    std::lock_guard<std::mutex> lk(mu_);
    const size_t per = CHUNK / elem;  // elements per chunk
    const size_t nchunks = (count + per - 1) / per;
    const int nt = (int)std::min<size_t>(nt_, nchunks);
    std::string err;
    std::mutex emu;
    auto worker = [&](int t) {
        try {
            GG_HIP(hipSetDevice(device_));
            for (size_t k = (size_t)t; k < nchunks; k += (size_t)nt) {
                const size_t j0 = k * per, cnt = std::min(per, count - j0);
                const int b = next_[t];
                next_[t] ^= 1;
                GG_WAIT_EVENT(ev_[t][b]);  // previous DMA out of this buffer
                uint8_t* pin = (uint8_t*)pin_[t][b];
                const uint8_t* s = (const uint8_t*)src;
                if (stride == 1) {
                    memcpy(pin, s + (first + j0) * elem, cnt * elem);
                } else {
                    for (size_t j = 0; j < cnt; j++)
                        memcpy(pin + j * elem, s + (first + (j0 + j) * stride) * elem, elem);
                }
                GG_HIP(hipMemcpyAsync((uint8_t*)dst + j0 * elem, pin, cnt * elem, hipMemcpyHostToDevice,
                                      st_[t]));
                GG_HIP(hipEventRecord(ev_[t][b], st_[t]));
            }
        } catch (const std::exception& e) {
            std::lock_guard<std::mutex> g(emu);
            err = e.what();
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; t++) th.emplace_back(worker, t);
    worker(0);
    for (auto& x : th) x.join();
    GG_CHECK(err.empty(), GG_ERR_DEVICE, "host staging upload: " + err);
}

void Stager::upload(void* dst_dev, const void* src_host, size_t bytes) {
    run(dst_dev, src_host, 1, 0, 1, bytes);
}

void Stager::upload_strided(void* dst_dev, const void* src_host, size_t elem_bytes, size_t first,
                            size_t stride, size_t count) {
    GG_CHECK(elem_bytes && elem_bytes <= CHUNK, GG_ERR_INVALID_ARG, "bad element size");
    run(dst_dev, src_host, elem_bytes, first, stride, count);
}

void Stager::ready(const hipStream_t* consumers, int k) {
    std::lock_guard<std::mutex> lk(mu_);
    for (int t = 0; t < nst_; t++) {
        GG_HIP(hipEventRecord(end_[t], st_[t]));
        for (int i = 0; i < k; i++) GG_HIP(hipStreamWaitEvent(consumers[i], end_[t], 0));
    }
}

void Stager::sync() {
    std::lock_guard<std::mutex> lk(mu_);
    for (int t = 0; t < nst_; t++) GG_WAIT_STREAM(st_[t]);
}

}  // namespace gg
