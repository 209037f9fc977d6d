// Host -> HBM upload of per-proof inputs through pinned staging buffers.
//
// gnark hands the prover host slices (solution.W/A/B/C, icicle.go:231-278,
// 478-480).  A pageable hipMemcpy of those 2 GB (2^24 constraints) is a single
// host-synchronous copy at a fraction of the PCIe rate.  The stager instead
// splits the copy into chunks; NT host threads each memcpy their chunks into
// their own pair of pinned buffers and issue the DMA on their own stream, so
// host copies, DMAs and the GPU's kernels all overlap.  When upload() returns
// the caller's buffer is no longer referenced (the cgo rule: C keeps no Go
// pointer past the call); the DMAs may still be in flight, and ready() makes
// consumer streams wait for them.
#pragma once
#include "common.h"
#include <mutex>
#include <vector>

namespace gg {

class Stager {
public:
    static constexpr int NT = 16;                    // max host copy threads (= DMA streams)
    static constexpr size_t CHUNK = (size_t)8 << 20;  // bytes per staged chunk
    explicit Stager(int device);
    ~Stager();
    Stager(const Stager&) = delete;
    Stager& operator=(const Stager&) = delete;
    // dst_dev[0 .. bytes) = src_host[0 .. bytes)
    void upload(void* dst_dev, const void* src_host, size_t bytes);
    // dst_dev[j] = src_host[first + stride * j] for j < count (elem_bytes each):
    // the cyclic slice a rank of the distributed computeH needs
    void upload_strided(void* dst_dev, const void* src_host, size_t elem_bytes, size_t first,
                        size_t stride, size_t count);
    // every stream in `consumers` waits (device side) for all uploads so far
    void ready(const hipStream_t* consumers, int k);
    void sync();

private:
    void run(void* dst, const void* src, size_t elem, size_t first, size_t stride, size_t count);
    int device_;
    int nt_ = 8;   // copy threads used (GG_STAGE_NT, <= NT)
    int nst_ = 1;  // DMA streams (GG_STAGE_STREAMS, <= nt_)
    void* pin_[NT][2] = {};
    hipEvent_t ev_[NT][2] = {};
    hipEvent_t end_[NT] = {};
    hipStream_t st_[NT] = {};
    int next_[NT] = {};
    std::mutex mu_;
};

}  // namespace gg
