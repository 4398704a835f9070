// gpu_encoder.h -- device side of one encode (buffers, stream, stage kernels).
#pragma once

#include <hip/hip_runtime.h>

#include <functional>
#include <string>
#include <vector>

#include "jp2hip_internal.h"

namespace jp2hip {

struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
};

struct StageTimes {
    double ingest = 0, dwt = 0, quant = 0, t1_cm = 0, t1_mq = 0, pcrd = 0, d2h = 0;
};

// tier-1 kernels (t1.hip)
struct T1CmArgs {
    const int2 *items;  // (block, plane)
    int nitems;
    const BlockDesc *blocks;
    const uint64_t *bp;
    const int32_t *sm;
    const uint8_t *P;
    uint8_t *stream;
    const uint64_t *slot_off;
    uint4 *counts;    // [block][32] (end of SPP, end of MRP, end of CUP)
    int64_t *dspp;    // [block][32]
    int lossless;
};
struct T1MqArgs {
    const BlockDesc *blocks;
    const int32_t *order;
    int nblocks;
    const uint8_t *P;
    const uint8_t *pmin;  // lowest coded plane (slope prediction; 0 = all)
    const uint8_t *stream;
    const uint64_t *slot_off;
    const uint4 *counts;
    const int64_t *dspp, *dref, *dsig;
    uint8_t *out;
    int32_t *rates;
    int64_t *dists;
    uint8_t *npasses;
    int32_t *lengths;
    int *err;
    int lanes;  // blocks per wavefront (1..64)
    unsigned long long *span;  // [2] execution span in 100 MHz ticks (min start, max end)
    int64_t *dbg;  // optional per-block census [block][4] (debug)
};
// fused ingest + DWT (dwt.hip)
struct DwtLaunch {
    const void *tif;
    const uint64_t *strip_off;
    int rps, img_w, nc, bits, planar, big_endian, mct, spp_strips;
    int ntx, tile_w, tile_h, row0, plane_w, plane_h, ntc, levels, reversible;
    const int32_t *tc_w, *tc_h;
    void *coef, *scratch0, *scratch1;  // scratch: ntc * ceil(plane_w/2) * ceil(plane_h/2) words each
};
bool launch_dwt(const DwtLaunch &p, hipStream_t st);

void launch_t1_cm(const T1CmArgs &a, hipStream_t st);
void launch_t1_keys(int nblocks, const uint8_t *P, const uint8_t *pmin, const uint4 *counts, uint32_t *keys,
                    int32_t *vals, hipStream_t st);
void launch_t1_mq(const T1MqArgs &a, hipStream_t st);
uint32_t t1_plane_stream_cap(int w, int h);

// Owns all device memory of a context; buffers only grow, so repeated
// encodes of the same geometry never allocate.
class GpuEncoder {
  public:
    ~GpuEncoder();
    bool init(int device, std::string &err);

    // host -> device copy of a source buffer into the internal `src` buffer
    bool upload_source(const void *host, size_t len, std::string &err);
    const void *source() const { return src.ptr; }
    // LZW / PackBits strips (+ Predictor 2) -> an uncompressed staging copy
    // in HBM; `out` describes it (offsets in out_offs)
    bool unpack_strips(const void *d_src, const jp2hip_layout &lay, jp2hip_layout &out,
                       std::vector<uint64_t> &out_offs, const void **d_out, std::string &err);

    // Sums a slope-prediction histogram over the ranks of a tile-split
    // encode, in place; false = exchange failed (or another rank failed).
    using HistReduce = std::function<bool(std::vector<int64_t> &)>;
    // ingest, DWT, quantiser, tier-1, hulls; downloads per-block totals.
    // skip_target > 0: rate-driven encode of skip_target bytes with slope
    // prediction (bit-planes far below the predicted threshold not coded);
    // reduce (tile-split only) makes the prediction global.
    bool run_front(const void *d_src, const jp2hip_layout &lay, const Plan &plan, bool profile,
                   StageTimes &st, std::string &err, int64_t skip_target = 0,
                   const HistReduce *reduce = nullptr);
    // layer thresholds for the given data budgets -> per-block layer tables
    bool select(const Plan &plan, const std::vector<int64_t> &budgets, std::vector<uint8_t> &h_nl,
                std::vector<int32_t> &h_lrate, bool profile, StageTimes &st, std::string &err);
    // per-block layer tables for explicit slope thresholds K[layer]
    // (tile-split: thresholds agreed across ranks)
    bool select_keys(const Plan &plan, const std::vector<uint64_t> &K, std::vector<uint8_t> &h_nl,
                     std::vector<int32_t> &h_lrate, bool profile, StageTimes &st, std::string &err);
    // this encode's hull segments: slope keys (descending) and inclusive byte sums
    bool segments(std::vector<uint64_t> &keys, std::vector<int64_t> &cum, std::string &err);
    // compact the included bytes of every block and download them
    bool gather(const Plan &plan, const std::vector<int32_t> &final_len,
                const std::vector<uint64_t> &offsets, uint64_t total, const uint8_t **host_data,
                bool profile, StageTimes &st, std::string &err);

    bool t1_total_bytes(int64_t &bytes, int64_t &passes) const;
    const std::vector<int32_t> &block_lengths() const { return h_lengths; }
    const std::vector<uint8_t> &block_passes() const { return h_npasses; }
    const std::vector<uint8_t> &block_planes() const { return h_P; }
    const std::vector<uint8_t> &block_pmin() const { return h_pmin; }
    hipStream_t get_stream() const { return stream; }

  private:
    // debug: JP2HIP_DUMP_DIR=<dir> writes every stage's device buffer
    bool dump(const char *dir, const char *name, const DevBuf &b, size_t bytes, std::string &err);
    bool apply_thresholds(const Plan &plan, std::vector<uint8_t> &h_nl, std::vector<int32_t> &h_lrate,
                          bool profile, StageTimes &st, std::string &err);
    bool host_wait(std::string &err);
    static constexpr int kNumEvents = 12;
    int device = 0;
    hipEvent_t sync_ev = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev[kNumEvents] = {};
    DevBuf coef, blocks, order, bp, sm, P, dref, dsig, t1out, rates, dists, npasses, lengths, weight,
        nhull, hpass, hkey, budget, nl, lrate, dstoff, packed, err, tcw, tch, strips, src, segcnt, segoff,
        est, hist, kcut, pmin, mqspan, stage, soff, lzwtab, untiled, segkey, segkey2, llbuf0, llbuf1, ordkey, ordkey2, ordval, segval, segval2, segcum, thr, cubtmp, items, slotoff, stream_buf, counts, dspp,
        dbgbuf;
    int nseg = 0;
    uint8_t *h_packed = nullptr;
    size_t h_packed_cap = 0;
    std::vector<int32_t> h_lengths;
    std::vector<uint8_t> h_npasses, h_P, h_pmin;
    std::vector<int64_t> h_hist;
    std::vector<int2> h_items;
    std::vector<uint64_t> h_slot;
};

}  // namespace jp2hip
