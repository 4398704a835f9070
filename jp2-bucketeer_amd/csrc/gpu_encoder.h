// gpu_encoder.h -- device side of one encode (buffers, stream, stage kernels).
#pragma once

#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdint>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "jp2hip_internal.h"

namespace jp2hip {

struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
    size_t want = 0;  // bytes the current encode asked for (need accounting)
};

struct StageTimes {
    double ingest = 0, dwt = 0, quant = 0, t1_cm = 0, t1_mq = 0, pcrd = 0, d2h = 0, t2 = 0;
};

struct T2Args;  // t2_device.hip

// compressed strips / tiles -> uncompressed staging copy (kernels.hip, lzw.hip)
struct UnpackArgs {
    const uint8_t *src;
    const uint64_t *off, *cnt;  // per strip (tile): byte offset and compressed size
    int nstrips, per_plane, rps, h;
    uint64_t row_bytes, stride;  // decoded row and strip stride (bytes)
    uint64_t unit_bytes;         // tiles: every unit decodes to this many bytes
    uint8_t *dst;
    const int *only;  // k_unlzw: decode only strips with only[s] != 0 (nullptr: all)
    int *err;
    uint32_t *lnk;    // k_inflate: a link per output byte, strip s at lnk + s * stride
};
__host__ __device__ inline uint64_t strip_out_bytes(const UnpackArgs &a, int s) {
    if (a.unit_bytes) return a.unit_bytes;
    const int y0 = (s % a.per_plane) * a.rps;
    return (uint64_t)(a.rps < a.h - y0 ? a.rps : a.h - y0) * a.row_bytes;
}
// LZW strips, segment-parallel (lzw.hip): lzw_slices() lays out each
// strip's segment slots (returns their total), the caller uploads `slice` to
// the start of `scratch` (lzw_scratch_bytes); false on a launch error
uint64_t lzw_slices(const uint64_t *strip_bytes, int nstrips, std::vector<uint64_t> &slice);
size_t lzw_scratch_bytes(int nstrips, uint64_t segs);
bool launch_lzw(const UnpackArgs &u, uint64_t segs, void *scratch, hipStream_t st);

// the SDMA engines chosen per GPU and their probed rates (t2_device.hip)
std::string dma_engine_report();

// tier-1 kernels (t1.hip)
#ifndef JP2HIP_ORDER_SUB
#define JP2HIP_ORDER_SUB 16  // MQ lane-order buckets per octave of decision count
#endif
constexpr int kOrderSub = JP2HIP_ORDER_SUB;
constexpr int kOrderBuckets = 32 * kOrderSub;  // MQ lane-order buckets (decision count, 6.25 % wide)
// Work lists of k_t1_cm3, filled once the coded planes are known
// (emit_t1_items: k_plane_pmin, or k_t1_items without slope prediction):
// list k holds the blocks with more than k coded planes (item = plane k from
// the top of that block), in no particular order.
struct T1ItemArgs {
    int nb, kmax;               // kmax: largest Mb of the plan (<= 64)
    const uint8_t *P;
    uint8_t *pmin;              // k_t1_items writes 0 (every plane coded)
    uint32_t *dfill;            // [64] list fills (zeroed by k_quant)
    int32_t *dlist;             // [kmax][nb]
    unsigned long long *acc;    // [nb] (coded planes << 40): k_t1_cm3 counts planes down, decisions up
    uint8_t *npasses;           // blocks without a coded plane: 0 passes, 0 bytes (k_t1_mq never sees them)
    int32_t *lengths;
    // decision-stream slots, placed here (emit_t1_items)
    const BlockDesc *blocks;
    unsigned long long *pool_used;  // zeroed by k_quant; ends at the bytes needed
    unsigned long long pool_cap;    // bytes in the pool (stream_buf)
    uint64_t *slot_off;             // [nb]
    int *err;                       // kErrSlotPool when a block did not fit
};
struct T1CmArgs {
    const uint32_t *dfill;  // per-depth list fills
    const int32_t *dlist;
    int nb, kmax;
    int max_items;          // bound on the items (nb * kmax): the grid
    const BlockDesc *blocks;
    const uint64_t *bp;
    const int32_t *sm;
    const uint8_t *P;
    uint8_t *stream;
    const uint64_t *slot_off;
    uint4 *counts;    // [block][32] (end of SPP, end of MRP, end of CUP)
    int64_t *dspp;    // [block][32]
    unsigned long long *acc;  // [block] (planes left << 40) | decisions so far
    uint32_t *bfill;          // [256] MQ lane-order bucket fills (zeroed by k_quant)
    int32_t *bslots;          // [256][nb] blocks per bucket
    int lossless;
};
struct T1MqArgs {
    const BlockDesc *blocks;
    const uint32_t *bfill;   // lane order: bucket fills and members (k_t1_cm3)
    const int32_t *bslots;
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
    unsigned long long *span;  // [2] execution span in 100 MHz ticks (~min start, max end)
    int64_t *dbg;  // optional per-block census [block][6] (debug builds: decisions, modeller cycles
                   // and barrier cycles, coder cycles and barrier cycles, lane position)
};
// fused ingest + DWT (dwt.hip)
struct DwtLaunch {
    const void *tif;
    const uint64_t *strip_off;
    int rps, img_w, nc, bits, planar, big_endian, mct, spp_strips;
    int ntx, tile_w, tile_h, row0, plane_w, plane_h, ntc, levels, reversible;
    int last_tile_w;  // width of the last tile column (the others are tile_w)
    const int32_t *tc_w, *tc_h;
    void *coef, *scratch0, *scratch1;  // scratch: ntc * ceil(plane_w/2) * ceil(plane_h/2) words each
    QuantTab qt;                       // final coefficients are written as quantisation indices
};
bool launch_dwt(const DwtLaunch &p, hipStream_t st);

void launch_t1_cm(const T1CmArgs &a, hipStream_t st);
void launch_t1_items(const T1ItemArgs &a, hipStream_t st);
void launch_t1_mq(const T1MqArgs &a, hipStream_t st);
uint32_t t1_plane_stream_cap(int w, int h);

// Owns all device memory of a context; buffers only grow while the context
// stays within its soft limit, so repeated encodes of the same geometry never
// allocate.  Every allocation goes through ensure(), which keeps the total
// (device_bytes) and refuses to pass the hard limit; trim() releases every
// buffer after an image that left the context above its soft limit.
class GpuEncoder {
  public:
    ~GpuEncoder();
    bool init(int device, std::string &err);

    // device memory held by this context's buffers
    size_t device_bytes() const { return held; }
    // hard: no buffer may take the total past it (the encode fails with an
    // error -- before its kernels, or between them on a stream that is then
    // drained -- instead of faulting); soft: an encode that leaves the
    // context above it releases every buffer at its end (trim)
    void set_limits(size_t soft, size_t hard) {
        mem_soft = soft;
        mem_hard = hard;
    }
    size_t soft_limit() const { return mem_soft; }
    size_t hard_limit() const { return mem_hard; }
    // releases every device buffer if more than `soft` bytes are held (the
    // stream must be idle: called after an encode's last wait); true if it did
    bool trim(size_t soft);
    // need accounting: begin_encode() clears every buffer's request, and
    // need_bytes() is what this encode asked for (held may be more: buffers
    // keep the size of the largest image since the last trim)
    void begin_encode() {
        for (DevBuf *b : bufs()) b->want = 0;
    }
    size_t need_bytes() {
        size_t n = 0;
        for (DevBuf *b : bufs()) n += b->want;
        return n;
    }
    // called when hipMalloc fails: frees what other, idle contexts of the
    // device hold (api.cpp); true if anything was released
    std::function<bool()> reclaim;
    // waits for the stream, ignoring its errors (failure paths: no buffer is
    // released or reused while kernels may still read it)
    void quiesce();
    template <typename T>
    bool ensure(DevBuf &b, size_t count, std::string &err);

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
    // pool_worst: size the decision-stream pool for every plane of every
    // block (the tile-split path, whose ranks cannot repeat an exchange);
    // else the encode may end with kErrSlotPool in its summary's err, and
    // the caller grows the pool (pool_grow) and encodes again.
    bool run_front(const void *d_src, const jp2hip_layout &lay, const Plan &plan, bool profile,
                   StageTimes &st, std::string &err, int64_t skip_target = 0,
                   const HistReduce *reduce = nullptr, bool pool_worst = false);
    // after an encode that ended with kErrSlotPool: the next run_front
    // sizes the pool for what that encode needed (+12.5 %)
    bool pool_grow(std::string &err);
    size_t stream_pool_bytes() const { return stream_buf.bytes; }
    int take_pool_grows() {
        const int g = pool_grows;
        pool_grows = 0;
        return g;
    }
    // lossless "-rate -": per -flush_period stripe (the plan's rate-control
    // groups), layer budgets lossless_layer_frac of the stripe's tier-1
    // bytes, computed on the device (enqueued only; t2_size reads the result)
    bool select_lossless(const Plan &plan, std::string &err);
    // per-block layer tables for explicit slope thresholds K[layer]
    // (tile-split: thresholds agreed across ranks)
    bool select_keys(const Plan &plan, const std::vector<uint64_t> &K, std::string &err);
    // tier-2 on the device (t2_device.hip): tables for the tiles coded, one sizing
    // pass per layer table (one host wait: the summary), then the code-stream
    // part (tile-parts, in stream order) written in HBM and copied to host_dst
    bool t2_load(const Plan &plan, const T2Tables &T, std::string &err);
    bool t2_size(const Plan &plan, bool with_kc, bool profile, StageTimes &st, T2Summary &sum, std::string &err);
    // rate-driven encode: the whole rate loop on the device (RateState),
    // `batch` iterations enqueued per host wait; returns the final state and
    // the summary of the selection it stopped at.  restart = begin a new loop
    // (else continue the one on the device).
    bool rate_loop(const Plan &plan, const RateState &init, bool restart, int batch, bool profile, StageTimes &st,
                   RateState &rs, T2Summary &sum, std::string &err);
    // the device code-stream buffer t2_emit writes, sized for part_bytes
    // (t2_emit reserves it too; the split path reserves before its exchange)
    bool t2_reserve(uint64_t part_bytes, std::string &err);
    // host_dst must be pinned (hipHostMalloc) memory
    bool t2_emit(const Plan &plan, uint64_t base, uint64_t part_bytes, uint8_t *host_dst, bool profile,
                 StageTimes &st, std::string &err);
    // stage times of the last encode from its events (profile mode; call
    // after the encode's last host wait)
    bool collect_profile(StageTimes &st, std::string &err);
    // this encode's hull segments: slope keys (descending) and inclusive byte sums
    bool segments(const Plan &plan, std::vector<uint64_t> &keys, std::vector<int64_t> &cum, std::string &err);
    hipStream_t get_stream() const { return stream; }
    int get_device() const { return device; }
    // the stream and the main buffers are on this context's device (a
    // tile-split member is checked before every split encode)
    bool check_residency(std::string &err);
    // host waits since the last call (stats: host_waits per encode)
    int take_waits() {
        const int w = waits;
        waits = 0;
        return w;
    }

  private:
    // debug: JP2HIP_DUMP_DIR=<dir> writes every stage's device buffer
    bool dump(const char *dir, const char *name, const DevBuf &b, size_t bytes, std::string &err);
    bool apply_thresholds(const Plan &plan, const int *halt, std::string &err);
    void select_launch(const Plan &plan, const int *halt, const RateState *init = nullptr, RateState *rs = nullptr);
    T2Args t2_args(const Plan &plan) const;
    // tier-2 sizing; with rs (device rate loop) k_t2_total also runs the
    // loop's step, leaving state + summary at out_rs (host-mapped)
    void t2_size_launch(const Plan &plan, bool with_kc, const int *halt, RateState *rs = nullptr,
                        RateState *out_rs = nullptr);
    bool host_wait(std::string &err);
    // The code-stream D2H on an SDMA engine (ROCr hsa_amd_memory_async_copy):
    // the HIP runtime moves a device -> pinned-host copy with a blit kernel
    // on the CUs (tests/tools/d2h_engine_probe.sh), which under load waits
    // for CU slots like any kernel.  The copy is queued behind `dma_dep`,
    // which the stream's last kernel (k_release_dma) sets to 0 after the
    // emission kernels, so it starts with no host round trip; the host
    // waits on `dma_done`.
    bool dma_init(std::string &err);
    bool dma_to_host(uint8_t *host_dst, const void *src, size_t bytes, std::string &err);
    hsa_signal_t dma_dep{0}, dma_done{0};
    volatile hsa_signal_value_t *dma_dep_val = nullptr;
    hsa_agent_t dma_gpu{0}, dma_cpu{0};
    int dma_engine = -1;  // SDMA engine of this context (-1: the runtime's choice)
    bool dma_ok = false, hsa_up = false;
    // host -> device copy through this context's pinned staging memory: a
    // pageable source goes through the runtime's shared staging buffer and
    // blocks until the stream reaches the copy, serialising the contexts
    bool h2d(void *dst, const void *src, size_t bytes, std::string &err);
    struct PinnedChunk {
        uint8_t *p;
        size_t cap;
    };
    std::vector<PinnedChunk> stg;
    size_t stg_used = 0;
    hipEvent_t stg_ev = nullptr;  // after the last staged copy
    static constexpr int kNumEvents = 12;
    int device = 0;
    int waits = 0;
    hipEvent_t sync_ev = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev[kNumEvents] = {};
    DevBuf coef, blocks, order, bp, sm, P, dref, dsig, t1out, rates, dists, npasses, lengths, weight,
        nhull, hpass, hkey, budget, nl, lrate, dstoff, packed, err, tcw, tch, strips, src, segcnt, segoff,
        est, hist, kcut, pmin, mqspan, stage, soff, lzwseg, untiled, inflnk, segkey, llbuf0, llbuf1, ordkey, segval, thr, items,
        slotoff, stream_buf, counts, dspp, dbgbuf, t1fill, dbgsel;
    // PCRD selection (k_hull / k_select): slope-bin histogram, ticket + list
    // fills, candidate lists
    DevBuf pcrd_hb, pcrd_hc, sel_ctl, sel_key, sel_size;
    // rate-control groups (Plan::grp_b0, then each group's first candidate
    // slot) and each group's tier-1 bytes (k_hull)
    DevBuf grptab, gtot;
    // device tier-2 (t2_device.hip)
    DevBuf hdist, rstate, t2ticket;
    RateState *h_rs = nullptr;      // host-mapped: rate state, then the T2Summary (k_rate_step)
    RateState *d_rs_out = nullptr;  // its device address
    DevBuf t2prec, t2tp, t2tt, t2lblock, t2incl, t2pklen, t2pkoff, t2tplen, t2tphdr, t2tpoff, t2blkdst, t2out, t2sum;
    int t2_nprec = 0, t2_ntp = 0;
    bool t2_wave = true;  // precincts of <= 64 blocks: k_t2_wave (layer assignment fused in)
    uint64_t front_gen = 0, t2_gen = 0;  // plan generation whose tables are resident
    T2Summary *h_sum = nullptr;
    int64_t *h_tot = nullptr;  // pinned [8]: t1 total, -, k_t1_mq span[2], unpack error, segment tail[2]
    bool profiled = false;
    int nseg = 0;  // hull segments at most: the bound sum(3 Mb - 2)
    uint8_t *h_packed = nullptr;
    size_t h_packed_cap = 0;
    std::vector<int64_t> h_hist;
    std::vector<uint64_t> strips_host;  // strip offsets last uploaded to `strips`
    const void *strips_dev = nullptr;
    size_t held = 0, mem_soft = SIZE_MAX, mem_hard = SIZE_MAX;
    static constexpr int kReclaimWaitMs = 30000;
    // hipMalloc, or hipErrorOutOfMemory past JP2HIP_TEST_DEVICE_BYTES held by
    // every context of the process together (tests: a small device)
    hipError_t device_alloc(void **p, size_t n);
    void device_free(DevBuf &b);
    // decision-stream pool: the first encode of a geometry reserves this
    // fraction of the every-plane bound; pool_hint = what the last
    // overflowing encode needed (+12.5 %)
    static constexpr double kPoolFracLossy = 0.3, kPoolFracLossless = 0.7;
    uint64_t pool_hint = 0;
    int pool_grows = 0;
    double pool_frac_test = -1.0;  // JP2HIP_TEST_POOL_FRAC (tests: force the grow path)
    std::vector<DevBuf *> bufs();
};

// Grows b to at least count T's (12.5 % headroom), within the hard limit.
template <typename T>
bool GpuEncoder::ensure(DevBuf &b, size_t count, std::string &err) {
    size_t bytes = count * sizeof(T);
    if (bytes == 0) bytes = 16;
    if (bytes > b.want) b.want = bytes;  // (also when the buffer is big enough already)
    if (b.bytes >= bytes) return true;
    const size_t alloc = bytes + bytes / 8;
    if (held - b.bytes + alloc > mem_hard) {
        err = "device memory limit: this image needs a " + std::to_string(alloc) + "-byte buffer, the context holds " +
              std::to_string(held) + " of its " + std::to_string(mem_hard) + " bytes";
        return false;
    }
    device_free(b);
    hipError_t e = device_alloc(&b.ptr, alloc);
    // out of device memory: other contexts of this device that are idle give
    // their buffers back (they reallocate at their next encode), and an
    // encode in progress elsewhere is waited for -- up to kReclaimWaitMs --
    // before this encode fails
    // (every round counts 5 ms against the wait, freed or not, so two
    // contexts taking memory from each other cannot loop for ever)
    for (int waited = 0; e == hipErrorOutOfMemory && reclaim && waited <= kReclaimWaitMs; waited += 5) {
        (void)hipGetLastError();
        if (!reclaim()) std::this_thread::sleep_for(std::chrono::milliseconds(5));
        e = device_alloc(&b.ptr, alloc);
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        b.ptr = nullptr;
        err = std::string("hipMalloc(") + std::to_string(alloc) + "): " + hipGetErrorString(e);
        return false;
    }
    b.bytes = alloc;
    held += alloc;
    return true;
}

}  // namespace jp2hip
