// jp2hip_internal.h -- host-side model of one encode (geometry, quantiser,
// code-block table) shared by the HIP launch code (kernels.hip), tier-2
// (t2.cpp) and the C ABI (api.cpp).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "jp2hip.h"

namespace jp2hip {

constexpr int kMaxPasses = 96;    // 3*32-2 rounded up; per-block pass table stride
// slope prediction (kernels.hip k_plane_*, oracle predict_and_code): 1/8-octave
// bins of the double slope's bit pattern covering 2^-64 .. 2^64, and the
// margin (bins) kept below the predicted rate-target bin
constexpr int kSlopeBins = 1024;
constexpr int kSlopeBinBase = (1023 - 64) << 3;
constexpr int kSkipMargin = 12;
// PCRD threshold selection (kernels.hip k_hull / k_select): hull segment bytes
// histogrammed over 1/32-octave bins of the slope key (bits 47..62 of the
// IEEE double, 2^-64 .. 2^64, clamped at both ends); the exact threshold is
// then resolved inside the one bin where a layer's budget falls
constexpr int kPcrdBins = 4096;
constexpr int kPcrdBinBase = (1023 - 64) << 5;
constexpr int kMaxLayers = 32;
constexpr int kMaxLevels = 12;

// Per-band quantiser (Annex E).  For the reversible path eps follows the
// 5/3 BIBO-gain rule that reproduces test.jpx's QCD.
struct BandQuant {
    int eps = 0, mu = 0, Mb = 0;
    float inv_delta = 1.0f;
    double wnorm = 1.0;  // Delta^2 * synthesis energy gain
};

BandQuant band_quant(const jp2hip_recipe &rc, int bits, int level, int band);

// Every band's deadzone quantiser as the DWT's final writes apply it
// (dwt.hip): the coefficient plane holds quantisation indices in
// sign-magnitude, 16-bit when every band has at most 15 magnitude bit-planes
// (8-bit sources), else 32-bit; k_quant reads them.  Entry [d][b] = level d,
// band b (the LL band only at d = levels; levels = 0: [0][0]).
struct QuantTab {
    float inv[kMaxLevels + 1][4];    // 1 / Delta (1 for the reversible path)
    uint32_t lim[kMaxLevels + 1][4]; // 2^Mb - 1: the largest index
    int q16;
};
QuantTab quant_tab(const jp2hip_recipe &rc, int bits);

// One code-block, as the kernels see it (uploaded as-is).
// device error word bit: the decision-stream pool was too small for the
// coded planes (emit_t1_items); the host grows it and encodes again
constexpr int kErrSlotPool = 8;

struct BlockDesc {
    int32_t tc;         // tile-component plane index
    int16_t x0, y0;     // top-left inside the tile-component plane (Mallat layout)
    int16_t w, h;       // <= 64
    int8_t band;        // 0 LL, 1 HL, 2 LH, 3 HH
    int8_t Mb;          // magnitude bit-planes of the band
    int8_t pad0, pad1;
    float inv_delta;    // irreversible quantiser reciprocal
    uint32_t pad2;
    uint64_t bp_off;    // bit-plane storage offset, in uint64 words: (Mb+1)*64 column masks
                        // (kernels.hip k_quant)
    uint64_t sm_off;    // sign-magnitude storage offset, in int32 words
    uint64_t out_off;   // tier-1 output offset, bytes
    uint32_t out_cap;   // tier-1 output capacity, bytes
    uint32_t pad3;
};
static_assert(sizeof(BlockDesc) == 56, "BlockDesc layout");

struct PrecBand {
    int ncw = 0, nch = 0;
    int first = 0;  // index of the first block (raster order, contiguous)
};
struct Precinct {
    PrecBand pb[3];
    int nb = 0;
};
struct Resolution {
    int npx = 0, npy = 0;
    std::vector<Precinct> prec;
};
struct TileComp {
    Resolution res[kMaxLevels + 1];
};
struct Tile {
    int tx0, ty0, tx1, ty1;
    std::vector<TileComp> tc;
};

struct Plan {
    jp2hip_recipe rc;
    int w = 0, h = 0, nc = 0, bits = 0;
    int ntx = 0, nty = 0, ntc = 0;
    int plane_w = 0, plane_h = 0;           // tile-component plane stride / rows
    std::vector<Tile> tiles;
    std::vector<BlockDesc> blocks;
    std::vector<double> weight;             // PCRD weight per block
    std::vector<int32_t> t1_order;          // lane -> block mapping for tier-1
    std::vector<int32_t> tc_w, tc_h;        // tile-component sizes
    uint64_t bp_words = 0, sm_words = 0, out_bytes = 0;
    int64_t npackets = 0, ntileparts = 0;
    double compw[4] = {1, 1, 1, 1};
    // tile-split band (make_subplan): the device part covers tiles
    // [tile0, tile0 + ntc/nc) = image rows [row0, row0 + band_h); its blocks
    // are the full plan's blocks [block0, block0 + blocks.size())
    int row0 = 0, band_h = 0, tile0 = 0, block0 = 0;
    // first block of each tile of this plan (tiles in raster order; blocks
    // are emitted tile by tile), ntiles + 1 entries
    std::vector<int32_t> tile_b0;
    // rate-control groups: block ranges [grp_b0[g], grp_b0[g + 1]) whose
    // layer thresholds are chosen together.  Lossless ("-rate -"): one group
    // per -flush_period stripe (each stripe's layers from its own tier-1
    // bytes, oracle lossless_budget); rate-driven: the whole image, one group
    std::vector<int32_t> grp_b0;
    int ngroups() const { return (int)grp_b0.size() - 1; }
    // identity of this plan's contents (build_plan / make_subplan): a device
    // context that already holds the tables of generation `gen` skips
    // uploading them again
    uint64_t gen = 0;
};

bool build_plan(Plan &plan, const jp2hip_recipe &rc, int w, int h, int nc, int bits,
                std::string &err);

int prec_log2(const jp2hip_recipe &rc, int r, bool vertical);

// Lossless layer l of NL: the fraction (1/65536 units) of its stripe's
// tier-1 bytes the layer's threshold fits (oracle/jp2_oracle.c
// lossless_layer_frac, fitted to test.jpx's Kdu-Layer-Info); the last layer
// takes every pass (65536).
int32_t lossless_layer_frac(int l, int NL);

// Tile rows grouped the way "-flush_period P" flushes them
// (KakaduConverter.java:40; oracle flush_stripes): a stripe ends once the rows
// pushed reach the next multiple of P, and at the last tile row.  Returns one
// past the last tile row of each stripe.  P <= 0: one stripe per tile row.
std::vector<int> flush_stripe_ends(int nty, int tile_h, int h, int period);
// Tile rows [tr0, tr1) of rank `rank` out of `world`: contiguous runs of
// whole flush stripes, so each rank's tile-parts are contiguous in the file.
void split_tile_rows(int nty, int tile_h, int h, int period, int rank, int world, int &tr0, int &tr1);
// The device part of `full` for tile rows [tr0, tr1): same blocks, offsets
// rebased to the band (tier-2 keeps using `full` and global block indices).
void make_subplan(const Plan &full, int tr0, int tr1, Plan &sub);

// --------------------------------------------------------------------------
// Device tier-2 (t2_device.hip).  The host lays out, once per encode, the precincts
// of the tiles being coded in packet order (tile, resolution, py, px,
// component; RPCL) and the tile-parts in code-stream order (-flush_period
// stripes); the kernels code every packet header, size the tile-parts and
// write the code-stream in HBM.  Packet k of precinct p is packet p * L + k.
// --------------------------------------------------------------------------
struct PrecDesc {
    int32_t first[3];        // first code-block (encode-local index) of each precinct-band
    uint16_t ncw[3], nch[3]; // code-block grid of each precinct-band
    int32_t tt_off;          // tag-tree node scratch: (inclusion, zero bit-planes) per band
    int32_t nsop0;           // SOP sequence number of the precinct's first packet in its tile
    uint8_t nb, pad0, pad1, pad2;
};
static_assert(sizeof(PrecDesc) == 36, "PrecDesc layout");
struct TpDesc {
    int32_t tile, tpsot, tnsot;  // SOT fields (Isot, TPsot, TNsot)
    int32_t prec0, nprec;        // its precincts in the PrecDesc table
};
struct T2Tables {
    std::vector<PrecDesc> prec;
    std::vector<TpDesc> tp;   // code-stream order
    int64_t tt_nodes = 0;
    int max_prec_blocks = 0;  // code-blocks of the largest precinct
};
// Tables for tiles [tile0, tile1) of `P` (blocks rebased by -block0: a
// tile-split rank's blocks are its sub-plan's).
void t2_tables(const Plan &P, int tile0, int tile1, int block0, T2Tables &T);
// What the host reads back after a tier-2 sizing pass (one D2H per pass).
struct T2Summary {
    int64_t part_bytes;               // tile-parts of the tiles coded (SOT .. last packet)
    int64_t tp_hdr_bytes;             // SOT + PLT + SOD of those tile-parts
    int64_t layer_bytes[kMaxLayers];  // packet bytes per layer
    uint64_t kc[kMaxLayers];          // Kdu-Layer-Info slope keys (select() only)
    int64_t t1_bytes, coded_passes;   // tier-1 totals (every coded pass)
    int64_t decisions;                // MQ-coded decisions
    int32_t skipped, err;             // slope prediction skipped planes; tier-1 overflow
    int64_t stream_need;              // decision-stream pool bytes the coded planes took
};
// Rate control of a rate-driven encode, run on the device (kernels.hip
// k_rate_step; the oracle's loop in oracle_encode): iteration `it` selects
// with `budget`, sizes the code-stream, stops when it fits `target` (or after
// 8 iterations), else lowers the budget.  `halt` stops the remaining
// iterations' kernels; `safety` = slope prediction's safety net fired
// (planes were skipped yet every coded byte fits: the host re-runs the front
// with every plane coded).
struct RateState {
    int64_t budget, target, fixed, skip_target, cs_bytes;
    int32_t it, halt, safety, iters;
};
// Main header (SOC .. COM) for the Kdu-Layer-Info values (nullptr: zeros;
// the length does not depend on them).
void main_header(const Plan &P, std::vector<uint8_t> &v, const uint64_t *K, const int64_t *layer_end);

// JP2 / JPX boxes in front of the code-stream (0 bytes for raw J2K).
size_t file_header_bytes(const Plan &plan);
void write_file_header(const Plan &plan, uint64_t cs_bytes, uint8_t *dst);

}  // namespace jp2hip
