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

// One code-block, as the kernels see it (uploaded as-is).
struct BlockDesc {
    int32_t tc;         // tile-component plane index
    int16_t x0, y0;     // top-left inside the tile-component plane (Mallat layout)
    int16_t w, h;       // <= 64
    int8_t band;        // 0 LL, 1 HL, 2 LH, 3 HH
    int8_t Mb;          // magnitude bit-planes of the band
    int8_t pad0, pad1;
    float inv_delta;    // irreversible quantiser reciprocal
    uint32_t pad2;
    uint64_t bp_off;    // bit-plane storage offset, in uint64 words
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
};

bool build_plan(Plan &plan, const jp2hip_recipe &rc, int w, int h, int nc, int bits,
                std::string &err);

int prec_log2(const jp2hip_recipe &rc, int r, bool vertical);

// Tile rows [tr0, tr1) of rank `rank` out of `world` (contiguous bands).
void split_tile_rows(int nty, int rank, int world, int &tr0, int &tr1);
// The device part of `full` for tile rows [tr0, tr1): same blocks, offsets
// rebased to the band (tier-2 keeps using `full` and global block indices).
void make_subplan(const Plan &full, int tr0, int tr1, Plan &sub);

// Tier-2 inputs: the layer table chosen by PCRD.  `data` holds the included
// bytes of every block back to back at `data_off[b]` (needed by t2_emit only).
struct T2Input {
    const Plan *plan;
    const uint8_t *P;           // coded bit-planes per block
    const uint8_t *nl;          // [block][layers] cumulative passes per layer
    const int32_t *lrate;       // [block][layers] cumulative bytes per layer
    const uint8_t *data;
    const uint64_t *data_off;
    int threads;
    int tile0 = 0, tile1 = -1;  // tiles to code ([tile0, tile1); -1: all)
};

struct TagNode {
    int32_t parent, value, low;
    int32_t known;
};

// Per-tile result of the header pass (reused across calls; no reallocation
// once warm).
struct T2Tile {
    std::vector<uint8_t> hdr;        // coded packet headers, back to back
    std::vector<uint32_t> hdr_end;   // per packet: end offset in hdr
    std::vector<uint32_t> pk_len;    // per packet: SOP + header + EPH + body bytes
    std::vector<uint32_t> pk_cend;   // per packet: end index (in triples) into contrib
    std::vector<uint32_t> contrib;   // (block, first byte, end byte) of each body piece
    std::vector<int32_t> tp_npk;     // packets per tile-part
    std::vector<uint64_t> tp_bytes;  // Psot per tile-part
    std::vector<int32_t> tree;       // tag-tree roots per (c, r, precinct, band)
    uint64_t bytes = 0;
};
struct T2Worker {
    std::vector<int32_t> lblock;     // indexed by block (a tile touches only its own)
    std::vector<int8_t> incl;
    std::vector<TagNode> nodes;
};
struct T2State {
    std::vector<uint8_t> main;       // main header (SOC .. COM)
    std::vector<T2Tile> tiles;
    std::vector<T2Worker> workers;
    int64_t total = 0;               // code-stream bytes, SOC .. EOC
};

// Header pass: codes every packet header of tiles [in.tile0, in.tile1),
// returns main header + those tiles + EOC (the code-stream size when the
// range is every tile).
int64_t t2_headers(const T2Input &in, T2State &st);
// Writes the code-stream described by the last t2_headers() into dst
// (st.total bytes); in.data / in.data_off must be set.
void t2_emit(const T2Input &in, const T2State &st, uint8_t *dst);
// Tile-split: bytes of tiles [in.tile0, in.tile1) (+ main header / EOC when
// asked) as written by t2_emit_part.
uint64_t t2_part_bytes(const T2Input &in, const T2State &st, bool with_main, bool with_eoc);
void t2_emit_part(const T2Input &in, const T2State &st, uint8_t *dst, bool with_main, bool with_eoc);

// JP2 / JPX boxes in front of the code-stream (0 bytes for raw J2K).
size_t file_header_bytes(const Plan &plan);
void write_file_header(const Plan &plan, uint64_t cs_bytes, uint8_t *dst);

}  // namespace jp2hip
