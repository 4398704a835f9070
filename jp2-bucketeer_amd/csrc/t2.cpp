// t2.cpp -- host side of code-stream assembly: the main header (SIZ, COD,
// QCD, COM), the tables that lay out packets and tile-parts for the device
// tier-2 (t2_device.hip), and the JP2 / JPX boxes around the code-stream
// (ISO/IEC 15444-1 Annex A, I; 15444-2 for 'jpx ').
//
// Structure produced for the Bucketeer recipe (KakaduConverter.java:38-44):
// RPCL packets, SOP before and EPH after every packet header, one tile-part
// per resolution (ORGtparts=R) each carrying a PLT marker (ORGgen_plt=yes),
// tile-parts in -flush_period stripe order, COM markers in Kakadu's layout.
// The layout is the one oracle/jp2_oracle.c writes (write_codestream).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "jp2hip_internal.h"

namespace jp2hip {

namespace {

inline void be16(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
inline void be32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

}  // namespace

// COM markers in Kakadu's layout (test.jpx): a
// version string, then "Kdu-Layer-Info", one fixed-width line per layer --
// log2 of the layer's slope threshold (squared error of samples normalised to
// unit range, summed over the image, per byte; -192.0 = every pass) and the
// code-stream bytes through that layer (oracle: write_main_header).
static constexpr char kComVersion[] = "jp2hip-v0.2.0";
static constexpr char kLayerHdr[] = "Kdu-Layer-Info: log_2{Delta-D(squared-error)/Delta-L(bytes)}, L(bytes)\n";

static double layer_log_slope(uint64_t K, int bits) {
    if (K == 0) return -192.0;
    if (K >= 0x7FF0000000000000ull) return 192.0;  // nothing included
    double s;
    std::memcpy(&s, &K, 8);
    const double v = std::log2(s) - 2.0 * bits;
    return v < -192.0 ? -192.0 : (v > 192.0 ? 192.0 : v);
}

void main_header(const Plan &P, std::vector<uint8_t> &v, const uint64_t *K, const int64_t *layer_end) {
    const jp2hip_recipe &rc = P.rc;
    const int L = rc.levels, nc = P.nc;
    v.clear();
    auto u8 = [&](int x) { v.push_back((uint8_t)x); };
    auto u16 = [&](int x) { u8(x >> 8); u8(x); };
    auto u32 = [&](uint32_t x) { u16((int)(x >> 16)); u16((int)(x & 0xFFFF)); };
    auto raw = [&](const char *p, size_t n) { v.insert(v.end(), p, p + n); };
    u16(0xFF4F);
    u16(0xFF51);  // SIZ
    u16(38 + 3 * nc);
    u16(0);
    u32((uint32_t)P.w); u32((uint32_t)P.h);
    u32(0); u32(0);
    u32((uint32_t)rc.tile_w); u32((uint32_t)rc.tile_h);
    u32(0); u32(0);
    u16(nc);
    for (int c = 0; c < nc; c++) { u8(P.bits - 1); u8(1); u8(1); }
    u16(0xFF52);  // COD
    u16(12 + L + 1);
    u8(0x01 | (rc.sop ? 2 : 0) | (rc.eph ? 4 : 0));
    u8(rc.progression);
    u16(rc.layers);
    u8((rc.mct && nc >= 3) ? 1 : 0);
    u8(L);
    u8(rc.cblk_w_log2 - 2);
    u8(rc.cblk_h_log2 - 2);
    u8(0);
    u8(rc.reversible ? 1 : 0);
    for (int r = 0; r <= L; r++) u8((prec_log2(rc, r, true) << 4) | prec_log2(rc, r, false));
    u16(0xFF5C);  // QCD
    const int nbands = 3 * L + 1;
    u16(3 + (rc.reversible ? nbands : 2 * nbands));
    u8((rc.guard_bits << 5) | (rc.reversible ? 0 : 2));
    for (int i = 0; i < nbands; i++) {
        const int d = (i == 0) ? L : L - (i - 1) / 3;
        const int band = (i == 0) ? 0 : 1 + (i - 1) % 3;
        const BandQuant q = band_quant(rc, P.bits, d, band);
        if (rc.reversible) u8(q.eps << 3);
        else u16((q.eps << 11) | q.mu);
    }
    if (rc.comment) {
        const size_t nv = sizeof kComVersion - 1, nh = sizeof kLayerHdr - 1;
        u16(0xFF64);
        u16(4 + (int)nv);
        u16(1);  // Rcom: Latin-1 text
        raw(kComVersion, nv);
        u16(0xFF64);
        u16(4 + (int)nh + 17 * rc.layers);
        u16(1);
        raw(kLayerHdr, nh);
        for (int l = 0; l < rc.layers; l++) {
            char line[64];
            const int n = std::snprintf(line, sizeof line, "%6.1f, %8.1e\n", K ? layer_log_slope(K[l], P.bits) : 0.0,
                                        layer_end ? (double)layer_end[l] : 0.0);
            if (n != 17) {  // never for |slope| <= 192 and < 1e100 bytes
                std::memset(line, ' ', 16);
                line[16] = '\n';
            }
            raw(line, 17);
        }
    }
}

static int64_t tree_nodes(int w, int h) {
    int64_t n = 0;
    for (;;) {
        n += (int64_t)w * h;
        if (w == 1 && h == 1) return n;
        w = (w + 1) / 2;
        h = (h + 1) / 2;
    }
}

void t2_tables(const Plan &P, int tile0, int tile1, int block0, T2Tables &T) {
    const jp2hip_recipe &rc = P.rc;
    const int Lv = rc.levels, L = rc.layers;
    T.prec.clear();
    T.tp.clear();
    T.tt_nodes = 0;
    T.max_prec_blocks = 0;
    // tile-parts per tile, in tile order first
    std::vector<std::vector<TpDesc>> per_tile((size_t)std::max(0, tile1 - tile0));
    for (int t = tile0; t < tile1; t++) {
        const Tile &Tl = P.tiles[t];
        int nsop = 0;
        std::vector<TpDesc> &tps = per_tile[(size_t)(t - tile0)];
        for (int r = 0; r <= Lv; r++) {
            const Resolution &R0 = Tl.tc[0].res[r];
            if (R0.npx * R0.npy == 0) continue;
            if (rc.tparts_r || tps.empty()) tps.push_back(TpDesc{t, (int32_t)tps.size(), 0, (int32_t)T.prec.size(), 0});
            TpDesc &tp = tps.back();
            for (int py = 0; py < R0.npy; py++)
                for (int px = 0; px < R0.npx; px++)
                    for (int c = 0; c < P.nc; c++) {
                        const Precinct &pr = Tl.tc[c].res[r].prec[(size_t)py * R0.npx + px];
                        PrecDesc d;
                        std::memset(&d, 0, sizeof d);
                        d.nb = (uint8_t)pr.nb;
                        d.tt_off = (int32_t)T.tt_nodes;
                        d.nsop0 = nsop;
                        int blocks = 0;
                        for (int bi = 0; bi < pr.nb; bi++) {
                            const PrecBand &pb = pr.pb[bi];
                            d.first[bi] = pb.first - block0;
                            d.ncw[bi] = (uint16_t)pb.ncw;
                            d.nch[bi] = (uint16_t)pb.nch;
                            blocks += pb.ncw * pb.nch;
                            if (pb.ncw && pb.nch) T.tt_nodes += 2 * tree_nodes(pb.ncw, pb.nch);
                        }
                        T.max_prec_blocks = std::max(T.max_prec_blocks, blocks);
                        T.prec.push_back(d);
                        tp.nprec++;
                        nsop += L;
                    }
        }
        for (TpDesc &tp : tps) tp.tnsot = (&tp == &tps.back()) ? (int32_t)tps.size() : 0;
    }
    // code-stream order: per -flush_period stripe, resolution 0 of every tile,
    // then resolution 1, ... (test.jpx; t2_emit_part does the same on the host)
    const std::vector<int> ends = flush_stripe_ends(P.nty, rc.tile_h, P.h, rc.flush_period);
    int ty0 = 0;
    for (int e : ends) {
        const int a = std::max(tile0, ty0 * P.ntx), b = std::min(tile1, e * P.ntx);
        for (int k = 0; k <= Lv; k++)
            for (int t = a; t < b; t++) {
                const std::vector<TpDesc> &tps = per_tile[(size_t)(t - tile0)];
                if (k < (int)tps.size()) T.tp.push_back(tps[(size_t)k]);
            }
        ty0 = e;
    }
}

size_t file_header_bytes(const Plan &P) {
    if (P.rc.format == JP2HIP_FORMAT_J2K) return 0;
    const int nc = P.nc;
    const bool cdef = (nc == 4 || nc == 2);
    size_t n = 12;                                                                    // signature
    n += (P.rc.format == JP2HIP_FORMAT_JPX) ? (8 + 4 + 4 + 12) + (8 + 10) : (8 + 4 + 4 + 4);  // ftyp (+rreq)
    n += 8 + (8 + 14) + (8 + 7) + (cdef ? (size_t)(8 + 2 + 6 * nc) : 0);             // jp2h
    return n + 8;                                                                     // jp2c box header
}

void write_file_header(const Plan &P, uint64_t cs_bytes, uint8_t *dst) {
    if (P.rc.format == JP2HIP_FORMAT_J2K) return;
    uint8_t *p = dst;
    auto raw = [&](const void *s, size_t n) { std::memcpy(p, s, n); p += n; };
    auto u8 = [&](int x) { *p++ = (uint8_t)x; };
    auto u16 = [&](int x) { be16(p, (uint32_t)x); p += 2; };
    auto u32 = [&](uint32_t x) { be32(p, x); p += 4; };
    auto box = [&](uint32_t len, const char *type) { u32(len); raw(type, 4); };
    static const uint8_t sig[12] = {0, 0, 0, 12, 'j', 'P', ' ', ' ', 0x0D, 0x0A, 0x87, 0x0A};
    raw(sig, 12);
    const int nc = P.nc;
    if (P.rc.format == JP2HIP_FORMAT_JPX) {
        box(8 + 4 + 4 + 12, "ftyp");
        raw("jpx ", 4); u32(0);
        raw("jpx ", 4); raw("jp2 ", 4); raw("jpxb", 4);
        box(8 + 10, "rreq");  // reader requirements: feature 5 (JP2-compatible)
        u8(1); u8(0x80); u8(0x80);
        u16(1); u16(5); u8(0x80);
        u16(0);
    } else {
        box(8 + 4 + 4 + 4, "ftyp");
        raw("jp2 ", 4); u32(0); raw("jp2 ", 4);
    }
    const bool cdef = (nc == 4 || nc == 2);
    const uint32_t ihdr = 8 + 14, colr = 8 + 7, cdefl = cdef ? (uint32_t)(8 + 2 + 6 * nc) : 0;
    box(8 + ihdr + colr + cdefl, "jp2h");
    box(ihdr, "ihdr");
    u32((uint32_t)P.h); u32((uint32_t)P.w);
    u16(nc); u8(P.bits - 1); u8(7); u8(0); u8(0);
    box(colr, "colr");
    u8(1); u8(0); u8(0);
    u32(nc >= 3 ? 16 : 17);  // sRGB / greyscale
    if (cdef) {
        box(cdefl, "cdef");
        u16(nc);
        for (int c = 0; c < nc; c++) {
            const bool alpha = (c == nc - 1);
            u16(c); u16(alpha ? 1 : 0); u16(alpha ? 0 : c + 1);
        }
    }
    // a code-stream past 4 GiB: length 0 = "to the end of the file" (last box)
    box(8 + cs_bytes > 0xFFFFFFFFull ? 0u : (uint32_t)(8 + cs_bytes), "jp2c");
}

}  // namespace jp2hip
