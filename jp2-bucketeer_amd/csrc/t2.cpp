// t2.cpp -- tier-2 coding and code-stream / file assembly (ISO/IEC 15444-1
// Annex A, B.9-B.10, Annex I), run on host threads, one tile per task.
//
// Structure produced for the Bucketeer recipe (KakaduConverter.java:38-44):
// RPCL packets, SOP before and EPH after every packet header, one tile-part
// per resolution (ORGtparts=R) each carrying a PLT marker (ORGgen_plt=yes).
//
// Two phases, so the rate-control loop never touches code-block bytes:
//   t2_headers()  codes every packet header into per-tile arenas and records
//                 packet / tile-part lengths -> exact code-stream size;
//   t2_emit()     writes main header, SOT/PLT/SOD, SOP, the cached headers,
//                 EPH and the code-block bytes straight into the output.
// The layout is the one oracle/jp2_oracle.c writes (t2_tile / t2_packet).
#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

#include "jp2hip_internal.h"

namespace jp2hip {

namespace {

// Packet-header bit writer, B.10.1: MSB first; a byte after 0xFF carries 7 bits.
struct Bits {
    std::vector<uint8_t> &v;
    uint64_t acc = 0;
    int n = 0, cap = 8;
    explicit Bits(std::vector<uint8_t> &o) : v(o) {}
    void put(uint32_t val, int nb) {  // nb <= 32
        acc = (acc << nb) | val;
        n += nb;
        while (n >= cap) {
            n -= cap;
            const uint32_t byte = (uint32_t)(acc >> n) & ((1u << cap) - 1u);
            v.push_back((uint8_t)byte);
            cap = (byte == 0xFF) ? 7 : 8;
        }
    }
    void bit(int b) { put((uint32_t)(b & 1), 1); }
    void flush() {
        if (n) {
            const uint32_t byte = (uint32_t)(acc << (cap - n)) & ((1u << cap) - 1u);
            v.push_back((uint8_t)byte);
            cap = 8;
            n = 0;
        } else if (cap == 7) {  // a header may not end in 0xFF
            v.push_back(0);
            cap = 8;
        }
        acc = 0;
    }
};

// Tag trees (B.10.2): leaves in raster order, parents by 2x2 grouping; all
// trees of a tile share one node pool.
struct Trees {
    std::vector<TagNode> &nd;
    int build(int w, int h) {
        int lw[40], lh[40], nl = 0, tot = 0, cw = w, ch = h;
        for (;;) {
            lw[nl] = cw; lh[nl] = ch; tot += cw * ch; nl++;
            if (cw == 1 && ch == 1) break;
            cw = (cw + 1) / 2; ch = (ch + 1) / 2;
        }
        const int base0 = (int)nd.size();
        nd.resize(nd.size() + (size_t)tot, TagNode{-1, 1 << 20, 0, 0});
        int base = base0;
        for (int l = 0; l < nl; l++) {
            const int pbase = base + lw[l] * lh[l];
            for (int y = 0; y < lh[l]; y++)
                for (int x = 0; x < lw[l]; x++)
                    nd[(size_t)base + y * lw[l] + x].parent =
                        (l + 1 < nl) ? pbase + (y / 2) * lw[l + 1] + x / 2 : -1;
            base = pbase;
        }
        return base0;
    }
    void set(int leaf, int v) {
        for (int i = leaf; i >= 0 && nd[i].value > v; i = nd[i].parent) nd[i].value = v;
    }
    void encode(Bits &w, int leaf, int threshold) {
        int stk[40], ns = 0;
        for (int i = leaf; i >= 0; i = nd[i].parent) stk[ns++] = i;
        int low = 0;
        for (int k = ns - 1; k >= 0; k--) {
            TagNode &n = nd[stk[k]];
            if (low > n.low) n.low = low;
            else low = n.low;
            while (low < threshold) {
                if (low >= n.value) {
                    if (!n.known) { w.bit(1); n.known = 1; }
                    break;
                }
                w.bit(0);
                low++;
            }
            n.low = low;
        }
    }
};

inline int floor_log2(int v) { return 31 - __builtin_clz((unsigned)v); }

inline void be16(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
inline void be32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

inline int varint_len(uint32_t L) {
    int k = 1;
    while (L >>= 7) k++;
    return k;
}

// PLT segments (A.7.3) for a run of packet lengths: bytes, or write them.
size_t plt_bytes(const uint32_t *lens, int n) {
    size_t total = 0, seg = 0;
    for (int i = 0; i < n; i++) {
        const size_t k = (size_t)varint_len(lens[i]);
        if (i == 0 || seg + k > 65532) {
            if (i) total += 5 + seg;
            seg = 0;
        }
        seg += k;
    }
    return n ? total + 5 + seg : 0;
}

uint8_t *write_plt(uint8_t *o, const uint32_t *lens, int n) {
    int i = 0, z = 0;
    while (i < n) {
        uint8_t *hdr = o;
        o += 5;
        size_t seg = 0;
        while (i < n) {
            const uint32_t L = lens[i];
            const int k = varint_len(L);
            if (seg + (size_t)k > 65532) break;
            for (int j = k - 1; j >= 0; j--) *o++ = (uint8_t)(((L >> (7 * j)) & 0x7F) | (j ? 0x80 : 0));
            seg += (size_t)k;
            i++;
        }
        be16(hdr, 0xFF58);
        be16(hdr + 2, (uint32_t)(3 + seg));
        hdr[4] = (uint8_t)z++;
    }
    return o;
}

// Header pass for one tile (oracle: t2_tile).
void tile_headers(const T2Input &in, int t, T2Tile &tt, T2Worker &wk) {
    const Plan &P = *in.plan;
    const jp2hip_recipe &rc = P.rc;
    const Tile &T = P.tiles[t];
    const int Lv = rc.levels, L = rc.layers;
    const uint8_t *NL = in.nl;
    const int32_t *LR = in.lrate;
    tt.hdr.clear();
    tt.hdr_end.clear();
    tt.pk_len.clear();
    tt.pk_cend.clear();
    tt.contrib.clear();
    tt.tp_npk.clear();
    tt.tp_bytes.clear();
    tt.tree.clear();
    wk.nodes.clear();
    Trees trees{wk.nodes};
    // inclusion / zero-bit-plane trees of every precinct-band: [c][r][p] x 3 x 2
    std::vector<int> cr_base((size_t)P.nc * (Lv + 1));
    int idx = 0;
    for (int c = 0; c < P.nc; c++)
        for (int r = 0; r <= Lv; r++) {
            cr_base[(size_t)c * (Lv + 1) + r] = idx;
            const Resolution &R = T.tc[c].res[r];
            idx += R.npx * R.npy;
            for (int p = 0; p < R.npx * R.npy; p++) {
                const Precinct &pr = R.prec[p];
                for (int bi = 0; bi < 3; bi++) {
                    if (bi >= pr.nb || !pr.pb[bi].ncw || !pr.pb[bi].nch) {
                        tt.tree.push_back(-1);
                        tt.tree.push_back(-1);
                        continue;
                    }
                    const PrecBand &pb = pr.pb[bi];
                    const int ib = trees.build(pb.ncw, pb.nch);
                    const int zb = trees.build(pb.ncw, pb.nch);
                    tt.tree.push_back(ib);
                    tt.tree.push_back(zb);
                    for (int k = 0; k < pb.ncw * pb.nch; k++) {
                        const int b = pb.first + k;
                        wk.lblock[b] = 3;
                        wk.incl[b] = -1;
                        int first = L;
                        for (int l = 0; l < L; l++)
                            if (NL[(size_t)b * L + l] > 0) { first = l; break; }
                        trees.set(ib + k, first);
                        trees.set(zb + k, P.blocks[b].Mb - in.P[b]);
                    }
                }
            }
        }
    const uint32_t fixed = (rc.sop ? 6u : 0u) + (rc.eph ? 2u : 0u);
    int merged = 0;  // packets of the single tile-part when !tparts_r
    for (int r = 0; r <= Lv; r++) {
        const Resolution &R0 = T.tc[0].res[r];
        if (R0.npx * R0.npy == 0) continue;
        const size_t pk0 = tt.pk_len.size();
        for (int py = 0; py < R0.npy; py++)
            for (int px = 0; px < R0.npx; px++)
                for (int c = 0; c < P.nc; c++) {
                    const int pi = py * R0.npx + px;
                    const Precinct &pr = T.tc[c].res[r].prec[pi];
                    const int *tr = &tt.tree[(size_t)(cr_base[(size_t)c * (Lv + 1) + r] + pi) * 6];
                    for (int l = 0; l < L; l++) {
                        bool nonempty = false;
                        for (int bi = 0; bi < pr.nb && !nonempty; bi++) {
                            const PrecBand &pb = pr.pb[bi];
                            for (int k = 0; k < pb.ncw * pb.nch; k++) {
                                const uint8_t *nb = NL + (size_t)(pb.first + k) * L;
                                if (nb[l] > (l ? nb[l - 1] : 0)) { nonempty = true; break; }
                            }
                        }
                        const size_t h0 = tt.hdr.size();
                        uint32_t body = 0;
                        Bits w(tt.hdr);
                        w.bit(nonempty ? 1 : 0);
                        if (nonempty) {
                            for (int bi = 0; bi < pr.nb; bi++) {
                                const PrecBand &pb = pr.pb[bi];
                                for (int k = 0; k < pb.ncw * pb.nch; k++) {
                                    const int b = pb.first + k;
                                    const uint8_t *nb = NL + (size_t)b * L;
                                    const int n = nb[l] - (l ? nb[l - 1] : 0);
                                    if (wk.incl[b] < 0) trees.encode(w, tr[2 * bi] + k, l + 1);
                                    else w.bit(n > 0 ? 1 : 0);
                                    if (n <= 0) continue;
                                    if (wk.incl[b] < 0) {
                                        trees.encode(w, tr[2 * bi + 1] + k, 1 << 20);
                                        wk.incl[b] = (int8_t)l;
                                    }
                                    // number of passes, Table B.4
                                    if (n == 1) w.bit(0);
                                    else if (n == 2) w.put(2u, 2);
                                    else if (n <= 5) w.put((3u << 2) | (uint32_t)(n - 3), 4);
                                    else if (n <= 36) w.put((15u << 5) | (uint32_t)(n - 6), 9);
                                    else w.put((511u << 7) | (uint32_t)(n - 37), 16);
                                    const int32_t *lr = LR + (size_t)b * L;
                                    const int r0 = l ? lr[l - 1] : 0;
                                    const int len = lr[l] - r0;
                                    int nbits = wk.lblock[b] + floor_log2(n);
                                    while (len >= (1 << nbits)) { w.bit(1); wk.lblock[b]++; nbits++; }
                                    w.bit(0);
                                    w.put((uint32_t)len, nbits);
                                    body += (uint32_t)len;
                                    tt.contrib.push_back((uint32_t)b);
                                    tt.contrib.push_back((uint32_t)r0);
                                    tt.contrib.push_back((uint32_t)lr[l]);
                                }
                            }
                        }
                        w.flush();
                        tt.hdr_end.push_back((uint32_t)tt.hdr.size());
                        tt.pk_cend.push_back((uint32_t)(tt.contrib.size() / 3));
                        tt.pk_len.push_back(fixed + (uint32_t)(tt.hdr.size() - h0) + body);
                    }
                }
        const int npk = (int)(tt.pk_len.size() - pk0);
        if (rc.tparts_r) tt.tp_npk.push_back(npk);
        else merged += npk;
    }
    if (!rc.tparts_r && merged) tt.tp_npk.push_back(merged);
    // Psot of every tile-part: SOT(12) + PLT + SOD(2) + packets
    uint64_t total = 0;
    size_t pk = 0;
    for (int npk : tt.tp_npk) {
        uint64_t bytes = 14 + (rc.plt ? plt_bytes(tt.pk_len.data() + pk, npk) : 0);
        for (int i = 0; i < npk; i++) bytes += tt.pk_len[pk + i];
        tt.tp_bytes.push_back(bytes);
        total += bytes;
        pk += (size_t)npk;
    }
    tt.bytes = total;
}

// Code-stream bytes of one tile (oracle: t2_tile's output loop).
void tile_emit(const T2Input &in, int t, const T2Tile &tt, uint8_t *p) {
    const jp2hip_recipe &rc = in.plan->rc;
    const int ntp = (int)tt.tp_npk.size();
    size_t pk = 0;
    int nsop = 0;
    for (int tp = 0; tp < ntp; tp++) {
        be16(p, 0xFF90);
        be16(p + 2, 10);
        be16(p + 4, (uint32_t)t);
        be32(p + 6, (uint32_t)tt.tp_bytes[tp]);
        p[10] = (uint8_t)tp;
        p[11] = (uint8_t)ntp;
        p += 12;
        const int npk = tt.tp_npk[tp];
        if (rc.plt) p = write_plt(p, tt.pk_len.data() + pk, npk);
        be16(p, 0xFF93);
        p += 2;
        for (int i = 0; i < npk; i++, pk++, nsop++) {
            if (rc.sop) {
                be16(p, 0xFF91);
                be16(p + 2, 4);
                be16(p + 4, (uint32_t)(nsop & 0xFFFF));
                p += 6;
            }
            const uint32_t h0 = pk ? tt.hdr_end[pk - 1] : 0, h1 = tt.hdr_end[pk];
            std::memcpy(p, tt.hdr.data() + h0, h1 - h0);
            p += h1 - h0;
            if (rc.eph) {
                be16(p, 0xFF92);
                p += 2;
            }
            const uint32_t c0 = pk ? tt.pk_cend[pk - 1] : 0, c1 = tt.pk_cend[pk];
            for (uint32_t c = c0; c < c1; c++) {
                const uint32_t *e = &tt.contrib[(size_t)c * 3];
                std::memcpy(p, in.data + in.data_off[e[0]] + e[1], e[2] - e[1]);
                p += e[2] - e[1];
            }
        }
    }
}

void main_header(const Plan &P, std::vector<uint8_t> &v) {
    const jp2hip_recipe &rc = P.rc;
    const int L = rc.levels, nc = P.nc;
    v.clear();
    auto u8 = [&](int x) { v.push_back((uint8_t)x); };
    auto u16 = [&](int x) { u8(x >> 8); u8(x); };
    auto u32 = [&](uint32_t x) { u16((int)(x >> 16)); u16((int)(x & 0xFFFF)); };
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
        static const char msg[] = "jp2hip";
        u16(0xFF64);
        u16(4 + (int)(sizeof msg - 1));
        u16(1);
        for (size_t i = 0; i + 1 < sizeof msg; i++) u8(msg[i]);
    }
}

template <typename F>
void parallel_tiles(int ntiles, int threads, F &&f) {
    std::atomic<int> next(0);
    auto job = [&](int wid) {
        for (;;) {
            const int t = next.fetch_add(1);
            if (t >= ntiles) break;
            f(wid, t);
        }
    };
    const int nth = std::max(1, std::min(threads, ntiles));
    if (nth == 1) {
        job(0);
        return;
    }
    std::vector<std::thread> th;
    th.reserve((size_t)nth - 1);
    for (int i = 1; i < nth; i++) th.emplace_back(job, i);
    job(0);
    for (auto &x : th) x.join();
}

}  // namespace

static void tile_range(const T2Input &in, int &t0, int &t1) {
    const int ntiles = in.plan->ntx * in.plan->nty;
    t0 = std::max(0, in.tile0);
    t1 = in.tile1 < 0 ? ntiles : std::min(ntiles, in.tile1);
    if (t1 < t0) t1 = t0;
}

int64_t t2_headers(const T2Input &in, T2State &st) {
    const Plan &P = *in.plan;
    const int ntiles = P.ntx * P.nty;
    int t0, t1;
    tile_range(in, t0, t1);
    const int nth = std::max(1, std::min(in.threads, std::max(1, t1 - t0)));
    st.tiles.resize((size_t)ntiles);
    if ((int)st.workers.size() < nth) st.workers.resize((size_t)nth);
    for (auto &w : st.workers)
        if (w.lblock.size() < P.blocks.size()) {
            w.lblock.resize(P.blocks.size());
            w.incl.resize(P.blocks.size());
        }
    main_header(P, st.main);
    parallel_tiles(t1 - t0, nth, [&](int wid, int i) { tile_headers(in, t0 + i, st.tiles[t0 + i], st.workers[wid]); });
    int64_t total = (int64_t)st.main.size() + 2;
    for (int t = t0; t < t1; t++) total += (int64_t)st.tiles[t].bytes;
    st.total = total;
    return total;
}

uint64_t t2_part_bytes(const T2Input &in, const T2State &st, bool with_main, bool with_eoc) {
    int t0, t1;
    tile_range(in, t0, t1);
    uint64_t n = (with_main ? st.main.size() : 0) + (with_eoc ? 2 : 0);
    for (int t = t0; t < t1; t++) n += st.tiles[t].bytes;
    return n;
}

void t2_emit_part(const T2Input &in, const T2State &st, uint8_t *dst, bool with_main, bool with_eoc) {
    int t0, t1;
    tile_range(in, t0, t1);
    uint64_t o = 0;
    if (with_main) {
        std::memcpy(dst, st.main.data(), st.main.size());
        o = st.main.size();
    }
    std::vector<uint64_t> toff((size_t)(t1 - t0));
    for (int t = t0; t < t1; t++) {
        toff[t - t0] = o;
        o += st.tiles[t].bytes;
    }
    if (with_eoc) {
        dst[o] = 0xFF;
        dst[o + 1] = 0xD9;
    }
    parallel_tiles(t1 - t0, in.threads, [&](int, int i) { tile_emit(in, t0 + i, st.tiles[t0 + i], dst + toff[i]); });
}

void t2_emit(const T2Input &in, const T2State &st, uint8_t *dst) { t2_emit_part(in, st, dst, true, true); }

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
