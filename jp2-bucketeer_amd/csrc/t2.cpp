// t2.cpp -- tier-2 coding and code-stream / file assembly (ISO/IEC 15444-1
// Annex A, B.9-B.10, Annex I), run on host threads, one tile per task.
//
// Structure produced for the Bucketeer recipe (KakaduConverter.java:38-44):
// RPCL packets, SOP before and EPH after every packet header, one tile-part
// per resolution (ORGtparts=R) each carrying a PLT marker (ORGgen_plt=yes).
#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

#include "jp2hip_internal.h"

namespace jp2hip {

namespace {

struct Out {
    std::vector<uint8_t> &v;
    void u8(int x) { v.push_back((uint8_t)x); }
    void u16(int x) { u8(x >> 8); u8(x); }
    void u32(uint32_t x) { u16((int)(x >> 16)); u16((int)(x & 0xFFFF)); }
    void raw(const void *p, size_t n) {
        const uint8_t *b = (const uint8_t *)p;
        v.insert(v.end(), b, b + n);
    }
};

// Packet-header bit writer with the 0xFF bit-stuffing rule of B.10.1.
struct Bits {
    std::vector<uint8_t> &v;
    int acc = 0, n = 0;
    bool ff = false;
    explicit Bits(std::vector<uint8_t> &o) : v(o) {}
    void put(int b) {
        acc = (acc << 1) | (b & 1);
        if (++n == (ff ? 7 : 8)) {
            v.push_back((uint8_t)acc);
            ff = acc == 0xFF;
            acc = 0;
            n = 0;
        }
    }
    void put(uint32_t val, int nb) {
        for (int i = nb - 1; i >= 0; i--) put((int)((val >> i) & 1));
    }
    void flush() {
        if (n) {
            int cap = ff ? 7 : 8;
            int b = acc << (cap - n);
            v.push_back((uint8_t)b);
            ff = b == 0xFF;
            acc = 0;
            n = 0;
        }
        if (ff) {
            v.push_back(0);
            ff = false;
        }
    }
};

// Tag tree (B.10.2), leaves in raster order, parents by 2x2 grouping.
struct TagTree {
    struct Node { int parent, value, low; bool known; };
    std::vector<Node> nd;
    void build(int w, int h) {
        int lw[40], lh[40], nl = 0, tot = 0, cw = w, ch = h;
        for (;;) {
            lw[nl] = cw; lh[nl] = ch; tot += cw * ch; nl++;
            if (cw == 1 && ch == 1) break;
            cw = (cw + 1) / 2; ch = (ch + 1) / 2;
        }
        nd.assign((size_t)tot, Node{-1, 1 << 20, 0, false});
        int base = 0;
        for (int l = 0; l < nl; l++) {
            int pbase = base + lw[l] * lh[l];
            for (int y = 0; y < lh[l]; y++)
                for (int x = 0; x < lw[l]; x++)
                    nd[(size_t)base + y * lw[l] + x].parent =
                        (l + 1 < nl) ? pbase + (y / 2) * lw[l + 1] + x / 2 : -1;
            base = pbase;
        }
    }
    void set(int leaf, int v) {
        for (int i = leaf; i >= 0 && nd[i].value > v; i = nd[i].parent) nd[i].value = v;
    }
    void encode(Bits &w, int leaf, int threshold) {
        int stk[40], ns = 0;
        for (int i = leaf; i >= 0; i = nd[i].parent) stk[ns++] = i;
        int low = 0;
        for (int k = ns - 1; k >= 0; k--) {
            Node &n = nd[stk[k]];
            if (low > n.low) n.low = low;
            else low = n.low;
            while (low < threshold) {
                if (low >= n.value) {
                    if (!n.known) { w.put(1); n.known = true; }
                    break;
                }
                w.put(0);
                low++;
            }
            n.low = low;
        }
    }
};

int floor_log2(int v) {
    int r = -1;
    while (v) { v >>= 1; r++; }
    return r;
}

void put_plt(Out &o, const std::vector<uint32_t> &lens) {
    size_t i = 0;
    int z = 0;
    std::vector<uint8_t> seg;
    while (i < lens.size()) {
        seg.clear();
        while (i < lens.size()) {
            uint8_t tmp[5];
            int k = 0;
            uint32_t L = lens[i];
            tmp[k++] = (uint8_t)(L & 0x7F);
            L >>= 7;
            while (L) { tmp[k++] = (uint8_t)(0x80 | (L & 0x7F)); L >>= 7; }
            if (seg.size() + (size_t)k > 65532) break;
            for (int j = k - 1; j >= 0; j--) seg.push_back(tmp[j]);
            i++;
        }
        o.u16(0xFF58);
        o.u16((int)(3 + seg.size()));
        o.u8(z++);
        o.raw(seg.data(), seg.size());
    }
}

struct TileCoder {
    const T2Input &in;
    const Plan &P;
    int L;
    std::vector<int> lblock;   // indexed by block
    std::vector<int8_t> incl;  // first layer included, -1 none
    explicit TileCoder(const T2Input &i) : in(i), P(*i.plan), L(i.plan->rc.layers) {}

    int nl(int b, int l) const { return in.nl[(size_t)b * L + l]; }
    int rate(int b, int l) const { return in.lrate[(size_t)b * L + l]; }

    // appends one packet; returns its length (body included even when not copied)
    uint64_t packet(const Precinct &pr, std::vector<TagTree> &incl_tt, std::vector<TagTree> &zbp_tt,
                    int ttbase, int layer, int nsop, std::vector<uint8_t> &o) {
        const jp2hip_recipe &rc = P.rc;
        size_t start = o.size();
        if (rc.sop) {
            o.push_back(0xFF); o.push_back(0x91); o.push_back(0); o.push_back(4);
            o.push_back((uint8_t)((nsop >> 8) & 0xFF)); o.push_back((uint8_t)(nsop & 0xFF));
        }
        bool nonempty = false;
        for (int bi = 0; bi < pr.nb && !nonempty; bi++) {
            const PrecBand &pb = pr.pb[bi];
            for (int k = 0; k < pb.ncw * pb.nch; k++) {
                int b = pb.first + k;
                int prev = layer ? nl(b, layer - 1) : 0;
                if (nl(b, layer) > prev) { nonempty = true; break; }
            }
        }
        {
            Bits w(o);
            w.put(nonempty ? 1 : 0);
            if (nonempty) {
                for (int bi = 0; bi < pr.nb; bi++) {
                    const PrecBand &pb = pr.pb[bi];
                    for (int k = 0; k < pb.ncw * pb.nch; k++) {
                        int b = pb.first + k;
                        int prev = layer ? nl(b, layer - 1) : 0;
                        int n = nl(b, layer) - prev;
                        if (incl[b] < 0) incl_tt[ttbase + bi].encode(w, k, layer + 1);
                        else w.put(n > 0 ? 1 : 0);
                        if (n <= 0) continue;
                        if (incl[b] < 0) {
                            zbp_tt[ttbase + bi].encode(w, k, 1 << 20);
                            incl[b] = (int8_t)layer;
                        }
                        if (n == 1) w.put(0);
                        else if (n == 2) w.put(2u, 2);
                        else if (n <= 5) { w.put(3u, 2); w.put((uint32_t)(n - 3), 2); }
                        else if (n <= 36) { w.put(15u, 4); w.put((uint32_t)(n - 6), 5); }
                        else { w.put(511u, 9); w.put((uint32_t)(n - 37), 7); }
                        int r0 = layer ? rate(b, layer - 1) : 0;
                        int len = rate(b, layer) - r0;
                        int nb = lblock[b] + floor_log2(n);
                        while (len >= (1 << nb)) { w.put(1); lblock[b]++; nb++; }
                        w.put(0);
                        w.put((uint32_t)len, nb);
                    }
                }
            }
            w.flush();
        }
        if (rc.eph) { o.push_back(0xFF); o.push_back(0x92); }
        uint64_t body = 0;
        if (nonempty) {
            for (int bi = 0; bi < pr.nb; bi++) {
                const PrecBand &pb = pr.pb[bi];
                for (int k = 0; k < pb.ncw * pb.nch; k++) {
                    int b = pb.first + k;
                    int prev = layer ? nl(b, layer - 1) : 0;
                    if (nl(b, layer) <= prev) continue;
                    int r0 = layer ? rate(b, layer - 1) : 0, r1 = rate(b, layer);
                    if (in.data) {
                        const uint8_t *src = in.data + in.data_off[b] + r0;
                        o.insert(o.end(), src, src + (r1 - r0));
                    } else {
                        body += (uint64_t)(r1 - r0);
                    }
                }
            }
        }
        return (uint64_t)(o.size() - start) + body;
    }

    // all tile-parts of tile t; returns total bytes (bodies counted when not copied)
    uint64_t tile(int t, std::vector<uint8_t> &out) {
        const jp2hip_recipe &rc = P.rc;
        const Tile &T = P.tiles[t];
        const int Lv = rc.levels;
        int ntp = 0;
        for (int r = 0; r <= Lv; r++)
            if (T.tc[0].res[r].npx * T.tc[0].res[r].npy > 0) ntp++;
        // tag trees for every precinct-band of the tile
        std::vector<TagTree> itt, ztt;
        std::vector<int> ttbase;  // per (c, r, precinct)
        for (int c = 0; c < P.nc; c++)
            for (int r = 0; r <= Lv; r++) {
                const Resolution &R = T.tc[c].res[r];
                for (int p = 0; p < R.npx * R.npy; p++) {
                    const Precinct &pr = R.prec[p];
                    ttbase.push_back((int)itt.size());
                    for (int bi = 0; bi < pr.nb; bi++) {
                        const PrecBand &pb = pr.pb[bi];
                        itt.emplace_back();
                        ztt.emplace_back();
                        if (!pb.ncw || !pb.nch) continue;
                        itt.back().build(pb.ncw, pb.nch);
                        ztt.back().build(pb.ncw, pb.nch);
                        for (int k = 0; k < pb.ncw * pb.nch; k++) {
                            int b = pb.first + k;
                            lblock[b] = 3;
                            incl[b] = -1;
                            int first = L;
                            for (int l = 0; l < L; l++)
                                if (nl(b, l) > 0) { first = l; break; }
                            itt.back().set(k, first);
                            ztt.back().set(k, P.blocks[b].Mb - in.P[b]);
                        }
                    }
                }
            }
        // index of ttbase for (c, r, p)
        std::vector<int> cr_base((size_t)P.nc * (Lv + 1));
        {
            int idx = 0;
            for (int c = 0; c < P.nc; c++)
                for (int r = 0; r <= Lv; r++) {
                    cr_base[(size_t)c * (Lv + 1) + r] = idx;
                    idx += T.tc[c].res[r].npx * T.tc[c].res[r].npy;
                }
        }
        uint64_t total = 0;
        int tp = 0, nsop = 0;
        std::vector<uint8_t> pk;
        std::vector<uint32_t> plens;
        for (int r = 0; r <= Lv; r++) {
            const Resolution &R0 = T.tc[0].res[r];
            int np = R0.npx * R0.npy;
            if (np == 0) continue;
            for (int py = 0; py < R0.npy; py++)
                for (int px = 0; px < R0.npx; px++)
                    for (int c = 0; c < P.nc; c++) {
                        int pi = py * R0.npx + px;
                        const Precinct &pr = T.tc[c].res[r].prec[pi];
                        int tb = ttbase[cr_base[(size_t)c * (Lv + 1) + r] + pi];
                        for (int l = 0; l < L; l++) {
                            uint64_t len = packet(pr, itt, ztt, tb, l, nsop & 0xFFFF, pk);
                            nsop++;
                            plens.push_back((uint32_t)len);
                        }
                    }
            if (rc.tparts_r || r == Lv) {
                Out o{out};
                size_t sot = out.size();
                o.u16(0xFF90);
                o.u16(10);
                o.u16(t);
                o.u32(0);
                o.u8(tp);
                o.u8(rc.tparts_r ? ntp : 1);
                if (rc.plt) put_plt(o, plens);
                o.u16(0xFF93);
                uint64_t bodies = 0;
                for (uint32_t x : plens) bodies += x;
                uint64_t hdr = out.size() - sot;
                uint64_t psot = hdr + bodies;
                out[sot + 6] = (uint8_t)(psot >> 24);
                out[sot + 7] = (uint8_t)(psot >> 16);
                out[sot + 8] = (uint8_t)(psot >> 8);
                out[sot + 9] = (uint8_t)psot;
                out.insert(out.end(), pk.begin(), pk.end());
                total += psot;
                tp++;
                pk.clear();
                plens.clear();
            }
        }
        return total;
    }
};

void main_header(const Plan &P, std::vector<uint8_t> &v) {
    Out o{v};
    const jp2hip_recipe &rc = P.rc;
    int L = rc.levels, nc = P.nc;
    o.u16(0xFF4F);
    o.u16(0xFF51);
    o.u16(38 + 3 * nc);
    o.u16(0);
    o.u32((uint32_t)P.w); o.u32((uint32_t)P.h);
    o.u32(0); o.u32(0);
    o.u32((uint32_t)rc.tile_w); o.u32((uint32_t)rc.tile_h);
    o.u32(0); o.u32(0);
    o.u16(nc);
    for (int c = 0; c < nc; c++) { o.u8(P.bits - 1); o.u8(1); o.u8(1); }
    o.u16(0xFF52);
    o.u16(12 + L + 1);
    o.u8(0x01 | (rc.sop ? 2 : 0) | (rc.eph ? 4 : 0));
    o.u8(rc.progression);
    o.u16(rc.layers);
    o.u8((rc.mct && nc >= 3) ? 1 : 0);
    o.u8(L);
    o.u8(rc.cblk_w_log2 - 2);
    o.u8(rc.cblk_h_log2 - 2);
    o.u8(0);
    o.u8(rc.reversible ? 1 : 0);
    for (int r = 0; r <= L; r++) o.u8((prec_log2(rc, r, true) << 4) | prec_log2(rc, r, false));
    o.u16(0xFF5C);
    int nbands = 3 * L + 1;
    o.u16(3 + (rc.reversible ? nbands : 2 * nbands));
    o.u8((rc.guard_bits << 5) | (rc.reversible ? 0 : 2));
    for (int i = 0; i < nbands; i++) {
        int d = (i == 0) ? L : L - (i - 1) / 3;
        int band = (i == 0) ? 0 : 1 + (i - 1) % 3;
        BandQuant q = band_quant(rc, P.bits, d, band);
        if (rc.reversible) o.u8(q.eps << 3);
        else o.u16((q.eps << 11) | q.mu);
    }
    if (rc.comment) {
        static const char msg[] = "jp2hip";
        o.u16(0xFF64);
        o.u16(4 + (int)std::strlen(msg));
        o.u16(1);
        o.raw(msg, std::strlen(msg));
    }
}

}  // namespace

int64_t t2_write(const T2Input &in, std::vector<uint8_t> *out) {
    const Plan &P = *in.plan;
    const int ntiles = P.ntx * P.nty;
    std::vector<uint8_t> hdr;
    main_header(P, hdr);
    std::vector<std::vector<uint8_t>> tiles((size_t)ntiles);
    std::vector<uint64_t> sizes((size_t)ntiles, 0);
    std::atomic<int> next(0);
    // Each worker keeps its own per-block tier-2 state (Lblock, inclusion);
    // a tile only ever touches its own blocks.
    auto job = [&]() {
        TileCoder c(in);
        c.lblock.assign(P.blocks.size(), 3);
        c.incl.assign(P.blocks.size(), -1);
        for (;;) {
            int t = next.fetch_add(1);
            if (t >= ntiles) break;
            sizes[t] = c.tile(t, tiles[t]);
        }
    };
    const int nth = std::max(1, std::min(in.threads, ntiles));
    if (nth == 1) {
        job();
    } else {
        std::vector<std::thread> th;
        for (int i = 0; i < nth; i++) th.emplace_back(job);
        for (auto &x : th) x.join();
    }
    int64_t total = (int64_t)hdr.size() + 2;
    for (uint64_t s : sizes) total += (int64_t)s;
    if (out) {
        out->clear();
        out->reserve((size_t)total);
        out->insert(out->end(), hdr.begin(), hdr.end());
        for (auto &tv : tiles) out->insert(out->end(), tv.begin(), tv.end());
        out->push_back(0xFF);
        out->push_back(0xD9);
    }
    return total;
}

void wrap_file(const Plan &P, const std::vector<uint8_t> &cs, std::vector<uint8_t> &file) {
    file.clear();
    if (P.rc.format == JP2HIP_FORMAT_J2K) {
        file = cs;
        return;
    }
    Out o{file};
    static const uint8_t sig[12] = {0, 0, 0, 12, 'j', 'P', ' ', ' ', 0x0D, 0x0A, 0x87, 0x0A};
    o.raw(sig, 12);
    auto box = [&](uint32_t len, const char *t) { o.u32(len); o.raw(t, 4); };
    int nc = P.nc;
    if (P.rc.format == JP2HIP_FORMAT_JPX) {
        box(8 + 4 + 4 + 12, "ftyp");
        o.raw("jpx ", 4); o.u32(0);
        o.raw("jpx ", 4); o.raw("jp2 ", 4); o.raw("jpxb", 4);
        box(8 + 10, "rreq");
        o.u8(1); o.u8(0x80); o.u8(0x80);
        o.u16(1); o.u16(5); o.u8(0x80);
        o.u16(0);
    } else {
        box(8 + 4 + 4 + 4, "ftyp");
        o.raw("jp2 ", 4); o.u32(0); o.raw("jp2 ", 4);
    }
    bool cdef = (nc == 4 || nc == 2);
    uint32_t ihdr = 8 + 14, colr = 8 + 7, cdefl = cdef ? (uint32_t)(8 + 2 + 6 * nc) : 0;
    box(8 + ihdr + colr + cdefl, "jp2h");
    box(ihdr, "ihdr");
    o.u32((uint32_t)P.h); o.u32((uint32_t)P.w);
    o.u16(nc); o.u8(P.bits - 1); o.u8(7); o.u8(0); o.u8(0);
    box(colr, "colr");
    o.u8(1); o.u8(0); o.u8(0);
    o.u32(nc >= 3 ? 16 : 17);
    if (cdef) {
        box(cdefl, "cdef");
        o.u16(nc);
        for (int c = 0; c < nc; c++) {
            bool alpha = (c == nc - 1);
            o.u16(c); o.u16(alpha ? 1 : 0); o.u16(alpha ? 0 : c + 1);
        }
    }
    box((uint32_t)(8 + cs.size()), "jp2c");
    o.raw(cs.data(), cs.size());
}

}  // namespace jp2hip
