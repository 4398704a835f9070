// plan.cpp -- geometry of one encode: tiles, resolutions, precincts, bands
// and the flat code-block table the kernels consume; quantiser parameters.
//
// Geometry follows ISO/IEC 15444-1 B.5-B.7 for the recipe of
// KakaduConverter.java:38-44 (tiles anchored at 0, 2^L | tile size, so every
// decomposition level starts at an even coordinate).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <numeric>

#include "jp2hip_internal.h"

namespace jp2hip {

static int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
static uint64_t next_gen() {
    static std::atomic<uint64_t> g{0};
    return ++g;
}

int prec_log2(const jp2hip_recipe &rc, int r, bool vertical) {
    int idx = rc.levels - r;  // Kakadu lists the highest resolution first
    if (rc.nprecincts <= 0) return 15;
    if (idx >= rc.nprecincts) idx = rc.nprecincts - 1;
    return vertical ? rc.prec_h_log2[idx] : rc.prec_w_log2[idx];
}

// One-level synthesis basis vector: inverse lifting applied to an impulse.
static int synthesis_taps(bool rev, bool hi, double *taps) {
    constexpr int N = 64;
    double x[N] = {0};
    x[32 + (hi ? 1 : 0)] = 1.0;
    auto L = [&](int i) { return i ? x[i - 1] : x[1]; };
    auto R = [&](int i) { return i + 1 < N ? x[i + 1] : x[i - 1]; };
    if (rev) {
        for (int i = 0; i < N; i += 2) x[i] -= 0.25 * (L(i) + x[i + 1]);
        for (int i = 1; i < N; i += 2) x[i] += 0.5 * (x[i - 1] + R(i));
    } else {
        const double a = -1.586134342059924, b = -0.052980118572961, g = 0.882911075530934,
                     d = 0.443506852043971, K = 1.230174104914001;
        for (int i = 0; i < N; i += 2) x[i] *= K;
        for (int i = 1; i < N; i += 2) x[i] *= 1.0 / K;
        for (int i = 0; i < N; i += 2) x[i] -= d * (L(i) + x[i + 1]);
        for (int i = 1; i < N; i += 2) x[i] -= g * (x[i - 1] + R(i));
        for (int i = 0; i < N; i += 2) x[i] -= b * (L(i) + x[i + 1]);
        for (int i = 1; i < N; i += 2) x[i] -= a * (x[i - 1] + R(i));
    }
    int s = 0, e = N;
    while (s < e && x[s] == 0.0) s++;
    while (e > s && x[e - 1] == 0.0) e--;
    for (int i = s; i < e; i++) taps[i - s] = x[i];
    return e - s;
}

// Energy of the equivalent 1-D synthesis filter of a level-d band.
static double synthesis_energy(bool rev, int d, bool hi) {
    double g0[64], g1[64];
    int n0 = synthesis_taps(rev, false, g0), n1 = synthesis_taps(rev, true, g1);
    std::vector<double> f(1, 1.0), t;
    for (int k = d - 1; k >= 0; k--) {
        bool bh = (k == d - 1) && hi;
        const double *g = bh ? g1 : g0;
        int gn = bh ? n1 : n0, step = 1 << k;
        t.assign(f.size() + (size_t)(gn - 1) * step, 0.0);
        for (size_t i = 0; i < f.size(); i++)
            for (int j = 0; j < gn; j++) t[i + (size_t)j * step] += f[i] * g[j];
        f.swap(t);
    }
    double e = 0.0;
    for (double v : f) e += v * v;
    return e;
}

// L1 norm of the 5/3 analysis cascade (BIBO gain) for a level-d band axis.
static double bibo53(int d, bool hi) {
    static const double lo[5] = {-0.125, 0.25, 0.75, 0.25, -0.125};
    static const double h[3] = {-0.5, 1.0, -0.5};
    std::vector<double> f(1, 1.0), t;
    for (int k = 0; k < d; k++) {
        bool bh = (k == d - 1) && hi;
        const double *g = bh ? h : lo;
        int gl = bh ? 3 : 5, step = 1 << k;
        t.assign(f.size() + (size_t)(gl - 1) * step, 0.0);
        for (size_t i = 0; i < f.size(); i++)
            for (int j = 0; j < gl; j++) t[i + (size_t)j * step] += f[i] * g[j];
        f.swap(t);
    }
    double s = 0.0;
    for (double v : f) s += std::fabs(v);
    return s;
}

// tier-1 lanes: similar blocks side by side in a wavefront, biggest first
static void t1_lane_order(Plan &P) {
    P.t1_order.resize(P.blocks.size());
    std::iota(P.t1_order.begin(), P.t1_order.end(), 0);
    std::stable_sort(P.t1_order.begin(), P.t1_order.end(), [&](int a, int b) {
        const BlockDesc &A = P.blocks[a], &B = P.blocks[b];
        int wa = A.w * A.h, wb = B.w * B.h;
        if (wa != wb) return wa > wb;
        return A.Mb > B.Mb;
    });
}

int32_t lossless_layer_frac(int l, int NL) {
    // 6-layer fractions, indexed by layers below the top (fitted to
    // test.jpx's per-layer PSNR: tests/tools/fit_layers.py); other layer counts interpolate linearly at
    // the same relative depth, integer arithmetic as in the oracle
    static const int64_t f6[6] = {65536, 44515, 20178, 15645, 12923, 11253};
    if (l >= NL - 1) return 65536;
    const int64_t num = (int64_t)(NL - 1 - l) * 5, den = NL - 1;
    const int64_t i = num / den, r = num % den;
    if (i >= 5) return (int32_t)f6[5];
    return (int32_t)(f6[i] + (f6[i + 1] - f6[i]) * r / den);
}

// Rate-control groups of a plan whose tile rows are [tr0, tr1) of an image
// of `nty` tile rows (P.tile_b0 filled): the -flush_period stripes for a
// lossless recipe (whole stripes only: a tile-split band is made of them),
// else one group of every block.
static void rate_groups(Plan &P, int nty_full, int tr0, int tr1) {
    const int nb = (int)P.blocks.size();
    P.grp_b0.assign(1, 0);
    if (P.rc.rate_bpp <= 0.0 && nb) {
        const std::vector<int> ends = flush_stripe_ends(nty_full, P.rc.tile_h, P.h, P.rc.flush_period);
        for (int e : ends)
            if (e > tr0 && e <= tr1) P.grp_b0.push_back(P.tile_b0[(size_t)(e - tr0) * P.ntx]);
        if (P.grp_b0.back() != nb) P.grp_b0.push_back(nb);  // (never: the band ends on a stripe end)
    } else {
        P.grp_b0.push_back(nb);
    }
}

BandQuant band_quant(const jp2hip_recipe &rc, int bits, int d, int band) {
    BandQuant q;
    bool hx = (band == 1 || band == 3), hy = (band == 2 || band == 3);
    bool rev = rc.reversible != 0;
    double G = synthesis_energy(rev, d, hx) * synthesis_energy(rev, d, hy);
    if (rev) {
        double bibo = bibo53(d, hx) * bibo53(d, hy);
        q.eps = bits + (int)std::ceil(std::log2(1.1 * bibo));
        q.mu = 0;
        q.inv_delta = 1.0f;
        q.wnorm = G;
    } else {
        int gain = (hx ? 1 : 0) + (hy ? 1 : 0);
        double delta = rc.qstep * std::ldexp(1.0, bits) / std::sqrt(G);
        double ratio = delta / std::ldexp(1.0, bits + gain);
        int ex;
        double f = std::frexp(ratio, &ex);
        int eps = 1 - ex;
        int mu = (int)std::floor((2.0 * f - 1.0) * 2048.0 + 0.5);
        if (mu >= 2048) { mu = 0; eps -= 1; }
        eps = std::max(0, std::min(31, eps));
        q.eps = eps;
        q.mu = mu;
        double dq = std::ldexp(1.0 + mu / 2048.0, bits + gain - eps);
        q.inv_delta = 1.0f / (float)dq;
        q.wnorm = dq * dq * G;
    }
    q.Mb = rc.guard_bits + q.eps - 1;
    return q;
}

QuantTab quant_tab(const jp2hip_recipe &rc, int bits) {
    QuantTab t;
    std::memset(&t, 0, sizeof t);
    int mb = 0;
    auto put = [&](int d, int b) {
        const BandQuant q = band_quant(rc, bits, d, b);
        t.inv[d][b] = q.inv_delta;
        t.lim[d][b] = q.Mb >= 32 ? ~0u : (1u << q.Mb) - 1u;
        mb = std::max(mb, q.Mb);
    };
    for (int d = 1; d <= rc.levels; d++)
        for (int b = 1; b < 4; b++) put(d, b);
    put(rc.levels, 0);
    t.q16 = mb <= 15;
    return t;
}

bool build_plan(Plan &P, const jp2hip_recipe &rc, int w, int h, int nc, int bits,
                std::string &err) {
    if (w <= 0 || h <= 0 || nc < 1 || nc > 4 || (bits != 8 && bits != 16)) {
        err = "unsupported image geometry (1-4 components, 8 or 16 bits)";
        return false;
    }
    if (rc.progression != 2) { err = "only RPCL progression is implemented"; return false; }
    if (rc.levels < 0 || rc.levels > kMaxLevels || rc.layers < 1 || rc.layers > kMaxLayers) {
        err = "levels must be 0..12 and layers 1..32";
        return false;
    }
    if (rc.tile_w <= 0 || rc.tile_h <= 0 || (rc.tile_w % (1 << rc.levels)) ||
        (rc.tile_h % (1 << rc.levels)) || rc.tile_w > 4096 || rc.tile_h > 4096) {
        err = "tile size must be a multiple of 2^levels and <= 4096";
        return false;
    }
    if (rc.cblk_w_log2 < 2 || rc.cblk_w_log2 > 6 || rc.cblk_h_log2 < 2 || rc.cblk_h_log2 > 6) {
        err = "code-block size must be 4..64";
        return false;
    }
    P = Plan();
    P.rc = rc;
    P.w = w; P.h = h; P.nc = nc; P.bits = bits;
    P.ntx = (int)cdiv(w, rc.tile_w);
    P.nty = (int)cdiv(h, rc.tile_h);
    P.ntc = P.ntx * P.nty * nc;
    P.plane_w = rc.tile_w;
    P.plane_h = rc.tile_h;
    P.band_h = h;
    if (rc.mct && nc >= 3) {
        if (rc.reversible) { P.compw[0] = 3.0; P.compw[1] = 0.6875; P.compw[2] = 0.6875; }
        else {
            P.compw[0] = 3.0;
            P.compw[1] = 0.34413 * 0.34413 + 1.772 * 1.772;
            P.compw[2] = 1.402 * 1.402 + 0.71414 * 0.71414;
        }
    }
    const int L = rc.levels;
    // quantiser per (level, band), level 1..L
    std::vector<BandQuant> bq((size_t)(L + 1) * 4);
    for (int d = 1; d <= L; d++)
        for (int b = 1; b < 4; b++) bq[(size_t)d * 4 + b] = band_quant(rc, bits, d, b);
    bq[(size_t)L * 4 + 0] = band_quant(rc, bits, L, 0);

    P.tiles.resize((size_t)P.ntx * P.nty);
    P.tc_w.resize(P.ntc);
    P.tc_h.resize(P.ntc);
    uint64_t bpw = 0, smw = 0, ob = 0;
    for (int ty = 0; ty < P.nty; ty++) {
        for (int tx = 0; tx < P.ntx; tx++) {
            int t = ty * P.ntx + tx;
            Tile &T = P.tiles[t];
            P.tile_b0.push_back((int32_t)P.blocks.size());
            T.tx0 = tx * rc.tile_w; T.ty0 = ty * rc.tile_h;
            T.tx1 = std::min(w, T.tx0 + rc.tile_w);
            T.ty1 = std::min(h, T.ty0 + rc.tile_h);
            T.tc.resize(nc);
            int tw = T.tx1 - T.tx0, th = T.ty1 - T.ty0;
            int W[kMaxLevels + 2], H[kMaxLevels + 2];
            W[0] = tw; H[0] = th;
            for (int d = 1; d <= L; d++) { W[d] = (W[d - 1] + 1) / 2; H[d] = (H[d - 1] + 1) / 2; }
            for (int c = 0; c < nc; c++) {
                int tci = t * nc + c;
                P.tc_w[tci] = tw;
                P.tc_h[tci] = th;
                TileComp &TC = T.tc[c];
                for (int r = 0; r <= L; r++) {
                    int d = (r == 0) ? L : L - r + 1;
                    int sh = L - r;
                    int64_t trx0 = T.tx0 >> sh, try0 = T.ty0 >> sh;
                    int64_t trx1 = cdiv(T.tx1, (int64_t)1 << sh), try1 = cdiv(T.ty1, (int64_t)1 << sh);
                    int ppx = prec_log2(rc, r, false), ppy = prec_log2(rc, r, true);
                    Resolution &R = TC.res[r];
                    R.npx = trx1 > trx0 ? (int)(cdiv(trx1, (int64_t)1 << ppx) - (trx0 >> ppx)) : 0;
                    R.npy = try1 > try0 ? (int)(cdiv(try1, (int64_t)1 << ppy) - (try0 >> ppy)) : 0;
                    R.prec.assign((size_t)std::max(1, R.npx * R.npy), Precinct());
                    int pbx = (r == 0) ? ppx : ppx - 1, pby = (r == 0) ? ppy : ppy - 1;
                    int xcb = std::min(rc.cblk_w_log2, pbx), ycb = std::min(rc.cblk_h_log2, pby);
                    int nb = (r == 0) ? 1 : 3;
                    for (int bi = 0; bi < nb; bi++) {
                        int band = (r == 0) ? 0 : bi + 1;
                        bool hx = (band == 1 || band == 3), hy = (band == 2 || band == 3);
                        int64_t bx0 = T.tx0 >> d, by0 = T.ty0 >> d;
                        int bw = (r == 0) ? W[L] : (hx ? W[d - 1] - W[d] : W[d]);
                        int bh = (r == 0) ? H[L] : (hy ? H[d - 1] - H[d] : H[d]);
                        int offx = hx ? W[d] : 0, offy = hy ? H[d] : 0;
                        const BandQuant &q = bq[(size_t)d * 4 + band];
                        double wt = q.wnorm * P.compw[c] * 0.25;
                        for (int py = 0; py < R.npy; py++) {
                            for (int px = 0; px < R.npx; px++) {
                                Precinct &pr = R.prec[(size_t)py * R.npx + px];
                                pr.nb = nb;
                                PrecBand &pb = pr.pb[bi];
                                int64_t p0x = ((trx0 >> ppx) + px) << pbx;
                                int64_t p0y = ((try0 >> ppy) + py) << pby;
                                int64_t p1x = p0x + ((int64_t)1 << pbx), p1y = p0y + ((int64_t)1 << pby);
                                int64_t rx0 = std::max(p0x, bx0), ry0 = std::max(p0y, by0);
                                int64_t rx1 = std::min(p1x, bx0 + bw), ry1 = std::min(p1y, by0 + bh);
                                pb.first = (int)P.blocks.size();
                                if (rx1 <= rx0 || ry1 <= ry0) { pb.ncw = pb.nch = 0; continue; }
                                int64_t cx0 = rx0 >> xcb, cx1 = cdiv(rx1, (int64_t)1 << xcb);
                                int64_t cy0 = ry0 >> ycb, cy1 = cdiv(ry1, (int64_t)1 << ycb);
                                pb.ncw = (int)(cx1 - cx0);
                                pb.nch = (int)(cy1 - cy0);
                                for (int64_t cy = cy0; cy < cy1; cy++) {
                                    for (int64_t cx = cx0; cx < cx1; cx++) {
                                        int64_t x0 = std::max(cx << xcb, rx0), y0 = std::max(cy << ycb, ry0);
                                        int64_t x1 = std::min((cx + 1) << xcb, rx1), y1 = std::min((cy + 1) << ycb, ry1);
                                        BlockDesc bd;
                                        std::memset(&bd, 0, sizeof bd);
                                        bd.tc = tci;
                                        bd.x0 = (int16_t)(offx + (x0 - bx0));
                                        bd.y0 = (int16_t)(offy + (y0 - by0));
                                        bd.w = (int16_t)(x1 - x0);
                                        bd.h = (int16_t)(y1 - y0);
                                        bd.band = (int8_t)band;
                                        bd.Mb = (int8_t)q.Mb;
                                        bd.inv_delta = q.inv_delta;
                                        bd.bp_off = bpw;
                                        bd.sm_off = smw;
                                        bd.out_off = ob;
                                        uint64_t cap = ((uint64_t)bd.w * bd.h * (q.Mb + 1)) / 2 + 1024;
                                        cap = (cap + 15) & ~(uint64_t)15;
                                        bd.out_cap = (uint32_t)cap;
                                        bpw += (uint64_t)(q.Mb + 1) * 64;  // column masks (kernels.hip k_quant)
                                        smw += (uint64_t)64 * bd.h;
                                        ob += cap;
                                        P.blocks.push_back(bd);
                                        P.weight.push_back(wt);
                                    }
                                }
                            }
                        }
                    }
                }
            }
            for (int r = 0; r <= L; r++) {
                int np = T.tc[0].res[r].npx * T.tc[0].res[r].npy;
                P.npackets += (int64_t)np * nc * rc.layers;
                if (np) P.ntileparts++;
            }
        }
    }
    for (const BlockDesc &b : P.blocks)
        if (b.Mb > 30 || b.Mb < 0) { err = "band needs more than 30 magnitude bit-planes"; return false; }
    P.tile_b0.push_back((int32_t)P.blocks.size());
    P.bp_words = bpw;
    P.sm_words = smw;
    P.out_bytes = ob;
    rate_groups(P, P.nty, 0, P.nty);
    t1_lane_order(P);
    P.gen = next_gen();
    return true;
}

std::vector<int> flush_stripe_ends(int nty, int tile_h, int h, int period) {
    std::vector<int> ends;
    int64_t next = period;
    for (int ty = 0; ty < nty; ty++) {
        const int64_t bottom = std::min<int64_t>((int64_t)(ty + 1) * tile_h, h);
        if (period <= 0 || bottom >= next || ty == nty - 1) {
            ends.push_back(ty + 1);
            if (period > 0)
                while (next <= bottom) next += period;
        }
    }
    return ends;
}

void split_tile_rows(int nty, int tile_h, int h, int period, int rank, int world, int &tr0, int &tr1) {
    const std::vector<int> ends = flush_stripe_ends(nty, tile_h, h, period);
    const int64_t ns = (int64_t)ends.size();
    const int s0 = (int)(ns * rank / world), s1 = (int)(ns * (rank + 1) / world);
    tr0 = s0 > 0 ? ends[s0 - 1] : 0;
    tr1 = s1 > 0 ? ends[s1 - 1] : 0;
}

void make_subplan(const Plan &full, int tr0, int tr1, Plan &S) {
    S = Plan();
    S.rc = full.rc;
    S.w = full.w; S.h = full.h; S.nc = full.nc; S.bits = full.bits;
    S.ntx = full.ntx;
    S.nty = tr1 - tr0;
    S.ntc = S.ntx * S.nty * S.nc;
    S.plane_w = full.plane_w;
    S.plane_h = full.plane_h;
    std::memcpy(S.compw, full.compw, sizeof S.compw);
    S.tile0 = tr0 * full.ntx;
    const int tile1 = tr1 * full.ntx;
    S.row0 = std::min(full.h, tr0 * full.rc.tile_h);
    S.band_h = std::min(full.h, tr1 * full.rc.tile_h) - S.row0;
    const int tc0 = S.tile0 * full.nc, tc1 = tile1 * full.nc;
    S.tc_w.assign(full.tc_w.begin() + tc0, full.tc_w.begin() + tc1);
    S.tc_h.assign(full.tc_h.begin() + tc0, full.tc_h.begin() + tc1);
    // blocks are emitted tile by tile, so the band's blocks are contiguous
    const int nb = (int)full.blocks.size();
    int b0 = 0;
    while (b0 < nb && full.blocks[b0].tc < tc0) b0++;
    int b1 = b0;
    while (b1 < nb && full.blocks[b1].tc < tc1) b1++;
    S.block0 = b0;
    S.tile_b0.clear();
    for (int t = S.tile0; t <= tile1; t++) S.tile_b0.push_back(full.tile_b0[(size_t)t] - b0);
    S.blocks.assign(full.blocks.begin() + b0, full.blocks.begin() + b1);
    S.weight.assign(full.weight.begin() + b0, full.weight.begin() + b1);
    if (!S.blocks.empty()) {
        const BlockDesc f = S.blocks.front();
        for (BlockDesc &b : S.blocks) {
            b.tc -= tc0;
            b.bp_off -= f.bp_off;
            b.sm_off -= f.sm_off;
            b.out_off -= f.out_off;
        }
        const BlockDesc &l = S.blocks.back();
        S.bp_words = l.bp_off + (uint64_t)(l.Mb + 1) * 64;
        S.sm_words = l.sm_off + (uint64_t)64 * l.h;
        S.out_bytes = l.out_off + l.out_cap;
    }
    rate_groups(S, full.nty, tr0, tr1);
    t1_lane_order(S);
}

}  // namespace jp2hip
