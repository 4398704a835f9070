/*
 * jp2_oracle.c -- TEST INFRASTRUCTURE ONLY (see jp2_oracle.h).
 *
 * A deliberately plain, sample-at-a-time restatement of the JPEG 2000 Part 1
 * encode that Bucketeer asks Kakadu for:
 *
 *   kdu_compress -i <tif> -o <jpx> Clevels=6 Clayers=6
 *       Cprecincts={256,256},{256,256},{128,128} Stiles={512,512} Corder=RPCL
 *       ORGgen_plt=yes ORGtparts=R Cblk={64,64} Cuse_sop=yes Cuse_eph=yes
 *       -flush_period 1024 [Creversible=yes -rate - | -rate 3]
 *   (reference KakaduConverter.java:38-44, :61-68)
 *
 * Kakadu's source is not available, so every stage below
 * follows ISO/IEC 15444-1 directly:
 *   level shift + RCT/ICT ........ Annex G
 *   5/3 and 9/7 lifting DWT ...... Annex F (vertical pass, then horizontal)
 *   deadzone quantisation ........ Annex E (expounded step sizes)
 *   EBCOT tier-1 + MQ coder ...... Annex D, Annex C
 *   tier-2 packets, tag trees .... Annex B (RPCL, SOP/EPH, PLT, tile-part/R)
 *   JP2/JPX boxes ................ Annex I (and 15444-2 brand 'jpx ')
 * Rate control is the classical PCRD-opt convex-hull search with global
 * slope thresholds (one per quality layer).
 *
 * Choices that the standard leaves to the encoder are fixed here and
 * restated identically by libjp2hip (DESIGN.md "Encoder decisions"):
 *   - reversible exponents eps_b = B + ceil(log2(1.1 * BIBO_b)) where BIBO_b
 *     is the 5/3 analysis BIBO gain of the band; this reproduces the QCD of
 *     test.jpx byte for byte;
 *   - irreversible steps Delta_b = Qstep * 2^B / sqrt(G_b) (G_b = synthesis
 *     energy gain), Qstep = 1/256 (Kakadu default);
 *   - pass truncation lengths: bytes-so-far + 3, clipped to the terminated
 *     length, never ending on 0xFF;
 *   - per-pass distortion: exact squared error (half-units) of mid-point
 *     reconstruction, integer, weighted per band/component at PCRD time;
 *   - rate-driven ("-rate R") layer budgets halve from the final layer
 *     down, over the whole image;
 *   - lossless ("-rate -") layer budgets are fixed fractions of each
 *     -flush_period stripe's tier-1 bytes (lossless_layer_frac), so every
 *     stripe's layers are decided when its own tier-1 is done, as Kakadu's
 *     incremental flushing decides them; the fractions reproduce the
 *     per-layer PSNR of the reference's fixture test.jpx.
 */
#include "jp2_oracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* Experiment hooks (margin sweeps, decision censuses): read from the
 * environment only in a build with -DORACLE_EXPERIMENTS (make experiments ->
 * _build/liboracle_exp.so).  The parity oracle (liboracle.so) ignores the
 * environment, so no variable can change what the tests compare against. */
#ifdef ORACLE_EXPERIMENTS
#define ORACLE_EXP(name) getenv(name)
#else
#define ORACLE_EXP(name) ((const char *)0)
#endif

static char g_err[512];
static void set_err(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}
const char *oracle_last_error(void) { return g_err; }
void oracle_free(void *p) { free(p); }

static int ceil_div(int a, int b) { return (a + b - 1) / b; }
static int64_t ceil_div64(int64_t a, int64_t b) { return (a + b - 1) / b; }
static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

/* ------------------------------------------------------------------------ */
/* Recipe                                                                    */
/* ------------------------------------------------------------------------ */
void oracle_recipe_init(oracle_recipe *r, int lossless) {
    memset(r, 0, sizeof *r);
    r->levels = 6;
    r->layers = 6;
    r->tile_w = r->tile_h = 512;
    r->cblk_w_log2 = r->cblk_h_log2 = 6;
    r->nprecincts = 3;
    r->prec_w_log2[0] = r->prec_h_log2[0] = 8;
    r->prec_w_log2[1] = r->prec_h_log2[1] = 8;
    r->prec_w_log2[2] = r->prec_h_log2[2] = 7;
    r->progression = 2;
    r->sop = r->eph = r->plt = r->tparts_r = 1;
    r->guard_bits = 1;
    r->reversible = lossless ? 1 : 0;
    r->mct = 1;
    r->qstep = 1.0 / 256.0;
    r->rate_bpp = lossless ? 0.0 : 3.0;
    r->format = 2;
    r->comment = 1;
    r->slope_skip = 1;
    r->flush_period = 1024;
}

/* precinct exponent for resolution r (0 = lowest) given Kakadu ordering */
static int prec_log2(const oracle_recipe *rc, int r, int vertical) {
    int idx = rc->levels - r; /* 0 for the highest resolution */
    if (rc->nprecincts <= 0) return 15;
    if (idx >= rc->nprecincts) idx = rc->nprecincts - 1;
    return vertical ? rc->prec_h_log2[idx] : rc->prec_w_log2[idx];
}

/* ------------------------------------------------------------------------ */
/* TIFF (baseline, uncompressed strips, chunky or planar)                    */
/* ------------------------------------------------------------------------ */
typedef struct {
    const uint8_t *b;
    size_t n;
    int le;
} tiffbuf;

static uint32_t rd16(const tiffbuf *t, size_t off) {
    if (off + 2 > t->n) return 0;
    return t->le ? (uint32_t)(t->b[off] | (t->b[off + 1] << 8))
                 : (uint32_t)((t->b[off] << 8) | t->b[off + 1]);
}
static uint32_t rd32(const tiffbuf *t, size_t off) {
    if (off + 4 > t->n) return 0;
    if (t->le)
        return (uint32_t)t->b[off] | ((uint32_t)t->b[off + 1] << 8) |
               ((uint32_t)t->b[off + 2] << 16) | ((uint32_t)t->b[off + 3] << 24);
    return ((uint32_t)t->b[off] << 24) | ((uint32_t)t->b[off + 1] << 16) |
           ((uint32_t)t->b[off + 2] << 8) | (uint32_t)t->b[off + 3];
}

/* read value i of a tag (SHORT or LONG) */
static uint32_t tag_val(const tiffbuf *t, size_t entry, uint32_t i) {
    uint32_t type = rd16(t, entry + 2), cnt = rd32(t, entry + 4);
    uint32_t sz = (type == 3) ? 2 : (type == 4 ? 4 : 1);
    size_t base = (sz * cnt <= 4) ? entry + 8 : rd32(t, entry + 8);
    if (i >= cnt) return 0;
    if (sz == 2) return rd16(t, base + 2 * i);
    if (sz == 4) return rd32(t, base + 4 * i);
    return t->b[base + i];
}

int oracle_tiff_read(const uint8_t *buf, size_t len, int *W, int *H, int *NC,
                     int *BITS, void **PIX) {
    tiffbuf t = {buf, len, 1};
    if (len < 8) { set_err("tiff: too short"); return -1; }
    if (buf[0] == 'I' && buf[1] == 'I') t.le = 1;
    else if (buf[0] == 'M' && buf[1] == 'M') t.le = 0;
    else { set_err("tiff: bad byte order mark"); return -1; }
    if (rd16(&t, 2) != 42) { set_err("tiff: not a classic TIFF"); return -1; }
    size_t ifd = rd32(&t, 4);
    uint32_t n = rd16(&t, ifd);
    uint32_t w = 0, h = 0, spp = 1, bps = 8, comp = 1, planar = 1, rps = 0xFFFFFFFFu, fmt = 1;
    size_t e_off = 0, e_cnt = 0;
    uint32_t n_off = 0;
    for (uint32_t i = 0; i < n; i++) {
        size_t e = ifd + 2 + 12 * (size_t)i;
        uint32_t tag = rd16(&t, e);
        switch (tag) {
        case 256: w = tag_val(&t, e, 0); break;
        case 257: h = tag_val(&t, e, 0); break;
        case 258: bps = tag_val(&t, e, 0); break;
        case 259: comp = tag_val(&t, e, 0); break;
        case 273: e_off = e; n_off = rd32(&t, e + 4); break;
        case 277: spp = tag_val(&t, e, 0); break;
        case 278: rps = tag_val(&t, e, 0); break;
        case 279: e_cnt = e; break;
        case 284: planar = tag_val(&t, e, 0); break;
        case 339: fmt = tag_val(&t, e, 0); break;
        default: break;
        }
    }
    if (!w || !h || !e_off) { set_err("tiff: missing required tags"); return -1; }
    if (comp != 1) { set_err("tiff: compression %u not supported", comp); return -1; }
    if (bps != 8 && bps != 16) { set_err("tiff: %u bits/sample not supported", bps); return -1; }
    if (fmt != 1) { set_err("tiff: only unsigned integer samples"); return -1; }
    if (spp < 1 || spp > 4) { set_err("tiff: %u samples/pixel not supported", spp); return -1; }
    if (rps > h) rps = h;
    size_t bpsmp = bps / 8;
    size_t total = (size_t)w * h * spp * bpsmp;
    uint8_t *pix = (uint8_t *)malloc(total);
    if (!pix) { set_err("tiff: out of memory"); return -1; }
    uint32_t strips_per_plane = (h + rps - 1) / rps;
    uint32_t nplanes = (planar == 2) ? spp : 1;
    if (n_off < strips_per_plane * nplanes) { free(pix); set_err("tiff: strip count"); return -1; }
    for (uint32_t pl = 0; pl < nplanes; pl++) {
        for (uint32_t s = 0; s < strips_per_plane; s++) {
            uint32_t si = pl * strips_per_plane + s;
            size_t off = tag_val(&t, e_off, si);
            uint32_t y0 = s * rps, y1 = y0 + rps > h ? h : y0 + rps;
            size_t row = (size_t)w * (planar == 2 ? 1 : spp) * bpsmp;
            size_t need = row * (y1 - y0);
            if (off + need > len) { free(pix); set_err("tiff: strip out of range"); return -1; }
            (void)e_cnt;
            for (uint32_t y = y0; y < y1; y++) {
                const uint8_t *src = buf + off + (y - y0) * row;
                for (uint32_t x = 0; x < w; x++) {
                    for (uint32_t c = 0; c < (planar == 2 ? 1u : spp); c++) {
                        uint32_t cc = planar == 2 ? pl : c;
                        size_t si2 = ((size_t)x * (planar == 2 ? 1 : spp) + c) * bpsmp;
                        size_t di = (((size_t)y * w + x) * spp + cc) * bpsmp;
                        if (bpsmp == 1) pix[di] = src[si2];
                        else {
                            uint16_t v = t.le ? (uint16_t)(src[si2] | (src[si2 + 1] << 8))
                                              : (uint16_t)((src[si2] << 8) | src[si2 + 1]);
                            memcpy(pix + di, &v, 2);
                        }
                    }
                }
            }
        }
    }
    *W = (int)w; *H = (int)h; *NC = (int)spp; *BITS = (int)bps; *PIX = pix;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Wavelet constants and subband gains                                       */
/* ------------------------------------------------------------------------ */
/* Annex F, Table F.4 (9/7 irreversible lifting) */
#define A97 (-1.586134342059924f)
#define B97 (-0.052980118572961f)
#define G97 (0.882911075530934f)
#define D97 (0.443506852043971f)
#define K97 (1.230174104914001f)
#define INVK97 (0.8128930661159609f)

/* 1-D synthesis basis vector of one level: inverse lifting of an impulse
 * placed in the low (hi=0) or high (hi=1) channel, in double; returns the
 * non-zero taps. */
static int synth_taps(int rev, int hi, double *taps) {
    enum { N = 64 };
    double x[N];
    memset(x, 0, sizeof x);
    x[32 + hi] = 1.0;
    if (rev) {
        /* linearised 5/3: even -= (o+o)/4 ; odd += (e+e)/2 */
        for (int i = 0; i < N; i += 2) x[i] -= 0.25 * ((i ? x[i - 1] : x[1]) + x[i + 1]);
        for (int i = 1; i < N; i += 2) x[i] += 0.5 * (x[i - 1] + (i + 1 < N ? x[i + 1] : x[i - 1]));
    } else {
        const double a = -1.586134342059924, b = -0.052980118572961, g = 0.882911075530934,
                     d = 0.443506852043971, K = 1.230174104914001;
        for (int i = 0; i < N; i += 2) x[i] *= K;
        for (int i = 1; i < N; i += 2) x[i] *= 1.0 / K;
        for (int i = 0; i < N; i += 2) x[i] -= d * ((i ? x[i - 1] : x[1]) + x[i + 1]);
        for (int i = 1; i < N; i += 2) x[i] -= g * (x[i - 1] + (i + 1 < N ? x[i + 1] : x[i - 1]));
        for (int i = 0; i < N; i += 2) x[i] -= b * ((i ? x[i - 1] : x[1]) + x[i + 1]);
        for (int i = 1; i < N; i += 2) x[i] -= a * (x[i - 1] + (i + 1 < N ? x[i + 1] : x[i - 1]));
    }
    int s = 0, e = N;
    while (s < e && x[s] == 0.0) s++;
    while (e > s && x[e - 1] == 0.0) e--;
    for (int i = s; i < e; i++) taps[i - s] = x[i];
    return e - s;
}

/* equivalent 1-D synthesis filter energy for a band at level d (1-based)
 * along one axis: hi selects the high channel at the coarsest step.
 * f = up^{d-1}(g_band) * up^{d-2}(g0) * ... * g0 */
static double synth_energy_1d(int rev, int d, int hi) {
    double g0[64], g1[64];
    int n0 = synth_taps(rev, 0, g0), n1 = synth_taps(rev, 1, g1);
    static double f[1 << 16], tmp[1 << 16];
    int fl = 1;
    f[0] = 1.0;
    for (int k = d - 1; k >= 0; k--) {
        int band_hi = (k == d - 1) && hi;
        const double *g = band_hi ? g1 : g0;
        int gn = band_hi ? n1 : n0;
        int step = 1 << k;
        int nl = fl + (gn - 1) * step;
        for (int i = 0; i < nl; i++) tmp[i] = 0.0;
        for (int i = 0; i < fl; i++)
            for (int j = 0; j < gn; j++) tmp[i + j * step] += f[i] * g[j];
        fl = nl;
        for (int i = 0; i < fl; i++) f[i] = tmp[i];
    }
    double en = 0.0;
    for (int i = 0; i < fl; i++) en += f[i] * f[i];
    return en;
}

/* 1-D BIBO gain of the 5/3 analysis cascade (L1 norm), exact dyadic */
static double bibo53_1d(int d, int hi) {
    static const double lo[5] = {-0.125, 0.25, 0.75, 0.25, -0.125};
    static const double h[3] = {-0.5, 1.0, -0.5};
    static double f[1 << 16], tmp[1 << 16];
    int fl = 1;
    f[0] = 1.0;
    for (int k = 0; k < d; k++) {
        const double *g = (k == d - 1 && hi) ? h : lo;
        int gl = (k == d - 1 && hi) ? 3 : 5;
        int step = 1 << k;
        int nl = fl + (gl - 1) * step;
        for (int i = 0; i < nl; i++) tmp[i] = 0.0;
        for (int i = 0; i < fl; i++)
            for (int j = 0; j < gl; j++) tmp[i + j * step] += f[i] * g[j];
        fl = nl;
        for (int i = 0; i < fl; i++) f[i] = tmp[i];
    }
    double s = 0.0;
    for (int i = 0; i < fl; i++) s += fabs(f[i]);
    return s;
}

/* band parameters for (level d, orientation b): eps, mu, Mb, delta, weight */
typedef struct {
    int eps, mu, Mb;
    float inv_delta; /* irreversible only */
    double wnorm;    /* delta^2 * G_b (synthesis energy) */
} bandq;

static void band_quant(const oracle_recipe *rc, int B, int d, int b, bandq *q) {
    int hx = (b == 1 || b == 3), hy = (b == 2 || b == 3);
    double G = synth_energy_1d(rc->reversible, d, hx) * synth_energy_1d(rc->reversible, d, hy);
    if (rc->reversible) {
        double bibo = bibo53_1d(d, hx) * bibo53_1d(d, hy);
        int e = (int)ceil(log2(1.1 * bibo));
        q->eps = B + e;
        q->mu = 0;
        q->inv_delta = 1.0f;
        q->wnorm = G;
    } else {
        int gain = hx + hy;
        double delta = rc->qstep * ldexp(1.0, B) / sqrt(G);
        double ratio = delta / ldexp(1.0, B + gain);
        int ex;
        double f = frexp(ratio, &ex); /* ratio = f*2^ex, f in [0.5,1) */
        int eps = 1 - ex;
        int mu = (int)floor((2.0 * f - 1.0) * 2048.0 + 0.5);
        if (mu >= 2048) { mu = 0; eps -= 1; }
        if (eps < 0) eps = 0;
        if (eps > 31) eps = 31;
        q->eps = eps;
        q->mu = mu;
        double dq = ldexp(1.0 + mu / 2048.0, B + gain - eps);
        q->inv_delta = 1.0f / (float)dq;
        q->wnorm = dq * dq * G;
    }
    q->Mb = rc->guard_bits + q->eps - 1;
}

/* ------------------------------------------------------------------------ */
/* Forward DWT (Annex F): per level, vertical lifting then horizontal        */
/* ------------------------------------------------------------------------ */
static void fwd53_1d(int32_t *x, int n, int32_t *tmp) {
    if (n < 2) return;
    int nl = (n + 1) / 2, nh = n / 2;
    int32_t *s = tmp, *dd = tmp + nl;
    for (int k = 0; k < nh; k++) {
        int i = 2 * k + 1;
        int32_t r = (i + 1 < n) ? x[i + 1] : x[i - 1];
        dd[k] = x[i] - ((x[i - 1] + r) >> 1);
    }
    for (int k = 0; k < nl; k++) {
        int32_t dp = (k > 0) ? dd[k - 1] : dd[0];
        int32_t dn = (k < nh) ? dd[k] : dd[k - 1];
        s[k] = x[2 * k] + ((dp + dn + 2) >> 2);
    }
    memcpy(x, tmp, sizeof(int32_t) * (size_t)n);
}

static void fwd97_1d(float *x, int n, float *tmp) {
    if (n < 2) return;
    /* work in place on interleaved samples, then de-interleave */
    for (int i = 1; i < n; i += 2) {
        float r = (i + 1 < n) ? x[i + 1] : x[i - 1];
        float t = x[i - 1] + r;
        t = A97 * t;
        x[i] = x[i] + t;
    }
    for (int i = 0; i < n; i += 2) {
        float l = (i > 0) ? x[i - 1] : x[i + 1];
        float r = (i + 1 < n) ? x[i + 1] : x[i - 1];
        float t = l + r;
        t = B97 * t;
        x[i] = x[i] + t;
    }
    for (int i = 1; i < n; i += 2) {
        float r = (i + 1 < n) ? x[i + 1] : x[i - 1];
        float t = x[i - 1] + r;
        t = G97 * t;
        x[i] = x[i] + t;
    }
    for (int i = 0; i < n; i += 2) {
        float l = (i > 0) ? x[i - 1] : x[i + 1];
        float r = (i + 1 < n) ? x[i + 1] : x[i - 1];
        float t = l + r;
        t = D97 * t;
        x[i] = x[i] + t;
    }
    int nl = (n + 1) / 2;
    for (int k = 0; k < nl; k++) tmp[k] = x[2 * k] * INVK97;
    for (int k = 0; k < n / 2; k++) tmp[nl + k] = x[2 * k + 1] * K97;
    memcpy(x, tmp, sizeof(float) * (size_t)n);
}

void oracle_fdwt(void *data, int w, int h, int levels, int rev) {
    int maxn = imax(w, h);
    void *col = malloc(sizeof(int32_t) * (size_t)maxn);
    void *tmp = malloc(sizeof(int32_t) * (size_t)maxn);
    int cw = w, ch = h;
    for (int lv = 0; lv < levels; lv++) {
        /* vertical (columns) */
        for (int x = 0; x < cw; x++) {
            if (rev) {
                int32_t *d = (int32_t *)data, *c = (int32_t *)col;
                for (int y = 0; y < ch; y++) c[y] = d[(size_t)y * w + x];
                fwd53_1d(c, ch, (int32_t *)tmp);
                for (int y = 0; y < ch; y++) d[(size_t)y * w + x] = c[y];
            } else {
                float *d = (float *)data, *c = (float *)col;
                for (int y = 0; y < ch; y++) c[y] = d[(size_t)y * w + x];
                fwd97_1d(c, ch, (float *)tmp);
                for (int y = 0; y < ch; y++) d[(size_t)y * w + x] = c[y];
            }
        }
        /* horizontal (rows) */
        for (int y = 0; y < ch; y++) {
            if (rev) fwd53_1d((int32_t *)data + (size_t)y * w, cw, (int32_t *)tmp);
            else fwd97_1d((float *)data + (size_t)y * w, cw, (float *)tmp);
        }
        cw = (cw + 1) / 2;
        ch = (ch + 1) / 2;
    }
    free(col);
    free(tmp);
}

/* ------------------------------------------------------------------------ */
/* MQ coder (Annex C)                                                        */
/* ------------------------------------------------------------------------ */
static const uint16_t QE[47] = {
    0x5601, 0x3401, 0x1801, 0x0AC1, 0x0521, 0x0221, 0x5601, 0x5401, 0x4801, 0x3801, 0x3001, 0x2401,
    0x1C01, 0x1601, 0x5601, 0x5401, 0x5101, 0x4801, 0x3801, 0x3401, 0x3001, 0x2801, 0x2401, 0x2201,
    0x1C01, 0x1801, 0x1601, 0x1401, 0x1201, 0x1101, 0x0AC1, 0x09C1, 0x08A1, 0x0521, 0x0441, 0x02A1,
    0x0221, 0x0141, 0x0111, 0x0085, 0x0049, 0x0025, 0x0015, 0x0009, 0x0005, 0x0001, 0x5601};
static const uint8_t NMPS[47] = {1,  2,  3,  4,  5,  38, 7,  8,  9,  10, 11, 12, 13, 29, 15, 16,
                                 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32,
                                 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 45, 46};
static const uint8_t NLPS[47] = {1,  6,  9,  12, 29, 33, 6,  14, 14, 14, 17, 18, 20, 21, 14, 14,
                                 15, 16, 17, 18, 19, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29,
                                 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 46};
static const uint8_t SWTCH[47] = {1, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                  0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};

enum { CTX_RL = 17, CTX_UNI = 18, NCTX = 19 };

typedef struct {
    uint32_t C, A;
    int CT;
    uint8_t *bp, *start;
    uint8_t I[NCTX], MPS[NCTX];
} mqenc;

static void mq_init(mqenc *m, uint8_t *buf /* buf[-1] must exist */) {
    m->A = 0x8000;
    m->C = 0;
    m->CT = 12;
    m->bp = buf - 1;
    *m->bp = 0;
    m->start = buf;
    for (int i = 0; i < NCTX; i++) { m->I[i] = 0; m->MPS[i] = 0; }
    m->I[0] = 4;
    m->I[CTX_RL] = 3;
    m->I[CTX_UNI] = 46;
}

static void mq_byteout(mqenc *m) {
    if (*m->bp == 0xFF) {
        m->bp++;
        *m->bp = (uint8_t)(m->C >> 20);
        m->C &= 0xFFFFF;
        m->CT = 7;
    } else if ((m->C & 0x8000000) == 0) {
        m->bp++;
        *m->bp = (uint8_t)(m->C >> 19);
        m->C &= 0x7FFFF;
        m->CT = 8;
    } else {
        (*m->bp)++;
        if (*m->bp == 0xFF) {
            m->C &= 0x7FFFFFF;
            m->bp++;
            *m->bp = (uint8_t)(m->C >> 20);
            m->C &= 0xFFFFF;
            m->CT = 7;
        } else {
            m->bp++;
            *m->bp = (uint8_t)(m->C >> 19);
            m->C &= 0x7FFFF;
            m->CT = 8;
        }
    }
}

static void mq_renorm(mqenc *m) {
    do {
        m->A <<= 1;
        m->C <<= 1;
        if (--m->CT == 0) mq_byteout(m);
    } while ((m->A & 0x8000) == 0);
}

static int64_t g_decisions; /* debug counter (oracle_debug_decisions) */
int64_t oracle_debug_decisions(void) { int64_t v = g_decisions; g_decisions = 0; return v; }

static void mq_encode(mqenc *m, int cx, int d) {
    g_decisions++;
    int i = m->I[cx];
    uint32_t qe = QE[i];
    m->A -= qe;
    if (d == m->MPS[cx]) {
        if ((m->A & 0x8000) == 0) {
            if (m->A < qe) m->A = qe;
            else m->C += qe;
            m->I[cx] = NMPS[i];
            mq_renorm(m);
        } else {
            m->C += qe;
        }
    } else {
        if (m->A < qe) m->C += qe;
        else m->A = qe;
        if (SWTCH[i]) m->MPS[cx] ^= 1;
        m->I[cx] = NLPS[i];
        mq_renorm(m);
    }
}

static int mq_numbytes(const mqenc *m) { return (int)(m->bp - m->start); }

static int mq_flush(mqenc *m) {
    uint32_t tempc = m->C + m->A;
    m->C |= 0xFFFF;
    if (m->C >= tempc) m->C -= 0x8000;
    m->C <<= m->CT;
    mq_byteout(m);
    m->C <<= m->CT;
    mq_byteout(m);
    if (*m->bp != 0xFF) m->bp++;
    return (int)(m->bp - m->start);
}

/* ------------------------------------------------------------------------ */
/* Tier-1 (Annex D), one sample at a time                                    */
/* ------------------------------------------------------------------------ */
static int zc_context(int band, int h, int v, int d) {
    if (band == 1) { int t = h; h = v; v = t; } /* HL: swap roles */
    if (band == 3) {
        int hv = h + v;
        if (d >= 3) return 8;
        if (d == 2) return hv >= 1 ? 7 : 6;
        if (d == 1) return hv >= 2 ? 5 : (hv == 1 ? 4 : 3);
        return hv >= 2 ? 2 : (hv == 1 ? 1 : 0);
    }
    if (h == 2) return 8;
    if (h == 1) return v >= 1 ? 7 : (d >= 1 ? 6 : 5);
    if (v == 2) return 4;
    if (v == 1) return 3;
    if (d >= 2) return 2;
    return d == 1 ? 1 : 0;
}

/* distortion (half-units, squared) of value v known down to plane p */
static int64_t dist_at(uint32_t v, int p, int lossless) {
    int64_t t2 = 2 * (int64_t)v + (lossless ? 0 : 1);
    int64_t r2 = 0;
    if ((v >> p) != 0) {
        r2 = 2 * (int64_t)((v >> p) << p);
        if (!(lossless && p == 0)) r2 += (int64_t)1 << p;
    }
    int64_t e = t2 - r2;
    return e * e;
}

typedef struct {
    int w, h;
    const int32_t *sm;        /* sign-magnitude, row-major */
    uint8_t *sig, *pi, *ref;  /* (w+2)*(h+2), 1-sample border */
    int band, lossless;
    mqenc *mq;
} t1ctx;

#define IDX(t, x, y) (((y) + 1) * ((t)->w + 2) + (x) + 1)

static uint32_t mag(const t1ctx *t, int x, int y) { return (uint32_t)t->sm[y * t->w + x] & 0x7FFFFFFFu; }
static int sgn(const t1ctx *t, int x, int y) { return ((uint32_t)t->sm[y * t->w + x] >> 31) & 1; }

static void neigh_counts(const t1ctx *t, int x, int y, int *h, int *v, int *d) {
    int w2 = t->w + 2;
    const uint8_t *s = t->sig + IDX(t, x, y);
    *h = s[-1] + s[1];
    *v = s[-w2] + s[w2];
    *d = s[-w2 - 1] + s[-w2 + 1] + s[w2 - 1] + s[w2 + 1];
}

static void code_sign(t1ctx *t, int x, int y) {
    int w2 = t->w + 2;
    int k = IDX(t, x, y);
    int hc = 0, vc = 0;
    /* neighbour contributions: +1 positive significant, -1 negative */
    if (x > 0 && t->sig[k - 1]) hc += sgn(t, x - 1, y) ? -1 : 1;
    if (x + 1 < t->w && t->sig[k + 1]) hc += sgn(t, x + 1, y) ? -1 : 1;
    if (y > 0 && t->sig[k - w2]) vc += sgn(t, x, y - 1) ? -1 : 1;
    if (y + 1 < t->h && t->sig[k + w2]) vc += sgn(t, x, y + 1) ? -1 : 1;
    hc = hc < -1 ? -1 : (hc > 1 ? 1 : hc);
    vc = vc < -1 ? -1 : (vc > 1 ? 1 : vc);
    int ctx, xr;
    if (hc == 1) { xr = 0; ctx = vc == 1 ? 13 : (vc == 0 ? 12 : 11); }
    else if (hc == 0) { xr = vc == -1; ctx = vc == 0 ? 9 : 10; }
    else { xr = 1; ctx = vc == 1 ? 11 : (vc == 0 ? 12 : 13); }
    mq_encode(t->mq, ctx, sgn(t, x, y) ^ xr);
}

int oracle_t1_encode(const int32_t *sm, int w, int h, int band, int lossless,
                     uint8_t *out, int cap, int *out_len, int32_t *rates, int64_t *dists,
                     int *nplanes) {
    return oracle_t1_encode_planes(sm, w, h, band, lossless, 0, out, cap, out_len, rates, dists, nplanes);
}

/* Planes P-1 .. pmin only: the codeword is flushed after the last coded
 * pass, so the truncation lengths of the coded passes are those of a block
 * whose lower planes do not exist. */
static int64_t g_pass_dec[100];  /* experiments (ORACLE_PASS_WASTE): g_decisions at each pass end */
int oracle_t1_encode_planes(const int32_t *sm, int w, int h, int band, int lossless, int pmin,
                            uint8_t *out, int cap, int *out_len, int32_t *rates, int64_t *dists,
                            int *nplanes) {
    uint32_t maxv = 0;
    for (int i = 0; i < w * h; i++) {
        uint32_t v = (uint32_t)sm[i] & 0x7FFFFFFFu;
        if (v > maxv) maxv = v;
    }
    int P = 0;
    while (P < 31 && (maxv >> P)) P++;
    *nplanes = P;
    *out_len = 0;
    if (P == 0) return 0;
    size_t fs = (size_t)(w + 2) * (h + 2);
    uint8_t *flags = (uint8_t *)calloc(3 * fs, 1);
    uint8_t *buf = (uint8_t *)malloc((size_t)cap + 1);
    mqenc mq;
    mq_init(&mq, buf + 1);
    t1ctx t = {w, h, sm, flags, flags + fs, flags + 2 * fs, band, lossless, &mq};
    int np = 0;
    if (pmin < 0) pmin = 0;
    if (pmin > P - 1) pmin = P - 1;
    for (int p = P - 1; p >= pmin; p--) {
        for (int pass = (p == P - 1 ? 2 : 0); pass < 3; pass++) {
            int64_t dd = 0;
            for (int y0 = 0; y0 < h; y0 += 4) {
                for (int x = 0; x < w; x++) {
                    int y = y0;
                    if (pass == 2 && y0 + 4 <= h) {
                        /* run-length eligibility (D.3.4) */
                        int agg = 1;
                        for (int yy = y0; yy < y0 + 4 && agg; yy++) {
                            int k = IDX(&t, x, yy), hh, vv, dg;
                            neigh_counts(&t, x, yy, &hh, &vv, &dg);
                            if (t.sig[k] || t.pi[k] || hh + vv + dg) agg = 0;
                        }
                        if (agg) {
                            int r = -1;
                            for (int yy = y0; yy < y0 + 4; yy++)
                                if ((mag(&t, x, yy) >> p) & 1) { r = yy - y0; break; }
                            if (r < 0) {
                                mq_encode(&mq, CTX_RL, 0);
                                continue;
                            }
                            mq_encode(&mq, CTX_RL, 1);
                            mq_encode(&mq, CTX_UNI, r >> 1);
                            mq_encode(&mq, CTX_UNI, r & 1);
                            y = y0 + r;
                            uint32_t v = mag(&t, x, y);
                            dd += dist_at(v, p + 1, lossless) - dist_at(v, p, lossless);
                            t.sig[IDX(&t, x, y)] = 1;
                            code_sign(&t, x, y);
                            y++;
                        }
                    }
                    for (; y < y0 + 4 && y < h; y++) {
                        int k = IDX(&t, x, y);
                        uint32_t v = mag(&t, x, y);
                        int bit = (v >> p) & 1;
                        int hh, vv, dg;
                        neigh_counts(&t, x, y, &hh, &vv, &dg);
                        if (pass == 0) {
                            if (t.sig[k] || !(hh + vv + dg)) continue;
                            mq_encode(&mq, zc_context(band, hh, vv, dg), bit);
                            t.pi[k] = 1;
                            if (bit) {
                                dd += dist_at(v, p + 1, lossless) - dist_at(v, p, lossless);
                                t.sig[k] = 1;
                                code_sign(&t, x, y);
                            }
                        } else if (pass == 1) {
                            if (!t.sig[k] || t.pi[k]) continue;
                            int ctx = t.ref[k] ? 16 : ((hh + vv + dg) ? 15 : 14);
                            mq_encode(&mq, ctx, bit);
                            t.ref[k] = 1;
                            dd += dist_at(v, p + 1, lossless) - dist_at(v, p, lossless);
                        } else {
                            if (t.sig[k] || t.pi[k]) continue;
                            mq_encode(&mq, zc_context(band, hh, vv, dg), bit);
                            if (bit) {
                                dd += dist_at(v, p + 1, lossless) - dist_at(v, p, lossless);
                                t.sig[k] = 1;
                                code_sign(&t, x, y);
                            }
                        }
                    }
                }
            }
            if (pass == 2) memset(t.pi, 0, fs);
            dists[np] = dd;
            rates[np] = mq_numbytes(&mq) + 3;
            {   /* experiments: other truncation-length margins (round 6 layer-quality study) */
                const char *te = ORACLE_EXP("ORACLE_TRUNC_EXTRA");
                if (te) rates[np] = mq_numbytes(&mq) + atoi(te);
            }
            if (np < 100) g_pass_dec[np] = g_decisions;  /* experiments: decisions through each pass */
            np++;
            if (mq_numbytes(&mq) + 8 > cap) {
                free(flags); free(buf);
                set_err("t1: output capacity exceeded");
                return -1;
            }
        }
    }
    int len = mq_flush(&mq);
    rates[np - 1] = len;
    for (int i = 0; i < np; i++) {
        if (rates[i] > len) rates[i] = len;
        if (rates[i] > 1 && buf[1 + rates[i] - 1] == 0xFF) rates[i]--;
    }
    memcpy(out, buf + 1, (size_t)len);
    *out_len = len;
    free(flags);
    free(buf);
    return np;
}

/* ------------------------------------------------------------------------ */
/* Byte buffer and tier-2 bit writer (B.10.1)                                */
/* ------------------------------------------------------------------------ */
typedef struct { uint8_t *d; size_t n, cap; } bytes;
static void bput(bytes *b, const void *p, size_t n) {
    if (b->n + n > b->cap) {
        size_t nc = b->cap ? b->cap * 2 : 4096;
        while (nc < b->n + n) nc *= 2;
        b->d = (uint8_t *)realloc(b->d, nc);
        b->cap = nc;
    }
    memcpy(b->d + b->n, p, n);
    b->n += n;
}
static void bput8(bytes *b, int v) { uint8_t c = (uint8_t)v; bput(b, &c, 1); }
static void bput16(bytes *b, int v) { bput8(b, v >> 8); bput8(b, v); }
static void bput32(bytes *b, uint32_t v) { bput16(b, (int)(v >> 16)); bput16(b, (int)(v & 0xFFFF)); }
static void bset32(bytes *b, size_t at, uint32_t v) {
    b->d[at] = (uint8_t)(v >> 24); b->d[at + 1] = (uint8_t)(v >> 16);
    b->d[at + 2] = (uint8_t)(v >> 8); b->d[at + 3] = (uint8_t)v;
}

typedef struct { bytes *b; int acc, nbits, last_ff; } bitw;
static void bw_init(bitw *w, bytes *b) { w->b = b; w->acc = 0; w->nbits = 0; w->last_ff = 0; }
static void bw_bit(bitw *w, int bit) {
    int cap = w->last_ff ? 7 : 8;
    w->acc = (w->acc << 1) | (bit & 1);
    if (++w->nbits == cap) {
        bput8(w->b, w->acc);
        w->last_ff = (w->acc == 0xFF);
        w->acc = 0;
        w->nbits = 0;
    }
}
static void bw_bits(bitw *w, uint32_t v, int n) { for (int i = n - 1; i >= 0; i--) bw_bit(w, (v >> i) & 1); }
static void bw_flush(bitw *w) {
    if (w->nbits) {
        int cap = w->last_ff ? 7 : 8;
        int v = w->acc << (cap - w->nbits);
        bput8(w->b, v);
        w->last_ff = (v == 0xFF);
        w->acc = 0; w->nbits = 0;
    }
    if (w->last_ff) { bput8(w->b, 0); w->last_ff = 0; }
}

/* ------------------------------------------------------------------------ */
/* Tag trees (B.10.2)                                                        */
/* ------------------------------------------------------------------------ */
typedef struct { int parent, value, low, known; } ttnode;
typedef struct { int w, h, n; ttnode *nd; } tagtree;

static void tt_build(tagtree *t, int w, int h) {
    int lw[40], lh[40], nl = 0, tot = 0;
    int cw = w, ch = h;
    for (;;) {
        lw[nl] = cw; lh[nl] = ch; tot += cw * ch; nl++;
        if (cw == 1 && ch == 1) break;
        cw = (cw + 1) / 2; ch = (ch + 1) / 2;
    }
    t->w = w; t->h = h; t->n = tot;
    t->nd = (ttnode *)calloc((size_t)tot, sizeof(ttnode));
    int base = 0;
    for (int l = 0; l < nl; l++) {
        int pbase = base + lw[l] * lh[l];
        for (int y = 0; y < lh[l]; y++)
            for (int x = 0; x < lw[l]; x++)
                t->nd[base + y * lw[l] + x].parent =
                    (l + 1 < nl) ? pbase + (y / 2) * lw[l + 1] + x / 2 : -1;
        base = pbase;
    }
}
static void tt_reset(tagtree *t, int leaves_value_default) {
    for (int i = 0; i < t->n; i++) { t->nd[i].value = leaves_value_default; t->nd[i].low = 0; t->nd[i].known = 0; }
}
static void tt_set(tagtree *t, int leaf, int v) {
    int i = leaf;
    while (i >= 0 && t->nd[i].value > v) { t->nd[i].value = v; i = t->nd[i].parent; }
}
static void tt_encode(tagtree *t, bitw *w, int leaf, int threshold) {
    int stk[40], ns = 0;
    for (int i = leaf; i >= 0; i = t->nd[i].parent) stk[ns++] = i;
    int low = 0;
    for (int k = ns - 1; k >= 0; k--) {
        ttnode *n = &t->nd[stk[k]];
        if (low > n->low) n->low = low;
        else low = n->low;
        while (low < threshold) {
            if (low >= n->value) {
                if (!n->known) { bw_bit(w, 1); n->known = 1; }
                break;
            }
            bw_bit(w, 0);
            low++;
        }
        n->low = low;
    }
}

/* ------------------------------------------------------------------------ */
/* Code-stream model                                                         */
/* ------------------------------------------------------------------------ */
typedef struct {
    int band, w, h;      /* block size */
    int Mb, P, npasses;
    int32_t rates[100];  /* cumulative truncation lengths (pass n -> rates[n-1]) */
    int64_t dd[100];     /* per pass integer distortion decrease */
    uint8_t *data;
    int len;
    double weight;       /* PCRD weight (half-unit^2 -> image MSE) */
    int nhull, hull[101];
    double hslope[101];
    int nl[32];          /* cumulative passes after layer l */
    int lblock, incl;
    int32_t *sm;         /* quantised samples, kept until slope prediction ran */
    int pmin;            /* lowest coded bit-plane */
    uint32_t est[32];    /* predicted coded size of plane p, 1/16 bit */
    int64_t pd[32];      /* exact distortion decrease of plane p */
    int32_t *pdec;       /* experiments (ORACLE_PASS_WASTE): decisions per coded pass */
    int comp;            /* component (experiments) */
} cblk;

typedef struct {
    int ncw, nch;   /* code-block grid in this precinct-band */
    cblk **blk;
    tagtree incl, zbp;
} precband;

typedef struct { precband pb[3]; int nb; } precinct;

typedef struct {
    int npx, npy;
    precinct *prec;
} reslevel;

typedef struct {
    reslevel res[33];
} tilecomp;

typedef struct {
    int tx0, ty0, tx1, ty1;
    tilecomp *tc;
} tileinfo;

typedef struct {
    const oracle_recipe *rc;
    int w, h, nc, bits, ntx, nty;
    tileinfo *tiles;
    cblk **all;
    int nall, capall;
    double compw[4];
    int skip;            /* slope prediction active (rate-driven + slope_skip) */
    uint64_t K[32];      /* Kdu-Layer-Info slope keys per layer (0 = every pass) */
    int *tile_b0;        /* [ntiles + 1]: first block (in `all`) of each tile */
} encoder;

static void add_block(encoder *E, cblk *b) {
    if (E->nall == E->capall) {
        E->capall = E->capall ? E->capall * 2 : 1024;
        E->all = (cblk **)realloc(E->all, sizeof(cblk *) * (size_t)E->capall);
    }
    E->all[E->nall++] = b;
}

/* component samples for one tile after level shift and MCT */
static void tile_samples(const encoder *E, const void *pix, int tx0, int ty0, int tw, int th,
                         void **planes) {
    const oracle_recipe *rc = E->rc;
    int nc = E->nc, B = E->bits;
    int32_t off = 1 << (B - 1);
    int domct = rc->mct && nc >= 3;
    for (int y = 0; y < th; y++) {
        for (int x = 0; x < tw; x++) {
            size_t pi = ((size_t)(ty0 + y) * E->w + (tx0 + x)) * nc;
            int32_t s[4] = {0, 0, 0, 0};
            for (int c = 0; c < nc; c++)
                s[c] = (B == 8 ? (int32_t)((const uint8_t *)pix)[pi + c]
                               : (int32_t)((const uint16_t *)pix)[pi + c]) - off;
            size_t di = (size_t)y * tw + x;
            if (rc->reversible) {
                int32_t o[4] = {s[0], s[1 % nc], s[2 % nc], s[3 % nc]};
                if (domct) {
                    o[0] = (s[0] + 2 * s[1] + s[2]) >> 2;
                    o[1] = s[2] - s[1];
                    o[2] = s[0] - s[1];
                }
                for (int c = 0; c < nc; c++) ((int32_t *)planes[c])[di] = c < 3 ? o[c] : s[c];
            } else {
                float f[4];
                for (int c = 0; c < nc; c++) f[c] = (float)s[c];
                if (domct) {
                    float R = f[0], G = f[1], Bl = f[2];
                    float y0 = 0.299f * R; y0 = y0 + 0.587f * G; y0 = y0 + 0.114f * Bl;
                    float cb = -0.16875f * R; cb = cb - 0.33126f * G; cb = cb + 0.5f * Bl;
                    float cr = 0.5f * R; cr = cr - 0.41869f * G; cr = cr - 0.08131f * Bl;
                    f[0] = y0; f[1] = cb; f[2] = cr;
                }
                for (int c = 0; c < nc; c++) ((float *)planes[c])[di] = f[c];
            }
        }
    }
}

/* ------------------------------------------------------------------------ */
/* Slope prediction (rate-driven encodes only)                               */
/* ------------------------------------------------------------------------ */
/* kdu_compress with "-rate" (KakaduConverter.java:44) does not code the
 * passes PCRD-opt will certainly discard: its block coder stops at a slope
 * threshold predicted from the rate target.  Restated here exactly and
 * deterministically: each bit-plane p of a block gets a predicted coded size
 *     est = 16*refine + 56*new + 5*insignificant-next-to-significant
 * (1/16 bit: ~1 bit per refinement, ~3.5 bits per newly significant sample
 * with its sign, ~0.3 bit per zero decision next to significance) and its
 * exact distortion decrease pd; slope = pd * weight / est.  A histogram of
 * est over slope bins (1/8 octave) locates the bin where the predicted size
 * reaches the rate target; planes more than kSkipMargin bins (1.5 octaves)
 * below it are not coded.  PCRD-opt then runs on the coded passes as usual. */
enum { kSlopeBins = 1024, kSlopeBinBase = (1023 - 64) << 3, kSkipMargin = 12 };

static int slope_bin(double s) {
    if (!(s > 0.0)) return -1;
    uint64_t k;
    memcpy(&k, &s, 8);
    int b = (int)(k >> 49) - kSlopeBinBase;
    return b < 0 ? 0 : (b >= kSlopeBins ? kSlopeBins - 1 : b);
}

static int plane_bin(const cblk *b, int p) {
    if (b->est[p] == 0) return b->pd[p] > 0 ? kSlopeBins - 1 : -1;
    return slope_bin((double)b->pd[p] * b->weight / (double)b->est[p]);
}

static void plane_stats(cblk *b, const int32_t *sm, int lossless) {
    uint32_t maxv = 0;
    int w = b->w, h = b->h;
    for (int i = 0; i < w * h; i++) {
        uint32_t v = (uint32_t)sm[i] & 0x7FFFFFFFu;
        if (v > maxv) maxv = v;
    }
    int P = 0;
    while (P < 31 && (maxv >> P)) P++;
    b->P = P;
    for (int p = 0; p < P; p++) {
        int64_t nref = 0, nnew = 0, nnb = 0, pd = 0;
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                uint32_t v = (uint32_t)sm[y * w + x] & 0x7FFFFFFFu;
                if (v >> p) {
                    pd += dist_at(v, p + 1, lossless) - dist_at(v, p, lossless);
                    if (v >> (p + 1)) nref++;
                    else nnew++;
                    continue;
                }
                int nb = 0;
                for (int dy = -1; dy <= 1 && !nb; dy++)
                    for (int dx = -1; dx <= 1 && !nb; dx++) {
                        int xx = x + dx, yy = y + dy;
                        if ((dx || dy) && xx >= 0 && xx < w && yy >= 0 && yy < h &&
                            (((uint32_t)sm[yy * w + xx] & 0x7FFFFFFFu) >> p))
                            nb = 1;
                    }
                nnb += nb;
            }
        b->est[p] = (uint32_t)(16 * nref + 56 * nnew + 5 * nnb);
        b->pd[p] = pd;
    }
}

/* lowest plane to code: the lowest whose bin reaches kcut (at least the top) */
static int plane_cut(const cblk *b, int kcut) {
    int pmin = b->P > 0 ? b->P - 1 : 0;
    for (int p = 0; p < b->P; p++)
        if (plane_bin(b, p) >= kcut) { pmin = p; break; }
    return pmin;
}

/* bin threshold for a target of `target` bytes from the summed histogram */
static int predict_cut(const int64_t *hist, int64_t target) {
    int64_t acc = 0, goal = target * 128;  /* est is in 1/16 bit */
    int k = kSlopeBins - 1;
    for (; k > 0; k--) {
        acc += hist[k];
        if (acc >= goal) break;
    }
    const char *m = ORACLE_EXP("ORACLE_SKIP_MARGIN");  /* experiments only (margin sweeps) */
    return k - (m ? atoi(m) : kSkipMargin);
}

/* T1-code every block with its predicted plane range (skip mode) */
static int predict_and_code(encoder *E, int64_t target) {
    int64_t *hist = (int64_t *)calloc(kSlopeBins, sizeof(int64_t));
    for (int i = 0; i < E->nall; i++) {
        cblk *b = E->all[i];
        for (int p = 0; p < b->P; p++) {
            int k = plane_bin(b, p);
            if (k >= 0) hist[k] += b->est[p];
        }
    }
    int kcut = predict_cut(hist, target);
    if (ORACLE_EXP("ORACLE_SKIP_DEBUG")) { int64_t tot = 0; int lo = -1, hi = -1; for (int k = 0; k < kSlopeBins; k++) { tot += hist[k]; if (hist[k] && lo < 0) lo = k; if (hist[k]) hi = k; } fprintf(stderr, "skip: target %lld est_total_bytes %lld bins %d..%d kcut %d\n", (long long)target, (long long)(tot / 128), lo, hi, kcut); }
    free(hist);
    int lossless = E->rc->reversible;
    /* pass 0: predicted plane ranges.  Safety net: if every coded byte
     * together stays below the target while planes were skipped, the
     * prediction undershot -- code everything (pass 1). */
    for (int pass = 0; pass < 2; pass++) {
        int64_t total = 0;
        int skipped = 0;
        for (int i = 0; i < E->nall; i++) {
            cblk *b = E->all[i];
            b->pmin = pass == 0 ? plane_cut(b, kcut) : 0;
            skipped |= b->pmin > 0;
            int cap = b->w * b->h * 8 + 256;
            if (!b->data) b->data = (uint8_t *)malloc((size_t)cap);
            const int64_t dec0 = g_decisions;
            int np = oracle_t1_encode_planes(b->sm, b->w, b->h, b->band, lossless, b->pmin, b->data, cap,
                                             &b->len, b->rates, b->dd, &b->P);
            if (ORACLE_EXP("ORACLE_BLOCK_DECISIONS")) {  /* experiments: decisions per block */
                FILE *f = fopen(ORACLE_EXP("ORACLE_BLOCK_DECISIONS"), "a");
                if (f) { fprintf(f, "%lld %d\n", (long long)(g_decisions - dec0), np); fclose(f); }
            }
            if (np < 0) return -1;
            if (ORACLE_EXP("ORACLE_PASS_WASTE") && np > 0) {  /* experiments: decisions per coded pass */
                if (!b->pdec) b->pdec = (int32_t *)malloc(sizeof(int32_t) * 100);
                for (int q = 0; q < np && q < 100; q++) b->pdec[q] = (int32_t)(g_pass_dec[q] - (q ? g_pass_dec[q - 1] : dec0));
            }
            b->npasses = np;
            total += b->len;
        }
        if (ORACLE_EXP("ORACLE_SKIP_DEBUG")) fprintf(stderr, "skip pass %d: coded %lld bytes, %lld decisions so far\n", pass, (long long)total, (long long)g_decisions);
        if (pass == 0 && !(skipped && total < target)) break;
    }
    for (int i = 0; i < E->nall; i++) { free(E->all[i]->sm); E->all[i]->sm = NULL; }
    return 0;
}

/* encode all code-blocks of one tile-component; builds the precinct model */
static int code_tilecomp(encoder *E, tileinfo *T, int c, void *buf, int tw, int th) {
    const oracle_recipe *rc = E->rc;
    int L = rc->levels;
    tilecomp *tc = &T->tc[c];
    /* LL widths per level */
    int W[34], Hh[34];
    W[0] = tw; Hh[0] = th;
    for (int d = 1; d <= L; d++) { W[d] = (W[d - 1] + 1) / 2; Hh[d] = (Hh[d - 1] + 1) / 2; }
    for (int r = 0; r <= L; r++) {
        int d = (r == 0) ? L : L - r + 1;  /* decomposition level of the bands */
        int sh = L - r;
        int trx0 = T->tx0 >> sh, try0 = T->ty0 >> sh;
        int trx1 = (int)ceil_div64(T->tx1, (int64_t)1 << sh), try1 = (int)ceil_div64(T->ty1, (int64_t)1 << sh);
        int ppx = prec_log2(rc, r, 0), ppy = prec_log2(rc, r, 1);
        reslevel *rl = &tc->res[r];
        rl->npx = (trx1 > trx0) ? (int)(ceil_div64(trx1, (int64_t)1 << ppx) - (trx0 >> ppx)) : 0;
        rl->npy = (try1 > try0) ? (int)(ceil_div64(try1, (int64_t)1 << ppy) - (try0 >> ppy)) : 0;
        rl->prec = (precinct *)calloc((size_t)imax(1, rl->npx * rl->npy), sizeof(precinct));
        int pbx = (r == 0) ? ppx : ppx - 1, pby = (r == 0) ? ppy : ppy - 1;
        int xcb = imin(rc->cblk_w_log2, pbx), ycb = imin(rc->cblk_h_log2, pby);
        int nb = (r == 0) ? 1 : 3;
        for (int bi = 0; bi < nb; bi++) {
            int band = (r == 0) ? 0 : bi + 1;
            int hx = (band == 1 || band == 3), hy = (band == 2 || band == 3);
            /* band rectangle in global band coordinates and in the buffer */
            int bx0 = T->tx0 >> d, by0 = T->ty0 >> d;
            int bw = (r == 0) ? W[L] : (hx ? W[d - 1] - W[d] : W[d]);
            int bh = (r == 0) ? Hh[L] : (hy ? Hh[d - 1] - Hh[d] : Hh[d]);
            int offx = hx ? W[d] : 0, offy = hy ? Hh[d] : 0;
            bandq q;
            band_quant(rc, E->bits, d, band, &q);
            for (int py = 0; py < rl->npy; py++) {
                for (int px = 0; px < rl->npx; px++) {
                    precinct *pr = &rl->prec[py * rl->npx + px];
                    pr->nb = nb;
                    precband *pb = &pr->pb[bi];
                    /* precinct region in band coordinates */
                    int64_t p0x = ((int64_t)((trx0 >> ppx) + px)) << pbx;
                    int64_t p0y = ((int64_t)((try0 >> ppy) + py)) << pby;
                    int64_t p1x = p0x + ((int64_t)1 << pbx), p1y = p0y + ((int64_t)1 << pby);
                    int64_t rx0 = p0x > bx0 ? p0x : bx0, ry0 = p0y > by0 ? p0y : by0;
                    int64_t rx1 = p1x < bx0 + bw ? p1x : bx0 + bw, ry1 = p1y < by0 + bh ? p1y : by0 + bh;
                    if (rx1 <= rx0 || ry1 <= ry0) { pb->ncw = pb->nch = 0; continue; }
                    int cx0 = (int)(rx0 >> xcb), cx1 = (int)ceil_div64(rx1, (int64_t)1 << xcb);
                    int cy0 = (int)(ry0 >> ycb), cy1 = (int)ceil_div64(ry1, (int64_t)1 << ycb);
                    pb->ncw = cx1 - cx0;
                    pb->nch = cy1 - cy0;
                    pb->blk = (cblk **)calloc((size_t)(pb->ncw * pb->nch), sizeof(cblk *));
                    tt_build(&pb->incl, pb->ncw, pb->nch);
                    tt_build(&pb->zbp, pb->ncw, pb->nch);
                    for (int cy = cy0; cy < cy1; cy++) {
                        for (int cx = cx0; cx < cx1; cx++) {
                            int64_t x0 = (int64_t)cx << xcb, y0 = (int64_t)cy << ycb;
                            int64_t x1 = x0 + ((int64_t)1 << xcb), y1 = y0 + ((int64_t)1 << ycb);
                            if (x0 < rx0) x0 = rx0;
                            if (y0 < ry0) y0 = ry0;
                            if (x1 > rx1) x1 = rx1;
                            if (y1 > ry1) y1 = ry1;
                            cblk *b = (cblk *)calloc(1, sizeof(cblk));
                            b->band = band;
                            b->comp = c;
                            b->w = (int)(x1 - x0);
                            b->h = (int)(y1 - y0);
                            b->Mb = q.Mb;
                            b->weight = q.wnorm * E->compw[c] * 0.25;
                            /* quantise */
                            int32_t *sm = (int32_t *)malloc(sizeof(int32_t) * (size_t)(b->w * b->h));
                            uint32_t vmax = (q.Mb >= 31) ? 0x7FFFFFFFu : ((1u << q.Mb) - 1u);
                            for (int yy = 0; yy < b->h; yy++) {
                                for (int xx = 0; xx < b->w; xx++) {
                                    size_t bi2 = (size_t)(offy + (y0 - by0) + yy) * tw + (size_t)(offx + (x0 - bx0) + xx);
                                    uint32_t v, s;
                                    if (rc->reversible) {
                                        int32_t cf = ((int32_t *)buf)[bi2];
                                        s = cf < 0;
                                        v = (uint32_t)(cf < 0 ? -cf : cf);
                                    } else {
                                        float cf = ((float *)buf)[bi2];
                                        s = cf < 0.0f;
                                        float a = fabsf(cf) * q.inv_delta;
                                        v = (uint32_t)floorf(a);
                                    }
                                    if (v > vmax) v = vmax;
                                    sm[yy * b->w + xx] = (int32_t)((s << 31) | v);
                                }
                            }
                            if (E->skip) {
                                /* slope prediction first needs every block's
                                 * plane statistics: code later */
                                plane_stats(b, sm, rc->reversible);
                                b->sm = sm;
                                pb->blk[(cy - cy0) * pb->ncw + (cx - cx0)] = b;
                                add_block(E, b);
                                continue;
                            }
                            int cap = b->w * b->h * 8 + 256;
                            b->data = (uint8_t *)malloc((size_t)cap);
                            int64_t dec0 = g_decisions;
                            int np = oracle_t1_encode(sm, b->w, b->h, band, rc->reversible, b->data, cap,
                                                      &b->len, b->rates, b->dd, &b->P);
                            if (ORACLE_EXP("ORACLE_T1_STATS")) {
                                FILE *sf = fopen(ORACLE_EXP("ORACLE_T1_STATS"), "a");
                                if (sf) {
                                    fprintf(sf, "%d %d %d %d %d %d %lld %d\n", c, d, band, b->w, b->h, b->P,
                                            (long long)(g_decisions - dec0), b->len);
                                    fclose(sf);
                                }
                            }
                            free(sm);
                            if (np < 0) return -1;
                            b->npasses = np;
                            pb->blk[(cy - cy0) * pb->ncw + (cx - cx0)] = b;
                            add_block(E, b);
                        }
                    }
                }
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* PCRD-opt                                                                  */
/* ------------------------------------------------------------------------ */
static void build_hull(cblk *b) {
    int64_t D[101];
    int32_t R[101];
    D[0] = 0; R[0] = 0;
    for (int n = 1; n <= b->npasses; n++) { D[n] = D[n - 1] + b->dd[n - 1]; R[n] = b->rates[n - 1]; }
    b->nhull = 1;
    b->hull[0] = 0;
    b->hslope[0] = 0.0;
    for (int n = 1; n <= b->npasses; n++) {
        for (;;) {
            int h = b->hull[b->nhull - 1];
            int64_t dD = D[n] - D[h];
            int32_t dR = R[n] - R[h];
            if (dD <= 0) break;
            if (dR <= 0) { b->nhull--; continue; } /* h dominated (h > 0 here) */
            double s = (double)dD * b->weight / (double)dR;
            if (b->nhull >= 2 && s >= b->hslope[b->nhull - 1]) { b->nhull--; continue; }
            b->hull[b->nhull] = n;
            b->hslope[b->nhull] = s;
            b->nhull++;
            break;
        }
    }
}

typedef struct { uint64_t key; int32_t dr; } seg;
static int seg_cmp(const void *a, const void *b) {
    uint64_t x = ((const seg *)a)->key, y = ((const seg *)b)->key;
    return x < y ? 1 : (x > y ? -1 : 0);
}
static uint64_t slope_key(double s) { uint64_t k; memcpy(&k, &s, 8); return k; }

/* threshold key: smallest key K such that sum of dR over segments with
 * key >= K is <= budget (all segments of equal key taken together).
 * *Kc (the Kdu-Layer-Info slope): the smallest key k with that sum <= budget,
 * i.e. one above the first key not taken (0 if every segment is taken) --
 * the value a tile-split encode's bisection finds, so both agree. */
static uint64_t select_threshold(const seg *S, int ns, int64_t budget, uint64_t *Kc) {
    int64_t acc = 0;
    uint64_t K = UINT64_MAX;
    int i = 0;
    while (i < ns) {
        int j = i;
        int64_t grp = 0;
        while (j < ns && S[j].key == S[i].key) { grp += S[j].dr; j++; }
        if (acc + grp > budget) break;
        acc += grp;
        K = S[i].key;
        i = j;
    }
    *Kc = i < ns ? S[i].key + 1 : 0;
    return K;
}

/* Lossless ("-rate -") layer budgets: layer l of NL keeps the passes of a
 * stripe whose slopes clear the threshold that fits lossless_budget(T, l, NL)
 * bytes of that stripe's T tier-1 bytes; the last layer keeps every pass.
 * The fractions (1/65536 units, indexed by layers below the top) are fitted
 * (tests/tools/fit_layers.py) so that the first l layers decode
 * (opj_decompress -l l) to test.jpx's own RGB PSNR at layer l: 35.01 / 36.62 /
 * 39.06 / 42.36 / 55.50 dB (KakaduConverter.java:38-42 recipe).  A fit, so
 * tests/test_oracle.py's 0.3 dB check on test.jpx is a fit check; parity of
 * layer quality is unpinned for other images and layer counts.  Another layer
 * count interpolates the 6-layer curve linearly at the same relative depth,
 * in integers, so libjp2hip (plan.cpp lossless_layer_frac) computes the same. */
static const int64_t kLosslessFrac6[6] = {65536, 44515, 20178, 15645, 12923, 11253};

static int64_t lossless_layer_frac(int l, int NL) {
    if (l >= NL - 1) return 65536;
    const int64_t num = (int64_t)(NL - 1 - l) * 5, den = NL - 1;
    const int64_t i = num / den, r = num % den;
    if (i >= 5) return kLosslessFrac6[5];
    return kLosslessFrac6[i] + (kLosslessFrac6[i + 1] - kLosslessFrac6[i]) * r / den;
}

static int64_t lossless_budget(int64_t total, int l, int NL) {
    const char *ov = ORACLE_EXP("ORACLE_LAYER_FRACS");  /* experiments: fitting the table */
    if (ov && NL == 6 && l < NL - 1) {
        int64_t f[5];
        if (sscanf(ov, "%ld,%ld,%ld,%ld,%ld", &f[0], &f[1], &f[2], &f[3], &f[4]) == 5) return (total * f[l]) >> 16;
    }
    return (total * lossless_layer_frac(l, NL)) >> 16;
}

static int passes_for_key(const cblk *b, uint64_t K) {
    int n = 0;
    for (int i = 1; i < b->nhull; i++)
        if (slope_key(b->hslope[i]) >= K) n = b->hull[i];
    return n;
}

/* ------------------------------------------------------------------------ */
/* Tier-2 + code-stream                                                      */
/* ------------------------------------------------------------------------ */
static void reset_t2(encoder *E) {
    for (int i = 0; i < E->nall; i++) { E->all[i]->lblock = 3; E->all[i]->incl = -1; }
    const oracle_recipe *rc = E->rc;
    for (int t = 0; t < E->ntx * E->nty; t++)
        for (int c = 0; c < E->nc; c++)
            for (int r = 0; r <= rc->levels; r++) {
                reslevel *rl = &E->tiles[t].tc[c].res[r];
                for (int p = 0; p < rl->npx * rl->npy; p++)
                    for (int bi = 0; bi < rl->prec[p].nb; bi++) {
                        precband *pb = &rl->prec[p].pb[bi];
                        if (!pb->ncw || !pb->nch) continue;
                        tt_reset(&pb->incl, 1 << 20);
                        tt_reset(&pb->zbp, 1 << 20);
                        for (int k = 0; k < pb->ncw * pb->nch; k++) {
                            cblk *b = pb->blk[k];
                            int first = rc->layers;
                            for (int l = 0; l < rc->layers; l++)
                                if (b->nl[l] > 0) { first = l; break; }
                            tt_set(&pb->incl, k, first);
                            tt_set(&pb->zbp, k, b->Mb - b->P);
                        }
                    }
            }
}

static int floor_log2(int v) { int r = -1; while (v) { v >>= 1; r++; } return r; }

static void encode_packet(encoder *E, precinct *pr, int layer, bytes *out, int nsop) {
    const oracle_recipe *rc = E->rc;
    if (rc->sop) { bput16(out, 0xFF91); bput16(out, 4); bput16(out, nsop & 0xFFFF); }
    int nonempty = 0;
    for (int bi = 0; bi < pr->nb; bi++) {
        precband *pb = &pr->pb[bi];
        for (int k = 0; k < pb->ncw * pb->nch; k++) {
            cblk *b = pb->blk[k];
            int prev = layer ? b->nl[layer - 1] : 0;
            if (b->nl[layer] > prev) nonempty = 1;
        }
    }
    bytes hdr = {0, 0, 0};
    bitw w;
    bw_init(&w, &hdr);
    bw_bit(&w, nonempty);
    if (nonempty) {
        for (int bi = 0; bi < pr->nb; bi++) {
            precband *pb = &pr->pb[bi];
            for (int k = 0; k < pb->ncw * pb->nch; k++) {
                cblk *b = pb->blk[k];
                int prev = layer ? b->nl[layer - 1] : 0;
                int n = b->nl[layer] - prev;
                if (b->incl < 0) {
                    tt_encode(&pb->incl, &w, k, layer + 1);
                } else {
                    bw_bit(&w, n > 0);
                }
                if (n <= 0) continue;
                if (b->incl < 0) {
                    tt_encode(&pb->zbp, &w, k, 1 << 20);
                    b->incl = layer;
                }
                /* number of passes, Table B.4 */
                if (n == 1) bw_bit(&w, 0);
                else if (n == 2) bw_bits(&w, 2, 2);
                else if (n <= 5) { bw_bits(&w, 3, 2); bw_bits(&w, (uint32_t)(n - 3), 2); }
                else if (n <= 36) { bw_bits(&w, 15, 4); bw_bits(&w, (uint32_t)(n - 6), 5); }
                else { bw_bits(&w, 511, 9); bw_bits(&w, (uint32_t)(n - 37), 7); }
                int r0 = prev ? b->rates[prev - 1] : 0;
                int len = b->rates[b->nl[layer] - 1] - r0;
                int nb = b->lblock + floor_log2(n);
                while (len >= (1 << nb)) { bw_bit(&w, 1); b->lblock++; nb++; }
                bw_bit(&w, 0);
                bw_bits(&w, (uint32_t)len, nb);
            }
        }
    }
    bw_flush(&w);
    bput(out, hdr.d, hdr.n);
    free(hdr.d);
    if (rc->eph) bput16(out, 0xFF92);
    if (nonempty) {
        for (int bi = 0; bi < pr->nb; bi++) {
            precband *pb = &pr->pb[bi];
            for (int k = 0; k < pb->ncw * pb->nch; k++) {
                cblk *b = pb->blk[k];
                int prev = layer ? b->nl[layer - 1] : 0;
                if (b->nl[layer] <= prev) continue;
                int r0 = prev ? b->rates[prev - 1] : 0;
                int r1 = b->rates[b->nl[layer] - 1];
                bput(out, b->data + r0, (size_t)(r1 - r0));
            }
        }
    }
}

/* COM markers in Kakadu's layout (test.jpx): a
 * version string, then "Kdu-Layer-Info" with one line per quality layer:
 * log2 of the layer's slope threshold (squared error of samples normalised
 * to unit range, summed over the image, per byte) and the code-stream bytes
 * through that layer.  -192.0 marks "every pass" (the lossless last layer). */
#define JP2HIP_COM_VERSION "jp2hip-v0.2.0"
#define KDU_LAYER_HDR "Kdu-Layer-Info: log_2{Delta-D(squared-error)/Delta-L(bytes)}, L(bytes)\n"

static double layer_log_slope(uint64_t K, int bits) {
    if (K == 0) return -192.0;
    if (K >= 0x7FF0000000000000ull) return 192.0; /* nothing included */
    double s;
    memcpy(&s, &K, 8);
    double v = log2(s) - 2.0 * bits;
    return v < -192.0 ? -192.0 : (v > 192.0 ? 192.0 : v);
}

static int layer_info_len(int layers) { return (int)strlen(KDU_LAYER_HDR) + 17 * layers; }

static void write_main_header(encoder *E, bytes *o, const int64_t *layer_end) {
    const oracle_recipe *rc = E->rc;
    int L = rc->levels, nc = E->nc;
    bput16(o, 0xFF4F);
    /* SIZ */
    bput16(o, 0xFF51);
    bput16(o, 38 + 3 * nc);
    bput16(o, 0);
    bput32(o, (uint32_t)E->w); bput32(o, (uint32_t)E->h);
    bput32(o, 0); bput32(o, 0);
    bput32(o, (uint32_t)rc->tile_w); bput32(o, (uint32_t)rc->tile_h);
    bput32(o, 0); bput32(o, 0);
    bput16(o, nc);
    for (int c = 0; c < nc; c++) { bput8(o, E->bits - 1); bput8(o, 1); bput8(o, 1); }
    /* COD */
    bput16(o, 0xFF52);
    bput16(o, 12 + L + 1);
    bput8(o, 0x01 | (rc->sop ? 2 : 0) | (rc->eph ? 4 : 0));
    bput8(o, rc->progression);
    bput16(o, rc->layers);
    bput8(o, (rc->mct && nc >= 3) ? 1 : 0);
    bput8(o, L);
    bput8(o, rc->cblk_w_log2 - 2);
    bput8(o, rc->cblk_h_log2 - 2);
    bput8(o, 0);
    bput8(o, rc->reversible ? 1 : 0);
    for (int r = 0; r <= L; r++) bput8(o, (prec_log2(rc, r, 1) << 4) | prec_log2(rc, r, 0));
    /* QCD */
    bput16(o, 0xFF5C);
    int nbands = 3 * L + 1;
    bput16(o, 3 + (rc->reversible ? nbands : 2 * nbands));
    bput8(o, (rc->guard_bits << 5) | (rc->reversible ? 0 : 2));
    for (int i = 0; i < nbands; i++) {
        int d = (i == 0) ? L : L - (i - 1) / 3;
        int band = (i == 0) ? 0 : 1 + (i - 1) % 3;
        bandq q;
        band_quant(rc, E->bits, d, band, &q);
        if (rc->reversible) bput8(o, q.eps << 3);
        else bput16(o, (q.eps << 11) | q.mu);
    }
    if (rc->comment) {
        const char *ver = JP2HIP_COM_VERSION;
        bput16(o, 0xFF64);
        bput16(o, 4 + (int)strlen(ver));
        bput16(o, 1); /* Rcom: Latin-1 text */
        bput(o, ver, strlen(ver));
        bput16(o, 0xFF64);
        bput16(o, 4 + layer_info_len(rc->layers));
        bput16(o, 1);
        bput(o, KDU_LAYER_HDR, strlen(KDU_LAYER_HDR));
        for (int l = 0; l < rc->layers; l++) {
            char line[64];
            int n = snprintf(line, sizeof line, "%6.1f, %8.1e\n", layer_log_slope(E->K[l], E->bits),
                             (double)(layer_end ? layer_end[l] : 0));
            if (n != 17) { /* never for |slope| <= 192 and < 1e100 bytes */
                memset(line, ' ', 16);
                line[16] = '\n';
            }
            bput(o, line, 17);
        }
    }
}

static size_t main_header_len(encoder *E) {
    bytes h = {0, 0, 0};
    write_main_header(E, &h, NULL);
    size_t n = h.n;
    free(h.d);
    return n;
}

static void write_plt(bytes *o, const uint32_t *lens, int n) {
    int i = 0, z = 0;
    while (i < n) {
        bytes seg = {0, 0, 0};
        while (i < n) {
            uint8_t v[5];
            int k = 0;
            uint32_t L = lens[i];
            v[k++] = (uint8_t)(L & 0x7F);
            L >>= 7;
            while (L) { v[k++] = (uint8_t)(0x80 | (L & 0x7F)); L >>= 7; }
            if (seg.n + (size_t)k > 65532) break;
            for (int j = k - 1; j >= 0; j--) bput8(&seg, v[j]);
            i++;
        }
        bput16(o, 0xFF58);
        bput16(o, (int)(3 + seg.n));
        bput8(o, z++);
        bput(o, seg.d, seg.n);
        free(seg.d);
    }
}

/* Tile rows grouped the way "-flush_period P" flushes them
 * (KakaduConverter.java:40): tile rows are pushed top to bottom, and a flush
 * happens once the rows pushed reach the next multiple of P (and at the end
 * of the image); each flush writes the tile-parts of the tile rows it
 * completes.  ends[i] = one past the last tile row of stripe i.  P <= 0: one
 * stripe per tile row.  For test.jpx (2000 rows, 512-row tiles, P = 1024):
 * stripes {0, 1} and {2, 3}. */
static int flush_stripes(int nty, int tile_h, int h, int period, int *ends) {
    int n = 0;
    int64_t next = period;
    for (int ty = 0; ty < nty; ty++) {
        int64_t bottom = (int64_t)(ty + 1) * tile_h;
        if (bottom > h) bottom = h;
        if (period <= 0 || bottom >= next || ty == nty - 1) {
            ends[n++] = ty + 1;
            if (period > 0)
                while (next <= bottom) next += period;
        }
    }
    return n;
}

/* Packets of every tile in RPCL order, one tile-part per resolution with
 * ORGtparts=R (TNsot = 0 except on a tile's last tile-part, which carries the
 * count, as test.jpx does), written stripe by stripe: within a flush stripe,
 * resolution 0 of every tile, then resolution 1, ... (test.jpx: tiles 0-7
 * res 0, tiles 0-7 res 1, ..., then tiles 8-15). */
static void write_codestream(encoder *E, bytes *o) {
    const oracle_recipe *rc = E->rc;
    int L = rc->levels, NL = rc->layers, ntiles = E->ntx * E->nty;
    reset_t2(E);
    bytes *tp = (bytes *)calloc((size_t)ntiles * (L + 1), sizeof(bytes));
    int *ntp = (int *)calloc((size_t)ntiles, sizeof(int));
    int64_t layer_bytes[32];
    int64_t tp_hdr_bytes = 0;
    memset(layer_bytes, 0, sizeof layer_bytes);
    for (int t = 0; t < ntiles; t++) {
        tileinfo *T = &E->tiles[t];
        int nres = 0;
        for (int r = 0; r <= L; r++) {
            reslevel *rl = &T->tc[0].res[r];
            if (rl->npx * rl->npy > 0) nres++;
        }
        int nsop = 0;
        bytes pk = {0, 0, 0};
        uint32_t *plens = NULL;
        int npk = 0, cappk = 0;
        for (int r = 0; r <= L; r++) {
            reslevel *r0 = &T->tc[0].res[r];
            if (r0->npx * r0->npy == 0) continue;
            for (int py = 0; py < r0->npy; py++)
                for (int px = 0; px < r0->npx; px++)
                    for (int c = 0; c < E->nc; c++)
                        for (int l = 0; l < NL; l++) {
                            precinct *pr = &T->tc[c].res[r].prec[py * r0->npx + px];
                            size_t before = pk.n;
                            encode_packet(E, pr, l, &pk, nsop++);
                            if (npk == cappk) {
                                cappk = cappk ? 2 * cappk : 256;
                                plens = (uint32_t *)realloc(plens, sizeof(uint32_t) * (size_t)cappk);
                            }
                            plens[npk++] = (uint32_t)(pk.n - before);
                            layer_bytes[l] += (int64_t)(pk.n - before);
                        }
            if (rc->tparts_r || r == L) {
                bytes *o2 = &tp[(size_t)t * (L + 1) + ntp[t]];
                int k = ntp[t]++;
                bput16(o2, 0xFF90);
                bput16(o2, 10);
                bput16(o2, t);
                bput32(o2, 0);
                bput8(o2, k);
                /* TNsot: known (and written) on the tile's last tile-part */
                bput8(o2, rc->tparts_r ? (k == nres - 1 ? nres : 0) : 1);
                if (rc->plt) write_plt(o2, plens, npk);
                bput16(o2, 0xFF93);
                tp_hdr_bytes += (int64_t)o2->n;
                bput(o2, pk.d, pk.n);
                bset32(o2, 6, (uint32_t)o2->n);
                pk.n = 0;
                npk = 0;
            }
        }
        free(pk.d);
        free(plens);
    }
    /* Kdu-Layer-Info byte counts: the code-stream through each layer */
    int64_t layer_end[32];
    int64_t acc = (int64_t)main_header_len(E) + tp_hdr_bytes;
    for (int l = 0; l < NL; l++) { acc += layer_bytes[l]; layer_end[l] = acc; }
    if (ORACLE_EXP("ORACLE_LAYER_END"))  /* experiments: exact Kdu-Layer-Info bytes (fit_layers.py) */
        for (int l = 0; l < NL; l++) fprintf(stderr, "layer_end %d %lld\n", l, (long long)layer_end[l]);
    write_main_header(E, o, layer_end);
    int *ends = (int *)malloc(sizeof(int) * (size_t)(E->nty > 0 ? E->nty : 1));
    int ns = flush_stripes(E->nty, rc->tile_h, E->h, rc->flush_period, ends);
    for (int s = 0, ty0 = 0; s < ns; ty0 = ends[s++]) {
        int t0 = ty0 * E->ntx, t1 = ends[s] * E->ntx;
        for (int k = 0; k <= L; k++)
            for (int t = t0; t < t1; t++)
                if (k < ntp[t]) bput(o, tp[(size_t)t * (L + 1) + k].d, tp[(size_t)t * (L + 1) + k].n);
    }
    for (int i = 0; i < ntiles * (L + 1); i++) free(tp[i].d);
    free(tp);
    free(ntp);
    free(ends);
    bput16(o, 0xFFD9);
}

static void box_header(bytes *o, uint32_t len, const char *t) { bput32(o, len); bput(o, t, 4); }

static void wrap_file(encoder *E, const bytes *cs, bytes *o) {
    const oracle_recipe *rc = E->rc;
    int nc = E->nc;
    static const uint8_t sig[12] = {0, 0, 0, 12, 'j', 'P', ' ', ' ', 0x0D, 0x0A, 0x87, 0x0A};
    bput(o, sig, 12);
    if (rc->format == 2) {
        box_header(o, 8 + 4 + 4 + 12, "ftyp");
        bput(o, "jpx ", 4); bput32(o, 0);
        bput(o, "jpx ", 4); bput(o, "jp2 ", 4); bput(o, "jpxb", 4);
        /* reader requirements: one standard feature (5 = JPEG 2000 Part 1 compatible) */
        box_header(o, 8 + 1 + 1 + 1 + 2 + 1 + 2 + 1 + 1, "rreq");
        bput8(o, 1);              /* ML */
        bput8(o, 0x80);           /* FUAM */
        bput8(o, 0x80);           /* DCM */
        bput16(o, 1);             /* NSF */
        bput16(o, 5); bput8(o, 0x80);
        bput16(o, 0);             /* NVF */
    } else {
        box_header(o, 8 + 4 + 4 + 4, "ftyp");
        bput(o, "jp2 ", 4); bput32(o, 0); bput(o, "jp2 ", 4);
    }
    int cdef = (nc == 4 || nc == 2);
    uint32_t ihdr = 8 + 14, colr = 8 + 7, cdefl = cdef ? (uint32_t)(8 + 2 + 6 * nc) : 0;
    box_header(o, 8 + ihdr + colr + cdefl, "jp2h");
    box_header(o, ihdr, "ihdr");
    bput32(o, (uint32_t)E->h); bput32(o, (uint32_t)E->w);
    bput16(o, nc); bput8(o, E->bits - 1); bput8(o, 7); bput8(o, 0); bput8(o, 0);
    box_header(o, colr, "colr");
    bput8(o, 1); bput8(o, 0); bput8(o, 0);
    bput32(o, nc >= 3 ? 16 : 17);
    if (cdef) {
        box_header(o, cdefl, "cdef");
        bput16(o, nc);
        for (int c = 0; c < nc; c++) {
            int alpha = (c == nc - 1);
            bput16(o, c); bput16(o, alpha ? 1 : 0); bput16(o, alpha ? 0 : c + 1);
        }
    }
    box_header(o, (uint32_t)(8 + cs->n), "jp2c");
    bput(o, cs->d, cs->n);
}

static void free_encoder(encoder *E) {
    if (E->tiles) {
        for (int t = 0; t < E->ntx * E->nty; t++) {
            if (!E->tiles[t].tc) continue;
            for (int c = 0; c < E->nc; c++)
                for (int r = 0; r <= E->rc->levels; r++) {
                    reslevel *rl = &E->tiles[t].tc[c].res[r];
                    if (!rl->prec) continue;
                    for (int p = 0; p < rl->npx * rl->npy; p++)
                        for (int bi = 0; bi < 3; bi++) {
                            precband *pb = &rl->prec[p].pb[bi];
                            free(pb->blk);
                            free(pb->incl.nd);
                            free(pb->zbp.nd);
                        }
                    free(rl->prec);
                }
            free(E->tiles[t].tc);
        }
        free(E->tiles);
    }
    for (int i = 0; i < E->nall; i++) { free(E->all[i]->data); free(E->all[i]->sm); free(E->all[i]->pdec); free(E->all[i]); }
    free(E->all);
    free(E->tile_b0);
}

int oracle_encode(const void *pix, int w, int h, int nc, int bits, const oracle_recipe *rc,
                  uint8_t **out, size_t *out_len) {
    if (w <= 0 || h <= 0 || nc < 1 || nc > 4 || (bits != 8 && bits != 16)) {
        set_err("encode: unsupported image geometry"); return -1;
    }
    if (rc->progression != 2) { set_err("encode: only RPCL is supported"); return -1; }
    if (rc->levels < 0 || rc->levels > 12 || rc->layers < 1 || rc->layers > 32) {
        set_err("encode: levels must be 0..12 and layers 1..32"); return -1;
    }
    if ((rc->tile_w % (1 << rc->levels)) || (rc->tile_h % (1 << rc->levels))) {
        set_err("encode: tile size must be a multiple of 2^levels"); return -1;
    }
    encoder E;
    memset(&E, 0, sizeof E);
    E.rc = rc; E.w = w; E.h = h; E.nc = nc; E.bits = bits;
    E.skip = rc->slope_skip && rc->rate_bpp > 0.0;
    E.ntx = ceil_div(w, rc->tile_w);
    E.nty = ceil_div(h, rc->tile_h);
    /* component MSE weights: energy of the inverse colour transform columns */
    for (int c = 0; c < 4; c++) E.compw[c] = 1.0;
    if (rc->mct && nc >= 3) {
        if (rc->reversible) { E.compw[0] = 3.0; E.compw[1] = 0.6875; E.compw[2] = 0.6875; }
        else {
            E.compw[0] = 3.0;
            E.compw[1] = 0.34413 * 0.34413 + 1.772 * 1.772;
            E.compw[2] = 1.402 * 1.402 + 0.71414 * 0.71414;
        }
    }
    E.tiles = (tileinfo *)calloc((size_t)(E.ntx * E.nty), sizeof(tileinfo));
    E.tile_b0 = (int *)calloc((size_t)(E.ntx * E.nty) + 1, sizeof(int));
    for (int ty = 0; ty < E.nty; ty++) {
        for (int tx = 0; tx < E.ntx; tx++) {
            tileinfo *T = &E.tiles[ty * E.ntx + tx];
            E.tile_b0[ty * E.ntx + tx] = E.nall;
            T->tx0 = tx * rc->tile_w; T->ty0 = ty * rc->tile_h;
            T->tx1 = imin(w, T->tx0 + rc->tile_w); T->ty1 = imin(h, T->ty0 + rc->tile_h);
            T->tc = (tilecomp *)calloc((size_t)nc, sizeof(tilecomp));
            int tw = T->tx1 - T->tx0, th = T->ty1 - T->ty0;
            void *planes[4];
            for (int c = 0; c < nc; c++) planes[c] = malloc(sizeof(int32_t) * (size_t)tw * th);
            tile_samples(&E, pix, T->tx0, T->ty0, tw, th, planes);
            for (int c = 0; c < nc; c++) {
                oracle_fdwt(planes[c], tw, th, rc->levels, rc->reversible);
                if (code_tilecomp(&E, T, c, planes[c], tw, th)) {
                    for (int k = 0; k < nc; k++) free(planes[k]);
                    free_encoder(&E);
                    return -1;
                }
            }
            for (int c = 0; c < nc; c++) free(planes[c]);
        }
    }
    E.tile_b0[E.ntx * E.nty] = E.nall;
    if (E.skip &&
        predict_and_code(&E, (int64_t)floor(rc->rate_bpp * (double)w * (double)h / 8.0))) {
        free_encoder(&E);
        return -1;
    }
    /* PCRD */
    int ns = 0;
    for (int i = 0; i < E.nall; i++) { build_hull(E.all[i]); ns += E.all[i]->nhull - 1; }
    seg *S = (seg *)malloc(sizeof(seg) * (size_t)(ns ? ns : 1));
    int k = 0;
    int64_t total = 0;
    for (int i = 0; i < E.nall; i++) {
        cblk *b = E.all[i];
        for (int j = 1; j < b->nhull; j++) {
            S[k].key = slope_key(b->hslope[j]);
            S[k].dr = b->rates[b->hull[j] - 1] - (b->hull[j - 1] ? b->rates[b->hull[j - 1] - 1] : 0);
            k++;
        }
        if (b->npasses) total += b->rates[b->npasses - 1];
    }
    qsort(S, (size_t)ns, sizeof(seg), seg_cmp);
    int NL = rc->layers;
    int npackets = 0, ntparts = 0;
    for (int t = 0; t < E.ntx * E.nty; t++)
        for (int r = 0; r <= rc->levels; r++) {
            int np = E.tiles[t].tc[0].res[r].npx * E.tiles[t].tc[0].res[r].npy;
            npackets += np * nc * NL;
            if (np) ntparts++;
        }
    bytes cs = {0, 0, 0};
    if (rc->rate_bpp <= 0.0) {
        /* per -flush_period stripe: its own hull segments, its own budgets */
        int *ends = (int *)malloc(sizeof(int) * (size_t)(E.nty > 0 ? E.nty : 1));
        int nst = flush_stripes(E.nty, rc->tile_h, E.h, rc->flush_period, ends);
        for (int l = 0; l < NL; l++) E.K[l] = 0;
        for (int st = 0, ty0 = 0; st < nst; ty0 = ends[st++]) {
            int b0 = E.tile_b0[ty0 * E.ntx], b1 = E.tile_b0[ends[st] * E.ntx];
            int nss = 0;
            int64_t stotal = 0;
            for (int i = b0; i < b1; i++) {
                cblk *b = E.all[i];
                for (int j = 1; j < b->nhull; j++) {
                    S[nss].key = slope_key(b->hslope[j]);
                    S[nss].dr = b->rates[b->hull[j] - 1] - (b->hull[j - 1] ? b->rates[b->hull[j - 1] - 1] : 0);
                    nss++;
                }
                if (b->npasses) stotal += b->rates[b->npasses - 1];
            }
            qsort(S, (size_t)nss, sizeof(seg), seg_cmp);
            for (int l = 0; l < NL; l++) {
                uint64_t Kc = 0;
                uint64_t K = (l == NL - 1) ? 0 : select_threshold(S, nss, lossless_budget(stotal, l, NL), &Kc);
                {   /* experiments: fixed normalised slope thresholds instead of budgets */
                    const char *ls = ORACLE_EXP("ORACLE_LOSSLESS_SLOPES");
                    double q[5];
                    if (ls && l < 5 && sscanf(ls, "%lf,%lf,%lf,%lf,%lf", &q[0], &q[1], &q[2], &q[3], &q[4]) == 5)
                        K = Kc = slope_key(ldexp(pow(2.0, q[l]), 2 * E.bits));
                }
                if (Kc > E.K[l]) E.K[l] = Kc;  /* Kdu-Layer-Info: the strictest stripe's */
                for (int i = b0; i < b1; i++) {
                    cblk *b = E.all[i];
                    b->nl[l] = (l == NL - 1) ? b->npasses : passes_for_key(b, K);
                }
            }
        }
        free(ends);
        write_codestream(&E, &cs);
    } else {
        int64_t target = (int64_t)floor(rc->rate_bpp * (double)w * (double)h / 8.0);
        int64_t budget = target - 16 * (int64_t)npackets - 16 * (int64_t)ntparts - 256;
        for (int it = 0; it < 8; it++) {
            if (budget < 0) budget = 0;
            for (int l = 0; l < NL; l++) {
                uint64_t Kc;
                uint64_t K = select_threshold(S, ns, budget >> (NL - 1 - l), &Kc);
                E.K[l] = Kc;
                for (int i = 0; i < E.nall; i++) E.all[i]->nl[l] = passes_for_key(E.all[i], K);
            }
            cs.n = 0;
            write_codestream(&E, &cs);
            if ((int64_t)cs.n <= target) break;
            if (ORACLE_EXP("ORACLE_RATE_DEBUG")) fprintf(stderr, "rate it %d budget %lld size %zu target %lld\n", it, (long long)budget, cs.n, (long long)target);
            /* exponential back-off, plus 1/16 of the overshoot and 64 bytes so
             * the second pass (headers grow with the data they describe)
             * normally lands under the target instead of needing a third */
            budget -= (((int64_t)cs.n - target) << it) + (((int64_t)cs.n - target) >> 4) + 64;
        }
    }
    free(S);
    if (ORACLE_EXP("ORACLE_LAYER_DIST")) {  /* experiments: predicted distortion left after each layer */
        FILE *f = fopen(ORACLE_EXP("ORACLE_LAYER_DIST"), "a");
        for (int l = 0; f && l < NL; l++) {
            double left[4] = {0, 0, 0, 0};
            for (int i = 0; i < E.nall; i++) {
                cblk *b = E.all[i];
                double d = 0.0;
                for (int q = b->nl[l]; q < b->npasses; q++) d += (double)b->dd[q];
                left[b->comp] += d * b->weight;
            }
            fprintf(f, "%d %.6g %.6g %.6g %.6g\n", l, left[0], left[1], left[2], left[3]);
        }
        if (f) fclose(f);
    }
    if (ORACLE_EXP("ORACLE_PASS_WASTE")) {  /* experiments: coded decisions PCRD discards, by pass */
        FILE *f = fopen(ORACLE_EXP("ORACLE_PASS_WASTE"), "a");
        int64_t all = 0, kept = 0, lost[3] = {0, 0, 0}, lost_last[3] = {0, 0, 0}, lost_plane = 0;
        for (int i = 0; f && i < E.nall; i++) {
            cblk *b = E.all[i];
            if (!b->pdec) continue;
            int n = b->npasses, keep = b->nl[NL - 1];
            for (int q = 0; q < n && q < 100; q++) {
                int ty = q == 0 ? 2 : (q - 1) % 3;  /* 0 SPP, 1 MRP, 2 CUP */
                all += b->pdec[q];
                if (q < keep) { kept += b->pdec[q]; continue; }
                lost[ty] += b->pdec[q];
                if (q >= n - 3) lost_last[ty] += b->pdec[q];  /* the lowest coded plane */
                if (keep <= n - 3) lost_plane += b->pdec[q];   /* a whole plane or more discarded */
            }
        }
        if (f) {
            fprintf(f, "{\"decisions\": %lld, \"kept\": %lld, \"lost_spp\": %lld, \"lost_mrp\": %lld, \"lost_cup\": %lld, "
                       "\"lost_lowest_plane_spp\": %lld, \"lost_lowest_plane_mrp\": %lld, \"lost_lowest_plane_cup\": %lld, "
                       "\"lost_in_blocks_dropping_a_whole_plane\": %lld}\n",
                    (long long)all, (long long)kept, (long long)lost[0], (long long)lost[1], (long long)lost[2],
                    (long long)lost_last[0], (long long)lost_last[1], (long long)lost_last[2], (long long)lost_plane);
            fclose(f);
        }
    }
    bytes file = {0, 0, 0};
    if (rc->format == 0) file = cs;
    else { wrap_file(&E, &cs, &file); free(cs.d); }
    free_encoder(&E);
    *out = file.d;
    *out_len = file.n;
    return 0;
}

int oracle_encode_tiff(const uint8_t *tiff, size_t len, const oracle_recipe *r, uint8_t **out,
                       size_t *out_len) {
    int w, h, nc, bits;
    void *pix;
    if (oracle_tiff_read(tiff, len, &w, &h, &nc, &bits, &pix)) return -1;
    int rc = oracle_encode(pix, w, h, nc, bits, r, out, out_len);
    free(pix);
    return rc;
}
