// dwt.hip -- S1+S2+S3: TIFF ingest fused into the first DWT level, then the
// remaining levels (ISO/IEC 15444-1 Annex F, vertical lifting then
// horizontal lifting per level, symmetric extension, even start everywhere).
//
// Two kernels, both HBM-bound (B_dwt = C*[s + 4 + (8/3)(1 -
// 4^-(L-1))] bytes per pixel):
//
//   k_dwt_band<REV, INGEST, RB>  one decomposition level.  A workgroup owns
//       a band of RB output rows of one tile-component region; each thread
//       holds one column's rows [r0-4, r0+RB+4) in registers for the
//       vertical lifting (the 4-row halo on each side absorbs the lifting
//       footprint, so the RB kept rows are exact) and vertical scaling; the
//       kept rows go through LDS for horizontal lifting and scaling, and the
//       de-interleaved write: HL/LH/HH go
//       straight to their final Mallat position in `dst`, LL goes to a
//       compact scratch plane that the next level reads.  With INGEST the
//       band is read from the TIFF strips resident in HBM (level shift, RCT
//       or ICT for this component), so level 1 reads s bytes/sample and
//       writes 4: exactly the B_dwt term.
//   k_dwt_tail<REV>  the remaining levels once a level's region is at most
//       64 x 64: one small workgroup per tile-component runs every remaining
//       level in LDS and writes only final coefficients.
//
// Each coefficient is computed with the same expressions, in the same order,
// as oracle/jp2_oracle.c (fwd53_1d / fwd97_1d, oracle_fdwt): the halo rows
// reproduce exactly the values the full-column lifting would produce, so the
// output is bit-identical (built with -ffp-contract=off).
//
// Final coefficients leave as quantisation indices (quant_sm: the deadzone
// quantiser k_quant applied before, same expression): 16-bit sign-magnitude
// words for 8-bit sources (QuantTab::q16), so the plane k_quant reads back is
// half the f32 plane.  Only the LL of a non-final level stays raw (the LL
// scratch the next level reads).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "device_common.h"
#include "gpu_encoder.h"

namespace jp2hip {

#define A97 (-1.586134342059924f)
#define B97 (-0.052980118572961f)
#define G97 (0.882911075530934f)
#define D97 (0.443506852043971f)
#define K97 (1.230174104914001f)
#define INVK97 (0.8128930661159609f)

constexpr int kDwtThreads = 256;
constexpr int kDwtHalo = 4;           // >= lifting steps (9/7: 4, 5/3: 2)
constexpr int kDwtLdsWords = 16384;   // 64 KiB: band workgroups for rows <= 1024, tail
constexpr int kDwtLdsWordsWide = 32768;  // 128 KiB: band workgroups for rows of 2048 / 4096 (8 rows)

// One lifting step over the LDS rows [ya, yb) of a column set (vertical) or
// over one row (horizontal).  Sample i of parity `par` is updated from
// i-1 / i+1 with symmetric extension at the true signal ends 0 and n-1; a
// sample whose neighbour lies outside the staged window [ya, yb) is left
// stale (it is halo and never written out).
template <bool REV>
__device__ __forceinline__ void lift_update(void *buf, int idx, int lidx, int ridx, int step) {
    if (REV) {
        int32_t *x = (int32_t *)buf;
        if (step == 0) x[idx] -= (x[lidx] + x[ridx]) >> 1;
        else x[idx] += (x[lidx] + x[ridx] + 2) >> 2;
    } else {
        float *x = (float *)buf;
        const float cf = step == 0 ? A97 : (step == 1 ? B97 : (step == 2 ? G97 : D97));
        float t = x[lidx] + x[ridx];
        t = cf * t;
        x[idx] = x[idx] + t;
    }
}

// Vertical lifting of staged rows [ya, yb) (global row numbers, signal
// length H), W columns, row stride ld, rows stored from LDS row 0 = ya.
template <bool REV, int NT>
__device__ __forceinline__ void lift_vertical(void *lds, int ya, int yb, int H, int W, int ld) {
    if (H < 2) return;
    const int nsteps = REV ? 2 : 4;
    const int tid = threadIdx.x;
    for (int s = 0; s < nsteps; s++) {
        const int par = (s & 1) ? 0 : 1;  // odd rows first
        const int y0 = ya + ((ya & 1) != par ? 1 : 0);
        const int nr = (yb - y0 + 1) / 2;
        for (int it = tid; it < nr * W; it += NT) {
            const int k = it / W, x = it - k * W;
            const int y = y0 + 2 * k;
            int l = y > 0 ? y - 1 : y + 1;
            int r = y + 1 < H ? y + 1 : y - 1;
            if (l < ya || r < ya || l >= yb || r >= yb) continue;
            lift_update<REV>(lds, (y - ya) * ld + x, (l - ya) * ld + x, (r - ya) * ld + x, s);
        }
        __syncthreads();
    }
}

// Horizontal lifting of `nrows` full rows of length W starting at LDS row
// `row0`, row stride ld.
template <bool REV, int NT>
__device__ __forceinline__ void lift_horizontal(void *lds, int row0, int nrows, int W, int ld) {
    if (W < 2) return;
    const int nsteps = REV ? 2 : 4;
    const int tid = threadIdx.x;
    for (int s = 0; s < nsteps; s++) {
        const int par = (s & 1) ? 0 : 1;
        const int cnt = par ? W / 2 : (W + 1) / 2;
        for (int it = tid; it < nrows * cnt; it += NT) {
            const int k = it / cnt, j = it - k * cnt;
            const int x = par + 2 * j;
            const int l = x > 0 ? x - 1 : x + 1;
            const int r = x + 1 < W ? x + 1 : x - 1;
            const int base = (row0 + k) * ld;
            lift_update<REV>(lds, base + x, base + l, base + r, s);
        }
        __syncthreads();
    }
}

struct DwtBandArgs {
    // INGEST source: TIFF strips in HBM
    const uint8_t *tif;
    const uint64_t *strip_off;
    int rps, img_w, nc, bits, planar, big_endian, mct, spp_strips;
    int ntx, tile_w, tile_h, row0;  // row0: image row of tile row 0 (tile-split bands)
    // non-INGEST source: LL of the previous level (compact scratch planes)
    const void *src;
    int src_stride;
    size_t src_tc;
    // outputs
    void *dst;            // final Mallat planes
    int plane_w;
    size_t plane;
    void *ll;             // LL scratch (nullptr: LL is final, goes to dst)
    int ll_stride;
    size_t ll_tc;
    const int32_t *tc_w, *tc_h;
    int level, R;
    int ragged;  // some tile width is not a multiple of 16 (k_dwt_l1s second launch)
    QuantTab qt;
};

__device__ __forceinline__ int32_t tiff_sample(const DwtBandArgs &a, size_t rowoff, int x, int c) {
    size_t off = rowoff + (size_t)(a.planar == 2 ? x : x * a.nc + c) * (a.bits >> 3);
    if (a.bits == 8) return (int32_t)a.tif[off];
    uint32_t b0 = a.tif[off], b1 = a.tif[off + 1];
    return (int32_t)(a.big_endian ? ((b0 << 8) | b1) : (b0 | (b1 << 8)));
}

// One source sample of the band kernel's staging loop, level-shifted and
// colour-transformed (INGEST) or read from the previous level's LL.
template <bool REV, bool INGEST>
__device__ __forceinline__ int32_t band_load(const DwtBandArgs &a, int tc, int y, int x) {
    if (!INGEST) {
        const int32_t *s = (const int32_t *)a.src + (size_t)tc * a.src_tc;
        return s[(size_t)y * a.src_stride + x];
    }
    const int c = tc % a.nc, t = tc / a.nc;
    const int gx = (t % a.ntx) * a.tile_w + x, gy = a.row0 + (t / a.ntx) * a.tile_h + y;
    const int32_t off = 1 << (a.bits - 1);
    const size_t row_bytes = (size_t)a.img_w * (a.planar == 2 ? 1 : a.nc) * (a.bits >> 3);
    const int strip = gy / a.rps;
    const size_t ly = (size_t)(gy - strip * a.rps) * row_bytes;
    if (!(a.mct && a.nc >= 3 && c < 3)) {
        const uint64_t so = a.strip_off[a.planar == 2 ? (size_t)c * a.spp_strips + strip : (size_t)strip];
        const int32_t v = tiff_sample(a, so + ly, gx, c) - off;
        return REV ? v : __float_as_int((float)v);
    }
    int32_t sm[3];
#pragma unroll
    for (int q = 0; q < 3; q++) {
        const uint64_t so = a.strip_off[a.planar == 2 ? (size_t)q * a.spp_strips + strip : (size_t)strip];
        sm[q] = tiff_sample(a, so + ly, gx, q) - off;
    }
    if (REV) return c == 0 ? (sm[0] + 2 * sm[1] + sm[2]) >> 2 : (c == 1 ? sm[2] - sm[1] : sm[0] - sm[1]);
    const float R = (float)sm[0], G = (float)sm[1], B = (float)sm[2];
    float f;
    if (c == 0) { f = 0.299f * R; f = f + 0.587f * G; f = f + 0.114f * B; }
    else if (c == 1) { f = -0.16875f * R; f = f - 0.33126f * G; f = f + 0.5f * B; }
    else { f = 0.5f * R; f = f - 0.41869f * G; f = f - 0.08131f * B; }
    return __float_as_int(f);
}

// Vertical lifting of one column held in registers: v[i] is row
// y = y0 + i (y0 even, rows outside [0, H) are don't-care).  Symmetric
// extension at rows 0 and H-1; samples whose footprint leaves the window
// come out wrong and are never kept.
template <bool REV, int NR>
__device__ __forceinline__ void lift_regs(int32_t (&v)[NR], int y0, int H) {
    const int nsteps = REV ? 2 : 4;
    // a window wholly inside [0, H) needs no boundary selects (wave-uniform
    // for the vertical pass; per item for the horizontal one)
    const bool interior = y0 >= 0 && y0 + NR <= H;
#pragma unroll
    for (int s = 0; s < nsteps; s++) {
        const int par = (s & 1) ? 0 : 1;
#pragma unroll
        for (int i = par; i < NR; i += 2) {
            const int y = y0 + i;
            const int im = i > 0 ? i - 1 : i + 1, ip = i + 1 < NR ? i + 1 : i - 1;
            const int32_t l = (!interior && y == 0) ? v[ip] : v[im];
            const int32_t r = (interior || y + 1 < H) ? v[ip] : v[im];
            if (REV) {
                if (s == 0) v[i] -= (l + r) >> 1;
                else v[i] += (l + r + 2) >> 2;
            } else {
                const float cf = s == 0 ? A97 : (s == 1 ? B97 : (s == 2 ? G97 : D97));
                float t = __int_as_float(l) + __int_as_float(r);
                t = cf * t;
                v[i] = __float_as_int(__int_as_float(v[i]) + t);
            }
        }
    }
}

// One decomposition level for a band of RB output rows of one
// tile-component: vertical lifting in registers (thread = column, window of
// RB + 2*halo rows), the RB kept rows through LDS for horizontal lifting,
// then the de-interleaved write.
// Horizontal lifting (in LDS, thread = sample, row loop uniform), then
// scaling and the de-interleaved write -- consecutive threads store
// consecutive words, whole 256-byte runs per wave-instruction -- of NROWS
// staged rows (LDS row r at lds + kPadL + r * ld).  rows(r, o) fills row
// r's outputs (QRow; false: row r was not staged).  A register
// variant (16-sample segments, 16-byte stores) measured slower: its stores
// scatter over many lines per wave-instruction.
constexpr int kPadL = 4;   // LDS words in front of row 0 (the first segment's left halo)
// LDS row stride for W samples: a multiple of 4 words (16-byte reads), = 4
// mod 64 so consecutive rows start on different banks
__host__ __device__ constexpr int lds_row_stride(int W) { return ((W + 63) & ~63) + 4; }
constexpr int kPadR = 24;  // LDS words after the last row (the last segment's right halo)
// Skewed staging layout (k_dwt_l1s): 4 words of padding after every 16
// samples.  hlift_seg's lanes read 16-sample segments, 16 bytes at a time;
// in the dense layout the 16 lanes of a ds_read_b128 group sit 16 words
// apart, so only 4 distinct bank windows serve them (4-way conflicts); at 20
// words apart every lane of the group has its own 4 banks.
__host__ __device__ constexpr int skew_x(int x) { return x + ((x >> 4) << 2); }
__host__ __device__ constexpr int lds_row_stride_skew(int W) { return ((W + 15) >> 4) * 20 + 4; }
constexpr int kPadLs = 8;  // ... words in front of row 0: segment 0 reads 8 words before its samples

// Where one staged row's outputs go: its low half raw to the next level's LL
// row `ll` (a non-final level's even rows), or -- like its high half --
// quantised into the coefficient-plane row at `q` (element 0 = column 0 of
// the tile-component row; 2- or 4-byte elements), with the quantisers of
// the row's two bands.
struct QRow {
    int32_t *ll;
    uint8_t *q;
    float inv_lo, inv_hi;
    uint32_t lim_lo, lim_hi;
};
// Level lv's four quantisers (uniform: scalar loads from the arguments)
struct QLevel {
    float inv[4];
    uint32_t lim[4];
};
__device__ __forceinline__ QLevel qlevel(const QuantTab &qt, int lv) {
    QLevel l;
#pragma unroll
    for (int b = 0; b < 4; b++) {
        l.inv[b] = qt.inv[lv][b];
        l.lim[b] = qt.lim[lv][b];
    }
    return l;
}
// even rows: LL (final at the last level) + HL; odd rows: LH + HH.
// (Selects of register values: as selects of the struct's fields the
// compiler made the struct a scratch slot and each select a scratch load
// from a selected address, per staged row.)
__device__ __forceinline__ void qrow_bands(QRow &o, const QLevel &l, bool yodd) {
    float i0 = l.inv[0], i1 = l.inv[1], i2 = l.inv[2], i3 = l.inv[3];
    uint32_t m0 = l.lim[0], m1 = l.lim[1], m2 = l.lim[2], m3 = l.lim[3];
    asm("" : "+v"(i0), "+v"(i1), "+v"(i2), "+v"(i3), "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3));
    o.inv_lo = yodd ? i2 : i0;
    o.lim_lo = yodd ? m2 : m0;
    o.inv_hi = yodd ? i3 : i1;
    o.lim_hi = yodd ? m3 : m1;
}
// the coefficient-plane row `row` of tile-component tc
__device__ __forceinline__ uint8_t *qplane_row(void *dst, size_t plane, int tc, size_t row, int plane_w, bool q16) {
    return (uint8_t *)dst + (((size_t)tc * plane + row * (size_t)plane_w) << (q16 ? 1 : 2));
}
template <bool REV>
__device__ __forceinline__ void store_q1(uint8_t *q, int e, int32_t x, float inv, uint32_t lim, bool q16) {
    if (q16) ((uint16_t *)q)[e] = (uint16_t)quant_sm<REV>(x, inv, lim, 15);
    else ((uint32_t *)q)[e] = quant_sm<REV>(x, inv, lim, 31);
}
// n (<= 8) values v[s0], v[s0 + 2], ... quantised to elements e0 .. e0+n-1:
// one 16-byte store (16-bit) or two (32-bit) when whole and aligned
template <bool REV>
__device__ __forceinline__ void store_q8(uint8_t *q, int e0, const int32_t (&v)[24], int s0, int n, float inv,
                                         uint32_t lim, bool q16) {
    uint32_t w[8];
    if (q16) {
        // pairs: magnitudes in the halves, then the two sign bits (15, 31)
        uint32_t p[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int32_t x0 = v[s0 + 4 * i], x1 = v[s0 + 4 * i + 2];
            const uint32_t m = quant_mag<REV>(x0, inv, lim) | (quant_mag<REV>(x1, inv, lim) << 16);
            p[i] = (m | (((uint32_t)x0 >> 16) & 0x8000u)) | ((uint32_t)x1 & 0x80000000u);
        }
        uint16_t *d = (uint16_t *)q + e0;
        if (n == 8 && ((uintptr_t)d & 15) == 0) {
            *(uint4 *)d = make_uint4(p[0], p[1], p[2], p[3]);
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++)
                if (i < n) d[i] = (uint16_t)(p[i >> 1] >> (16 * (i & 1)));
        }
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) w[i] = quant_sm<REV>(v[s0 + 2 * i], inv, lim, 31);
        uint32_t *d = (uint32_t *)q + e0;
        if (n == 8 && ((uintptr_t)d & 15) == 0) {
            ((uint4 *)d)[0] = make_uint4(w[0], w[1], w[2], w[3]);
            ((uint4 *)d)[1] = make_uint4(w[4], w[5], w[6], w[7]);
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++)
                if (i < n) d[i] = w[i];
        }
    }
}

template <bool REV, int NROWS, typename RowFn>
__device__ __forceinline__ void hlift_write(int32_t *lds, int W, int ld, bool q16, RowFn rows) {
    const int tid = threadIdx.x;
    int32_t *base = lds + kPadL;
    if (W > 1) {
        const int nsteps = REV ? 2 : 4;
        for (int s = 0; s < nsteps; s++) {
            const int par = (s & 1) ? 0 : 1;
            const int cnt = par ? W / 2 : (W + 1) / 2;
            for (int r = 0; r < NROWS; r++) {
                QRow o;
                if (!rows(r, o)) continue;
                int32_t *row = base + r * ld;
                for (int j = tid; j < cnt; j += kDwtThreads) {
                    const int x = par + 2 * j;
                    const int l = x > 0 ? x - 1 : x + 1;
                    const int rr = x + 1 < W ? x + 1 : x - 1;
                    lift_update<REV>(row, x, l, rr, s);
                }
            }
            __syncthreads();
        }
    }
    // scale + de-interleave: consecutive threads write consecutive words
    const int nlh = (W + 1) / 2;
    for (int r = 0; r < NROWS; r++) {
        QRow o;
        if (!rows(r, o)) continue;
        const int32_t *row = base + r * ld;
        for (int j = tid; j < W; j += kDwtThreads) {
            const bool lo = j < nlh;
            const int x = lo ? 2 * j : 2 * (j - nlh) + 1;
            int32_t v = row[x];
            if (!REV && W > 1) v = __float_as_int(__int_as_float(v) * (lo ? INVK97 : K97));
            if (lo && o.ll) o.ll[j] = v;
            else store_q1<REV>(o.q, j, v, lo ? o.inv_lo : o.inv_hi, lo ? o.lim_lo : o.lim_hi, q16);
        }
    }
}

// Horizontal lifting without barriers: thread = (staged row, 16-sample
// segment), the segment's 16 samples plus a 4-sample halo on each side read
// from LDS into registers (six 16-byte reads), lifted there (the halo absorbs
// the 4-step footprint: the 16 kept samples are exact, as in lift_regs),
// scaled and written de-interleaved as 8 low + 8 high words (two 16-byte
// stores each when the row is aligned).  Rows as in hlift_write.
template <bool REV, int NROWS, bool ALIGNED, int NT = kDwtThreads, bool SKEW = false, typename RowFn>
__device__ __forceinline__ void hlift_seg(const int32_t *lds, int W, int ld, bool q16, RowFn rows,
                                          int nrows = NROWS) {
    const int nseg = (W + 15) >> 4;
    const int nlh = (W + 1) / 2;
    for (int it = threadIdx.x; it < nrows * nseg; it += NT) {
        const int r = it / nseg, k = it - r * nseg;
        const int x0 = (k << 4) - 4;  // window: samples x0 .. x0+23 (even start)
        int32_t v[24];
        if (SKEW) {  // segment k's samples at word 20 k: the halos are the neighbours' edges
            const int32_t *rb = lds + kPadLs + r * ld + 20 * k;
#pragma unroll
            for (int q = 0; q < 6; q++) {
                const int4 t = *(const int4 *)(rb + (q == 0 ? -8 : (q == 5 ? 20 : 4 * (q - 1))));
                v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
            }
        } else {
            const int4 *src = (const int4 *)(lds + kPadL + r * ld + x0);
#pragma unroll
            for (int q = 0; q < 6; q++) {
                const int4 t = src[q];
                v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
            }
        }
        if (ALIGNED) {  // caller: W > 1 and a multiple of 16
            // W a multiple of 16 (every full tile): the signal ends fall on
            // fixed window slots, so the symmetric extension is written into
            // the window (x = -i -> i, x = W-1+i -> W-1-i) and every segment
            // lifts the same straight-line code.  The lifting steps keep a
            // symmetric signal symmetric (commutative sums), so this equals
            // mirroring at every step, bit for bit.
            if (k == 0) {
                v[0] = v[8]; v[1] = v[7]; v[2] = v[6]; v[3] = v[5];
            }
            if (k == nseg - 1) {
                v[20] = v[18]; v[21] = v[17]; v[22] = v[16]; v[23] = v[15];
            }
            const int nsteps = REV ? 2 : 4;
#pragma unroll
            for (int st = 0; st < nsteps; st++) {
                const int par = (st & 1) ? 0 : 1;  // odd samples first
#pragma unroll
                for (int p = 1 + (par ^ 1); p < 23; p += 2) {
                    const int32_t l = v[p - 1], rr = v[p + 1];
                    if (REV) {
                        if (st == 0) v[p] -= (l + rr) >> 1;
                        else v[p] += (l + rr + 2) >> 2;
                    } else {
                        const float cf = st == 0 ? A97 : (st == 1 ? B97 : (st == 2 ? G97 : D97));
                        float t = __int_as_float(l) + __int_as_float(rr);
                        t = cf * t;
                        v[p] = __float_as_int(__int_as_float(v[p]) + t);
                    }
                }
            }
        } else if (W > 1) {
            const int pl = -x0;             // window slot of x = 0 (4 for segment 0)
            const int pr = W - 1 - x0;      // window slot of x = W-1
            const bool interior = x0 >= 0 && x0 + 24 <= W;
            const int nsteps = REV ? 2 : 4;
#pragma unroll
            for (int st = 0; st < nsteps; st++) {
                const int par = (st & 1) ? 0 : 1;  // odd samples first
#pragma unroll
                for (int p = 1 + (par ^ 1); p < 23; p += 2) {
                    int32_t l = v[p - 1], rr = v[p + 1];
                    if (!interior) {
                        if (p < pl || p > pr) continue;  // outside the signal
                        if (p == pl) l = v[p + 1];       // symmetric extension at x = 0
                        if (p == pr) rr = v[p - 1];      // ... and at x = W-1
                    }
                    if (REV) {
                        if (st == 0) v[p] -= (l + rr) >> 1;
                        else v[p] += (l + rr + 2) >> 2;
                    } else {
                        const float cf = st == 0 ? A97 : (st == 1 ? B97 : (st == 2 ? G97 : D97));
                        float t = __int_as_float(l) + __int_as_float(rr);
                        t = cf * t;
                        v[p] = __float_as_int(__int_as_float(v[p]) + t);
                    }
                }
            }
        }
        // the row's outputs, looked up only now (their registers are not held
        // through the lifting); a row that was not staged is lifted for
        // nothing and stores nothing
        QRow o;
        if (!rows(r, o)) continue;
        // slots 4..19 = samples k*16 .. k*16+15: even -> low j = x/2, odd -> high
        if (!REV && W > 1) {
#pragma unroll
            for (int q = 0; q < 8; q++) {
                v[4 + 2 * q] = __float_as_int(__int_as_float(v[4 + 2 * q]) * INVK97);
                v[5 + 2 * q] = __float_as_int(__int_as_float(v[5 + 2 * q]) * K97);
            }
        }
        const int j0 = k << 3;
        const int rem = W - (k << 4);  // samples of the row from this segment's first on
        const int nlo = min(8, (rem + 1) >> 1), nhi = min(8, rem >> 1);
        if (o.ll) {
            int32_t *ld_ = o.ll + j0;
            if (nlo == 8 && ((uintptr_t)ld_ & 15) == 0) {
                ((int4 *)ld_)[0] = make_int4(v[4], v[6], v[8], v[10]);
                ((int4 *)ld_)[1] = make_int4(v[12], v[14], v[16], v[18]);
            } else {
#pragma unroll
                for (int q = 0; q < 8; q++)
                    if (q < nlo) ld_[q] = v[4 + 2 * q];
            }
        } else {
            store_q8<REV>(o.q, j0, v, 4, nlo, o.inv_lo, o.lim_lo, q16);
        }
        store_q8<REV>(o.q, nlh + j0, v, 5, nhi, o.inv_hi, o.lim_hi, q16);
    }
}

template <bool REV, bool INGEST, int RB, int NT = kDwtThreads>
__global__ void __launch_bounds__(NT) k_dwt_band(DwtBandArgs a) {
    extern __shared__ int32_t lds[];
    constexpr int NR = RB + 2 * kDwtHalo;
    const int tc = blockIdx.y;
    const int sh = a.level - 1;
    const int W = (a.tc_w[tc] + (1 << sh) - 1) >> sh;
    const int H = (a.tc_h[tc] + (1 << sh) - 1) >> sh;
    const int r0 = blockIdx.x * RB;
    if (r0 >= H) return;
    const int nkeep = min(RB, H - r0);
    const int y0 = r0 - kDwtHalo;
    const int tid = threadIdx.x;
    const int ld = lds_row_stride(W);
    // ---- vertical: one column per thread, in registers ----
    for (int x = tid; x < W; x += NT) {
        int32_t v[NR];
        // every row load issues before any is used: rows outside the band
        // read a clamped (valid) row and are zeroed after (a load under a
        // per-row branch was waited for before the next one issued)
#pragma unroll
        for (int i = 0; i < NR; i++) v[i] = band_load<REV, INGEST>(a, tc, min(max(y0 + i, 0), H - 1), x);
#pragma unroll
        for (int i = 0; i < NR; i++) {
            const int y = y0 + i;
            v[i] = (y >= 0 && y < H) ? v[i] : 0;
        }
        if (H > 1) {
            lift_regs<REV, NR>(v, y0, H);
            if (!REV) {
#pragma unroll
                for (int i = kDwtHalo; i < kDwtHalo + RB; i++)
                    v[i] = __float_as_int(__int_as_float(v[i]) * ((i & 1) ? K97 : INVK97));
            }
        }
#pragma unroll
        for (int i = 0; i < RB; i++)
            if (i < nkeep) lds[kPadL + i * ld + x] = v[kDwtHalo + i];
    }
    __syncthreads();
    // ---- horizontal lifting, scaling and de-interleaved write ----
    const int nlv = (H + 1) / 2;
    int32_t *ll = a.ll ? (int32_t *)a.ll + (size_t)tc * a.ll_tc : nullptr;
    const bool q16 = a.qt.q16 != 0;
    const QLevel ql = qlevel(a.qt, a.level);
    auto rows = [&](int k, QRow &o) -> bool {
        if (k >= nkeep) return false;
        const int y = r0 + k;
        const bool ylo = (y & 1) == 0;
        o.q = qplane_row(a.dst, a.plane, tc, ylo ? (y >> 1) : nlv + (y >> 1), a.plane_w, q16);
        o.ll = (ylo && ll) ? ll + (size_t)(y >> 1) * a.ll_stride : nullptr;
        qrow_bands(o, ql, !ylo);
        return true;
    };
    if (W > 1 && (W & 15) == 0) hlift_seg<REV, RB, true, NT>(lds, W, ld, q16, rows);
    else hlift_seg<REV, RB, false, NT>(lds, W, ld, q16, rows);
}

// Level 1 with ingest, every component of a tile at once: a workgroup owns
// RB output rows of one tile; thread = column.  Each TIFF pixel of the band
// (+ halo) is read once for all its components -- the colour transform needs
// all three anyway -- instead of once per tile-component workgroup; the
// vertical lifting of each component runs in registers, the kept rows of all
// components go through LDS for the horizontal lifting, and the
// de-interleaved write puts HL/LH/HH in their final Mallat place and LL in the
// next level's scratch.  Same expressions as band_load / lift_regs /
// k_dwt_band (bit-exact with the oracle).
template <bool REV, int NC, int RB>
__global__ void __launch_bounds__(kDwtThreads) k_dwt_l1(DwtBandArgs a) {
    extern __shared__ int32_t lds[];
    constexpr int NR = RB + 2 * kDwtHalo;
    const int t = blockIdx.y;          // tile (part-local)
    const int tc0 = t * NC;
    const int W = a.tc_w[tc0], H = a.tc_h[tc0];
    const int r0 = blockIdx.x * RB;
    if (r0 >= H) return;
    const int nkeep = min(RB, H - r0);
    const int y0 = r0 - kDwtHalo;
    const int tid = threadIdx.x;
    const int ld = lds_row_stride(W);
    const int32_t off = 1 << (a.bits - 1);
    const size_t row_bytes = (size_t)a.img_w * (a.planar == 2 ? 1 : NC) * (a.bits >> 3);
    const int gx0 = (t % a.ntx) * a.tile_w, gy0 = a.row0 + (t / a.ntx) * a.tile_h;
    const bool mct = a.mct && NC >= 3;
    // byte offset of each window row (per component plane when planar):
    // wave-uniform, computed once per workgroup instead of per column
    uint64_t rowoff[NC][NR];
#pragma unroll
    for (int i = 0; i < NR; i++) {
        const int y = min(max(y0 + i, 0), H - 1);
        const int gy = gy0 + y;
        const int strip = gy / a.rps;
        const size_t ly = (size_t)(gy - strip * a.rps) * row_bytes;
#pragma unroll
        for (int c = 0; c < NC; c++)
            rowoff[c][i] = a.strip_off[a.planar == 2 ? (size_t)c * a.spp_strips + strip : (size_t)strip] + ly;
    }
    const int bps = a.bits >> 3;
    for (int x = tid; x < W; x += kDwtThreads) {
        int32_t v[NC][NR];
        const int gx = gx0 + x;
        const size_t xo = a.planar == 2 ? (size_t)gx * bps : (size_t)gx * NC * bps;
#pragma unroll
        for (int i = 0; i < NR; i++) {
            const int y = y0 + i;
            int32_t smp[NC];
            if (y >= 0 && y < H) {
#pragma unroll
                for (int c = 0; c < NC; c++) {
                    const uint8_t *p8 = a.tif + (a.planar == 2 ? rowoff[c][i] : rowoff[0][i] + (size_t)c * bps) + xo;
                    if (a.bits == 8) smp[c] = (int32_t)p8[0];
                    else smp[c] = a.big_endian ? (((int32_t)p8[0] << 8) | p8[1]) : (p8[0] | ((int32_t)p8[1] << 8));
                    smp[c] -= off;
                }
            } else {
#pragma unroll
                for (int c = 0; c < NC; c++) smp[c] = 0;
            }
#pragma unroll
            for (int c = 0; c < NC; c++) v[c][i] = REV ? smp[c] : __float_as_int((float)smp[c]);
            if constexpr (NC >= 3) if (mct) {
                if (REV) {
                    v[0][i] = (smp[0] + 2 * smp[1] + smp[2]) >> 2;
                    v[1][i] = smp[2] - smp[1];
                    v[2][i] = smp[0] - smp[1];
                } else {
                    const float R = (float)smp[0], G = (float)smp[1], B = (float)smp[2];
                    float f0 = 0.299f * R; f0 = f0 + 0.587f * G; f0 = f0 + 0.114f * B;
                    float f1 = -0.16875f * R; f1 = f1 - 0.33126f * G; f1 = f1 + 0.5f * B;
                    float f2 = 0.5f * R; f2 = f2 - 0.41869f * G; f2 = f2 - 0.08131f * B;
                    v[0][i] = __float_as_int(f0);
                    v[1][i] = __float_as_int(f1);
                    v[2][i] = __float_as_int(f2);
                }
            }
        }
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (H > 1) {
                lift_regs<REV, NR>(v[c], y0, H);
                if (!REV) {
#pragma unroll
                    for (int i = kDwtHalo; i < kDwtHalo + RB; i++)
                        v[c][i] = __float_as_int(__int_as_float(v[c][i]) * ((i & 1) ? K97 : INVK97));
                }
            }
#pragma unroll
            for (int i = 0; i < RB; i++)
                if (i < nkeep) lds[kPadL + (c * RB + i) * ld + x] = v[c][kDwtHalo + i];
        }
    }
    __syncthreads();
    // ---- horizontal lifting, scaling and de-interleaved write ----
    const int nlv = (H + 1) / 2;
    const bool q16 = a.qt.q16 != 0;
    const QLevel ql = qlevel(a.qt, a.level);
    hlift_write<REV, NC * RB>(lds, W, ld, q16, [&](int r, QRow &o) -> bool {
        const int c = r / RB, k = r - c * RB;
        if (k >= nkeep) return false;
        const int tc = tc0 + c, y = r0 + k;
        const bool ylo = (y & 1) == 0;
        o.q = qplane_row(a.dst, a.plane, tc, ylo ? (y >> 1) : nlv + (y >> 1), a.plane_w, q16);
        o.ll = (ylo && a.ll) ? (int32_t *)a.ll + (size_t)tc * a.ll_tc + (size_t)(y >> 1) * a.ll_stride : nullptr;
        qrow_bands(o, ql, !ylo);
        return true;
    });
}

// Level 1 with ingest, streaming: a workgroup owns a band of kStreamBand
// output rows of one tile (every component); thread = up to CPT columns.
// The vertical lifting runs as a pipeline down the band instead of over a
// window with a halo per 8 rows: at row pair (m-1, m) step k updates row
// m-1-k (k = 0..NS-1), after which rows m-NS and m-NS+1 are final, so each
// TIFF row is read and lifted once (plus NS rows above and below the band).
// Every 8 final rows go through LDS for the horizontal lifting and the
// de-interleaved write (hlift_write).  Each sample sees the same expressions
// in the same order as lift_regs / oracle fwd97_1d (bit-exact): an update
// whose neighbour lies outside the streamed rows is skipped, as lift_regs
// leaves a window's edge stale, and never reaches a kept row.
#ifndef JP2HIP_STREAM_BAND
#define JP2HIP_STREAM_BAND 64
#endif
constexpr int kStreamBand = JP2HIP_STREAM_BAND;
#ifndef JP2HIP_L1S_SKEW
#define JP2HIP_L1S_SKEW 1  // the skewed staging layout (hlift_seg's reads conflict-free)
#endif
constexpr bool kL1sSkew = JP2HIP_L1S_SKEW != 0;
#ifndef JP2HIP_L1S_PF
#define JP2HIP_L1S_PF 1  // row pairs fetched ahead (1, 2 or 3; 2 and 3 measured slower: profiles/r06/ab_l1s_prefetch.txt)
#endif
constexpr int kL1sPf = JP2HIP_L1S_PF;
static_assert(kL1sPf >= 1 && kL1sPf <= 3, "JP2HIP_L1S_PF: 1..3");
#ifndef JP2HIP_L1S_INTERIOR
#define JP2HIP_L1S_INTERIOR 0  // A/B: the select-free interior lifting path
#endif
#ifndef JP2HIP_L1S_R
#define JP2HIP_L1S_R 4  // rows per horizontal batch (4 or 8)
#endif
// (101 VGPRs, 4 waves per SIMD for the C2 variant; a budget for 5 --
// amdgpu_waves_per_eu(5), 5 VGPRs spilled -- measured no faster: 146.7 vs
// 146.4 us, profiles/r05/ab_select_fold.txt)
#ifndef JP2HIP_L1S_CENSUS
#define JP2HIP_L1S_CENSUS 0  // debug builds: shader cycles per phase of the row pipeline (output to stderr)
#endif
#if JP2HIP_L1S_CENSUS
__device__ unsigned long long g_l1s_census[8];  // phases 0..6, then waves
#define L1S_TICK(k)                                        \
    do {                                                   \
        __builtin_amdgcn_sched_barrier(0);                 \
        const uint64_t t_ = __builtin_readcyclecounter();  \
        cz[k] += t_ - tc;                                  \
        tc = t_;                                           \
        __builtin_amdgcn_sched_barrier(0);                 \
    } while (0)
#else
#define L1S_TICK(k) \
    do {            \
    } while (0)
#endif
template <bool REV, int NC, int CPT, int RB, bool ALIGNED>
__global__ void __launch_bounds__(kDwtThreads) k_dwt_l1s(DwtBandArgs a) {
#if JP2HIP_L1S_CENSUS
    uint64_t cz[7] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t tc = __builtin_readcyclecounter();
#endif
    extern __shared__ int32_t lds[];
    constexpr int NS = REV ? 2 : 4;  // lifting steps
    constexpr int NWIN = NS + 2;     // rows m-NS-1 .. m
    const int t = blockIdx.y;
    const int tc0 = t * NC;
    const int W = a.tc_w[tc0], H = a.tc_h[tc0];
    const int r0 = blockIdx.x * kStreamBand;
    // two launches cover the tiles: widths that are multiples of 16 (the
    // straight-line horizontal lifting) and the rest
    if (r0 >= H || ALIGNED != (W > 1 && (W & 15) == 0)) return;
    const int r1 = min(H, r0 + kStreamBand);
    const int s = max(0, r0 - NS), e = min(H, r1 + NS);  // rows streamed [s, e); s even
    const int tid = threadIdx.x;
    const int ld = kL1sSkew ? lds_row_stride_skew(W) : lds_row_stride(W);
    constexpr int kP = kL1sSkew ? kPadLs : kPadL;
    const int32_t off = 1 << (a.bits - 1);
    const int bps = a.bits >> 3;
    const size_t row_bytes = (size_t)a.img_w * (a.planar == 2 ? 1 : NC) * bps;
    const int gx0 = (t % a.ntx) * a.tile_w, gy0 = a.row0 + (t / a.ntx) * a.tile_h;
    const bool mct = a.mct && NC >= 3;
    // byte offset of every streamed row (per component plane when planar),
    // looked up once: a row fetch is then plain loads with no dependent
    // global read in front of them, so they stay in flight across the
    // lifting of the previous rows
    __shared__ uint64_t rowtab[(kStreamBand + 2 * 4) * NC];
    {
        const int ncp = a.planar == 2 ? NC : 1;
        for (int i = tid; i < (e - s) * ncp; i += kDwtThreads) {
            const int r = i / ncp, c = i - r * ncp;
            const int gy = gy0 + s + r;
            const int strip = gy / a.rps;
            rowtab[i] = a.strip_off[a.planar == 2 ? (size_t)c * a.spp_strips + strip : (size_t)strip] +
                        (size_t)(gy - strip * a.rps) * row_bytes;
        }
        __syncthreads();
    }
    int rnext = 0;  // next row to fetch, counted from s
    int32_t w[CPT][NC][NWIN];
#pragma unroll
    for (int j = 0; j < CPT; j++)
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int i = 0; i < NWIN; i++) w[j][c][i] = 0;
    // raw (level-shifted) samples of the next kL1sPf row pairs, fetched
    // ahead so the loads are in flight during the lifting of the rows before
    // them: row r (counted from s-1) lives in slot r % (2 kL1sPf)
    int32_t pf[2 * kL1sPf][CPT][NC];
    // raw sample bits only (a u8, or the u16 as stored): the level shift and
    // byte order wait for place(), so nothing uses a load until it is placed
    auto fetch = [&](int q) {  // the next row (s, s+1, ...) into pf[q]
        const int ncp = a.planar == 2 ? NC : 1;
        uint64_t ro[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) ro[c] = rowtab[rnext * ncp + (a.planar == 2 ? c : 0)];
        rnext++;
#pragma unroll
        for (int j = 0; j < CPT; j++) {
            const int x = min(tid + j * kDwtThreads, W - 1);  // columns past W repeat the last one
            const size_t xo = a.planar == 2 ? (size_t)(gx0 + x) * bps : (size_t)(gx0 + x) * NC * bps;
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const uint8_t *p8 = a.tif + (a.planar == 2 ? ro[c] : ro[0] + (size_t)c * bps) + xo;
                pf[q][j][c] = a.bits == 8 ? (int32_t)p8[0] : (int32_t)*(const uint16_t *)p8;
            }
        }
    };
    auto place = [&](int q, int slot) {  // colour transform, into window slot `slot`
#pragma unroll
        for (int j = 0; j < CPT; j++) {
            int32_t smp[NC];
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const uint32_t r = (uint32_t)pf[q][j][c];
                const int32_t v = (a.bits != 8 && a.big_endian) ? (int32_t)(((r & 0xFFu) << 8) | (r >> 8)) : (int32_t)r;
                smp[c] = v - off;
            }
#pragma unroll
            for (int c = 0; c < NC; c++) w[j][c][slot] = REV ? smp[c] : __float_as_int((float)smp[c]);
            if constexpr (NC >= 3) if (mct) {
                if (REV) {
                    w[j][0][slot] = (smp[0] + 2 * smp[1] + smp[2]) >> 2;
                    w[j][1][slot] = smp[2] - smp[1];
                    w[j][2][slot] = smp[0] - smp[1];
                } else {
                    const float R = (float)smp[0], G = (float)smp[1], B = (float)smp[2];
                    float f0 = 0.299f * R; f0 = f0 + 0.587f * G; f0 = f0 + 0.114f * B;
                    float f1 = -0.16875f * R; f1 = f1 - 0.33126f * G; f1 = f1 + 0.5f * B;
                    float f2 = 0.5f * R; f2 = f2 - 0.41869f * G; f2 = f2 - 0.08131f * B;
                    w[j][0][slot] = __float_as_int(f0);
                    w[j][1][slot] = __float_as_int(f1);
                    w[j][2][slot] = __float_as_int(f2);
                }
            }
        }
    };
    // rows s .. s + 2 kL1sPf - 2 ahead of the first iteration
    fetch(1);  // row s (iteration m = s takes rows s-1, s)
#pragma unroll
    for (int q = 2; q < 2 * kL1sPf; q++)
        if (s + q - 1 < e) fetch(q);
    const int nlv = (H + 1) / 2;
    const bool q16 = a.qt.q16 != 0;
    const QLevel ql = qlevel(a.qt, 1);
    int bb = r0;  // first row of the batch being filled
    // iteration m (even): rows m-1, m arrive; the last iteration emits row r1-1
    const int m_last = ((r1 - 1 + NS - 1) + 1) & ~1;
    // (the loop body is instantiated once per slot pair, so the prefetch
    // slots stay compile-time register indices)
    auto body = [&](int m, auto sa_c) {
        constexpr int SA = decltype(sa_c)::value, SB = SA + 1;
#pragma unroll
        for (int j = 0; j < CPT; j++)
#pragma unroll
            for (int c = 0; c < NC; c++)
#pragma unroll
                for (int i = 0; i + 2 < NWIN; i++) w[j][c][i] = w[j][c][i + 2];
        L1S_TICK(6);
        if (m - 1 >= s && m - 1 < e) place(SA, NWIN - 2);
        if (m < e) place(SB, NWIN - 1);
        L1S_TICK(0);
        if (m + 2 * kL1sPf - 1 < e) fetch(SA);
        if (m + 2 * kL1sPf < e) fetch(SB);
        L1S_TICK(1);
        // interior iterations (every step's rows and neighbours inside the
        // streamed rows and the signal, none at row 0): fixed neighbour slots,
        // no per-value selects -- the same expressions in the same order
        if (JP2HIP_L1S_INTERIOR && H > 1 && m - NS - 1 >= s && m < e) {
#pragma unroll
            for (int k = 0; k < NS; k++) {
                const int ti = NWIN - 2 - k;
#pragma unroll
                for (int j = 0; j < CPT; j++)
#pragma unroll
                    for (int c = 0; c < NC; c++) {
                        const int32_t lv = w[j][c][ti - 1], rv = w[j][c][ti + 1];
                        if (REV) {
                            if (k == 0) w[j][c][ti] -= (lv + rv) >> 1;
                            else w[j][c][ti] += (lv + rv + 2) >> 2;
                        } else {
                            const float cf = k == 0 ? A97 : (k == 1 ? B97 : (k == 2 ? G97 : D97));
                            float tt = __int_as_float(lv) + __int_as_float(rv);
                            tt = cf * tt;
                            w[j][c][ti] = __float_as_int(__int_as_float(w[j][c][ti]) + tt);
                        }
                    }
            }
        } else if (H > 1) {
#pragma unroll
            for (int k = 0; k < NS; k++) {
                const int tr = m - 1 - k, ti = NWIN - 2 - k;  // target row, its window slot
                if (tr < s || tr >= e) continue;
                // neighbours: window slots ti-1 / ti+1; symmetric extension at
                // rows 0 and H-1; a neighbour outside the streamed rows -> skip
                int li = ti - 1, ri = ti + 1;
                if (tr == 0) li = ti + 1;
                else if (tr - 1 < s) continue;
                if (tr + 1 >= H) ri = ti - 1;
                else if (tr + 1 >= e) continue;
#pragma unroll
                for (int j = 0; j < CPT; j++)
#pragma unroll
                    for (int c = 0; c < NC; c++) {
                        // constant slots after unrolling: select among the few candidates
                        const int32_t lv = li == ti - 1 ? w[j][c][ti - 1] : w[j][c][ti + 1];
                        const int32_t rv = ri == ti + 1 ? w[j][c][ti + 1] : w[j][c][ti - 1];
                        if (REV) {
                            if (k == 0) w[j][c][ti] -= (lv + rv) >> 1;
                            else w[j][c][ti] += (lv + rv + 2) >> 2;
                        } else {
                            const float cf = k == 0 ? A97 : (k == 1 ? B97 : (k == 2 ? G97 : D97));
                            float tt = __int_as_float(lv) + __int_as_float(rv);
                            tt = cf * tt;
                            w[j][c][ti] = __float_as_int(__int_as_float(w[j][c][ti]) + tt);
                        }
                    }
            }
        }
        L1S_TICK(2);
        // rows m-NS (even) and m-NS+1 (odd) are final: scale, stage in LDS
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int y = m - NS + q;
            if (y < r0 || y >= r1) continue;
#pragma unroll
            for (int j = 0; j < CPT; j++) {
                const int x = tid + j * kDwtThreads;
                if (x >= W) continue;
#pragma unroll
                for (int c = 0; c < NC; c++) {
                    int32_t v = w[j][c][1 + q];
                    if (!REV && H > 1) v = __float_as_int(__int_as_float(v) * (q ? K97 : INVK97));
                    lds[kP + (c * RB + (y - bb)) * ld + (kL1sSkew ? skew_x(x) : x)] = v;
                }
            }
        }
        const int ylast = m - NS + 1;
        L1S_TICK(3);
        if (ylast >= r0 && (ylast - bb == RB - 1 || ylast >= r1 - 1)) {
            __syncthreads();
            L1S_TICK(4);
            const int nkeep = min(RB, r1 - bb);
            hlift_seg<REV, NC * RB, ALIGNED, kDwtThreads, kL1sSkew>(lds, W, ld, q16, [&](int r, QRow &o) -> bool {
                const int c = r / RB, k = r - c * RB;
                if (k >= nkeep) return false;
                const int tc = tc0 + c, y = bb + k;
                const bool ylo = (y & 1) == 0;
                o.q = qplane_row(a.dst, a.plane, tc, ylo ? (y >> 1) : nlv + (y >> 1), a.plane_w, q16);
                o.ll = (ylo && a.ll) ? (int32_t *)a.ll + (size_t)tc * a.ll_tc + (size_t)(y >> 1) * a.ll_stride
                                     : nullptr;
                qrow_bands(o, ql, !ylo);
                return true;
            });
            L1S_TICK(5);
            __syncthreads();
            L1S_TICK(4);
            bb += RB;
        }
    };
    for (int m = s; m <= m_last; m += 2) {
        if (kL1sPf == 1 || (((m - s) >> 1) % kL1sPf) == 0) body(m, std::integral_constant<int, 0>{});
        else if (kL1sPf >= 2 && (((m - s) >> 1) % kL1sPf) == 1) body(m, std::integral_constant<int, (kL1sPf >= 2 ? 2 : 0)>{});
        else if (kL1sPf >= 3 && (((m - s) >> 1) % kL1sPf) == 2) body(m, std::integral_constant<int, (kL1sPf >= 3 ? 4 : 0)>{});
    }
#if JP2HIP_L1S_CENSUS
    if ((tid & 63) == 0) {  // per wave: vector atomics on a global word
        for (int k = 0; k < 7; k++) atomicAdd(&g_l1s_census[k], (unsigned long long)cz[k]);
        atomicAdd(&g_l1s_census[7], 1ull);
    }
#endif
}

struct DwtTailArgs {
    const void *src;      // LL of level `level`-1, compact scratch planes
    int src_stride;
    size_t src_tc;
    void *dst;
    int plane_w;
    size_t plane;
    const int32_t *tc_w, *tc_h;
    int level, levels;
    QuantTab qt;
};

// Levels level..levels of one tile-component, entirely in LDS, with the
// band kernels' window lifting (each level two barrier-separated passes
// instead of one barrier per lifting step):
//   vertical   thread = (column, group of kTailRG rows): the group plus a
//              4-row halo on each side read into registers, lifted there
//              (lift_regs: the halo absorbs the lifting footprint, the kept
//              rows are exact), scaled, written to the padded row layout
//              hlift_seg reads;
//   horizontal hlift_seg over every row (16-sample segments with halos in
//              registers), high bands (and the last level's LL) straight to
//              HBM, a non-final LL densely into `ll` for the next level.
// The level's input is dense (row stride = its width): the LL scratch of the
// previous level, then `ll`.  Same expressions in the same order as the
// oracle (bit-exact).
// The tail starts at the first level of <= 64 x 64 samples (the recipe's
// 512^2 and 1024^2 tiles reach it at levels 4 and 5): a workgroup of 256
// threads and 21 KB of LDS.  Sized for 128 x 128 levels it took 1 024
// threads and 82 KB -- half a CU -- and under the bench's load such a
// workgroup waited ~1.5 ms for a CU to free that much (C2 bench +7-9 %).
constexpr int kTailThreads = 256;
constexpr int kTailRG = 16;                                  // rows per vertical item
constexpr int kTailWords = 4096 + 64 * 4 + kPadL + kPadR;    // padded rows of a <= 64 x 64 level
constexpr int kTailLL = 1024;                                // the LL of a <= 64 x 64 level
template <bool REV>
__global__ void __launch_bounds__(kTailThreads) k_dwt_tail(DwtTailArgs a) {
    __shared__ __attribute__((aligned(16))) int32_t rows_[kTailWords];  // vertical output, padded rows
    __shared__ int32_t ll[kTailLL];                                      // the next level's input (dense)
    const int tc = blockIdx.x, tid = threadIdx.x;
    int sh = a.level - 1;
    int W = (a.tc_w[tc] + (1 << sh) - 1) >> sh;
    int H = (a.tc_h[tc] + (1 << sh) - 1) >> sh;
    // the first level reads the previous level's LL scratch in HBM directly,
    // later levels the LL the previous one left in `ll` (two inlined copies of
    // the vertical pass, so each knows its address space)
    const int32_t *g_src = (const int32_t *)a.src + (size_t)tc * a.src_tc;
    const bool q16 = a.qt.q16 != 0;
    constexpr int NR = kTailRG + 2 * kDwtHalo;
    for (int lv = a.level; lv <= a.levels; lv++) {
        const int ld = lds_row_stride(W);
        // ---- vertical: column x, rows [g * kTailRG, +kTailRG) ----
        auto vertical = [&](const int32_t *srcp, int sstride) {
            const int ngrp = (H + kTailRG - 1) / kTailRG;
            for (int it = tid; it < W * ngrp; it += kTailThreads) {
                const int g = it / W, x = it - g * W;
                const int r0 = g * kTailRG, y0 = r0 - kDwtHalo;
                int32_t v[NR];
                // every row load issues before any is used (clamped rows, zeroed after)
#pragma unroll
                for (int i = 0; i < NR; i++) v[i] = srcp[min(max(y0 + i, 0), H - 1) * sstride + x];
#pragma unroll
                for (int i = 0; i < NR; i++) {
                    const int y = y0 + i;
                    v[i] = (y >= 0 && y < H) ? v[i] : 0;
                }
                if (H > 1) {
                    lift_regs<REV, NR>(v, y0, H);
                    if (!REV) {
#pragma unroll
                        for (int i = kDwtHalo; i < kDwtHalo + kTailRG; i++)
                            v[i] = __float_as_int(__int_as_float(v[i]) * ((i & 1) ? K97 : INVK97));
                    }
                }
#pragma unroll
                for (int i = 0; i < kTailRG; i++)
                    if (r0 + i < H) rows_[kPadL + (r0 + i) * ld + x] = v[kDwtHalo + i];
            }
        };
        if (lv == a.level) vertical(g_src, a.src_stride);
        else vertical(ll, W);
        __syncthreads();
        // ---- horizontal lifting, scaling, de-interleaved write ----
        const int nlv = (H + 1) / 2;
        const bool last = lv == a.levels;
        const int nlh = (W + 1) / 2;
        const QLevel ql = qlevel(a.qt, lv);
        auto rowfn = [&](int y, QRow &o) -> bool {
            const bool ylo = (y & 1) == 0;
            o.q = qplane_row(a.dst, a.plane, tc, ylo ? (y >> 1) : nlv + (y >> 1), a.plane_w, q16);
            o.ll = (ylo && !last) ? ll + (y >> 1) * nlh : nullptr;
            qrow_bands(o, ql, !ylo);
            return true;
        };
        if (W > 1 && (W & 15) == 0) hlift_seg<REV, 0, true, kTailThreads>(rows_, W, ld, q16, rowfn, H);
        else if (W > 1) hlift_seg<REV, 0, false, kTailThreads>(rows_, W, ld, q16, rowfn, H);
        else {  // one column: no horizontal transform (the LL is the column itself)
            for (int y = tid; y < H; y += kTailThreads) {
                QRow o;
                rowfn(y, o);
                const int32_t v = rows_[kPadL + y * ld];
                if (o.ll) o.ll[0] = v;
                else store_q1<REV>(o.q, 0, v, o.inv_lo, o.lim_lo, q16);
            }
        }
        if (last) break;
        __syncthreads();
        W = nlh;
        H = nlv;
    }
}

template <bool REV, bool INGEST, int RB, int NT>
static void launch_band(dim3 g, size_t lds, hipStream_t st, const DwtBandArgs &a) {
    static bool wide = false;  // opt in to > 64 KiB dynamic LDS once per instance
    if (lds > (size_t)kDwtLdsWords * 4 && !wide) {
        (void)hipFuncSetAttribute((const void *)k_dwt_band<REV, INGEST, RB, NT>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kDwtLdsWordsWide * 4);
        wide = true;
    }
    hipLaunchKernelGGL((k_dwt_band<REV, INGEST, RB, NT>), g, dim3(NT), lds, st, a);
}
#ifndef JP2HIP_BAND_RB
#define JP2HIP_BAND_RB 16
#endif
#ifndef JP2HIP_BAND_NARROW
#define JP2HIP_BAND_NARROW 128  // levels at most this wide: workgroups of this many threads
#endif
constexpr int kBandRb = JP2HIP_BAND_RB;
// (a level of <= 128 columns in 128-thread workgroups: with 256 threads half
// of them had no column)
template <bool REV, bool INGEST>
static void launch_band_rb(int maxW, dim3 g, size_t lds, hipStream_t st, const DwtBandArgs &a) {
    if (!INGEST && JP2HIP_BAND_NARROW < kDwtThreads && maxW <= JP2HIP_BAND_NARROW)
        launch_band<REV, INGEST, kBandRb, (JP2HIP_BAND_NARROW < kDwtThreads ? JP2HIP_BAND_NARROW : kDwtThreads)>(
            g, lds, st, a);
    else
        launch_band<REV, INGEST, kBandRb, kDwtThreads>(g, lds, st, a);
}

template <bool REV, int NC>
static void launch_l1_nc(dim3 g, size_t lds, hipStream_t st, const DwtBandArgs &a) {
    static bool wide = false;
    if (lds > (size_t)kDwtLdsWords * 4 && !wide) {
        (void)hipFuncSetAttribute((const void *)k_dwt_l1<REV, NC, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kDwtLdsWordsWide * 4);
        wide = true;
    }
    hipLaunchKernelGGL((k_dwt_l1<REV, NC, 8>), g, dim3(kDwtThreads), lds, st, a);
}
template <bool REV, int NC, int CPT, int RB>
static void launch_l1s_rb(dim3 g, size_t lds, hipStream_t st, const DwtBandArgs &a) {
    static bool wide = false;
    if (lds > (size_t)kDwtLdsWords * 4 && !wide) {
        (void)hipFuncSetAttribute((const void *)k_dwt_l1s<REV, NC, CPT, RB, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kDwtLdsWordsWide * 4);
        (void)hipFuncSetAttribute((const void *)k_dwt_l1s<REV, NC, CPT, RB, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kDwtLdsWordsWide * 4);
        wide = true;
    }
    hipLaunchKernelGGL((k_dwt_l1s<REV, NC, CPT, RB, true>), g, dim3(kDwtThreads), lds, st, a);
    if (a.ragged) hipLaunchKernelGGL((k_dwt_l1s<REV, NC, CPT, RB, false>), g, dim3(kDwtThreads), lds, st, a);
#if JP2HIP_L1S_CENSUS
    unsigned long long h[8];
    if (hipStreamSynchronize(st) == hipSuccess &&
        hipMemcpyFromSymbol(h, HIP_SYMBOL(g_l1s_census), sizeof h) == hipSuccess && h[7]) {
        fprintf(stderr, "l1s census: waves %llu, cycles per wave: place %.0f fetch %.0f vlift %.0f stage %.0f "
                        "barriers %.0f hlift %.0f loop %.0f\n", h[7], (double)h[0] / h[7], (double)h[1] / h[7],
                (double)h[2] / h[7], (double)h[3] / h[7], (double)h[4] / h[7], (double)h[5] / h[7],
                (double)h[6] / h[7]);
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_l1s_census), z, sizeof z);
    }
#endif
}
template <bool REV, int NC, int CPT>
static void launch_l1s_c(dim3 g, size_t lds, hipStream_t st, const DwtBandArgs &a) {
    if (a.R == 8) launch_l1s_rb<REV, NC, CPT, 8>(g, lds, st, a);
    else launch_l1s_rb<REV, NC, CPT, 4>(g, lds, st, a);
}
template <bool REV, int NC>
static void launch_l1s_nc(int cpt, dim3 g, size_t lds, hipStream_t st, const DwtBandArgs &a) {
    if (cpt == 1) launch_l1s_c<REV, NC, 1>(g, lds, st, a);
    else if (cpt == 2) launch_l1s_c<REV, NC, 2>(g, lds, st, a);
    else launch_l1s_c<REV, NC, 4>(g, lds, st, a);
}
template <bool REV>
static void launch_l1s(int nc, int cpt, dim3 g, size_t lds, hipStream_t st, const DwtBandArgs &a) {
    if (nc == 1) launch_l1s_nc<REV, 1>(cpt, g, lds, st, a);
    else if (nc == 2) launch_l1s_nc<REV, 2>(cpt, g, lds, st, a);
    else if (nc == 3) launch_l1s_nc<REV, 3>(cpt, g, lds, st, a);
    else launch_l1s_nc<REV, 4>(cpt, g, lds, st, a);
}
template <bool REV>
static void launch_l1(int nc, dim3 g, size_t lds, hipStream_t st, const DwtBandArgs &a) {
    if (nc == 1) launch_l1_nc<REV, 1>(g, lds, st, a);
    else if (nc == 2) launch_l1_nc<REV, 2>(g, lds, st, a);
    else if (nc == 3) launch_l1_nc<REV, 3>(g, lds, st, a);
    else launch_l1_nc<REV, 4>(g, lds, st, a);
}

// Ingest + all DWT levels on `st`.  Returns false on a launch error.
bool launch_dwt(const DwtLaunch &p, hipStream_t st) {
    DwtBandArgs a;
    a.tif = (const uint8_t *)p.tif;
    a.strip_off = p.strip_off;
    a.rps = p.rps; a.img_w = p.img_w; a.nc = p.nc; a.bits = p.bits; a.planar = p.planar;
    a.big_endian = p.big_endian; a.mct = p.mct; a.spp_strips = p.spp_strips;
    a.ntx = p.ntx; a.tile_w = p.tile_w; a.tile_h = p.tile_h; a.row0 = p.row0;
    a.dst = p.coef;
    a.qt = p.qt;
    a.plane_w = p.plane_w;
    a.plane = (size_t)p.plane_w * p.plane_h;
    a.tc_w = p.tc_w; a.tc_h = p.tc_h;
    a.ragged = (p.tile_w & 15) || (p.last_tile_w & 15) || p.last_tile_w == 1;
    const int ll_stride = (p.plane_w + 1) / 2;
    const size_t ll_tc = (size_t)ll_stride * ((p.plane_h + 1) / 2);
    void *scratch[2] = {p.scratch0, p.scratch1};
    for (int lv = 1; lv <= p.levels; lv++) {
        const int maxW = (p.plane_w + (1 << (lv - 1)) - 1) >> (lv - 1);
        const int maxH = (p.plane_h + (1 << (lv - 1)) - 1) >> (lv - 1);
        if (lv >= 2 && ((maxW + 1) / 2) * ((maxH + 1) / 2) <= kTailLL &&
            lds_row_stride(maxW) * maxH + kPadL + kPadR <= kTailWords) {
            DwtTailArgs t;
            t.src = scratch[(lv - 1) & 1];
            t.src_stride = ll_stride;
            t.src_tc = ll_tc;
            t.dst = p.coef;
            t.plane_w = p.plane_w;
            t.plane = a.plane;
            t.tc_w = p.tc_w; t.tc_h = p.tc_h;
            t.level = lv; t.levels = p.levels;
            t.qt = p.qt;
            if (p.reversible) hipLaunchKernelGGL(k_dwt_tail<true>, dim3(p.ntc), dim3(kTailThreads), 0, st, t);
            else hipLaunchKernelGGL(k_dwt_tail<false>, dim3(p.ntc), dim3(kTailThreads), 0, st, t);
            return hipGetLastError() == hipSuccess;
        }
        const int R = kBandRb;  // kept rows per workgroup (16: 8 took 2 x 40 us for levels 2-3, 16 70 us, profiles/r04/ab_dwt_band.txt)
        a.level = lv;
        a.R = R;
        a.src = scratch[(lv - 1) & 1];
        a.src_stride = ll_stride;
        a.src_tc = ll_tc;
        a.ll = lv == p.levels ? nullptr : scratch[lv & 1];
        a.ll_stride = ll_stride;
        a.ll_tc = ll_tc;
        const size_t lds = ((size_t)R * lds_row_stride(maxW) + kPadL + kPadR) * 4;
        dim3 g((maxH + R - 1) / R, p.ntc);
        // level 1: every component of a tile in one workgroup when its rows
        // fit in LDS (each TIFF pixel read once)
        constexpr int kRb1 = 8;
        const size_t lds1 = ((size_t)p.nc * kRb1 * lds_row_stride(maxW) + kPadL + kPadR) * 4;
        const int cpt = maxW <= kDwtThreads ? 1 : (maxW <= 2 * kDwtThreads ? 2 : 4);
        if (lv == 1 && lds1 <= (size_t)kDwtLdsWordsWide * 4 && maxW <= 4 * kDwtThreads) {
            // streaming vertical pass (k_dwt_l1s), bands of kStreamBand rows,
            // horizontal batches of 4 rows
            a.R = JP2HIP_L1S_R;
            const size_t lds_s =
                ((size_t)p.nc * a.R * (kL1sSkew ? lds_row_stride_skew(maxW) : lds_row_stride(maxW)) +
                 (kL1sSkew ? kPadLs : kPadL) + kPadR) * 4;
            dim3 g1((maxH + kStreamBand - 1) / kStreamBand, p.ntc / p.nc);
            if (p.reversible) launch_l1s<true>(p.nc, cpt, g1, lds_s, st, a);
            else launch_l1s<false>(p.nc, cpt, g1, lds_s, st, a);
        } else if (lv == 1 && lds1 <= (size_t)kDwtLdsWordsWide * 4) {
            dim3 g1((maxH + kRb1 - 1) / kRb1, p.ntc / p.nc);
            if (p.reversible) launch_l1<true>(p.nc, g1, lds1, st, a);
            else launch_l1<false>(p.nc, g1, lds1, st, a);
        } else if (lv == 1) {
            if (p.reversible) launch_band_rb<true, true>(maxW, g, lds, st, a);
            else launch_band_rb<false, true>(maxW, g, lds, st, a);
        } else {
            if (p.reversible) launch_band_rb<true, false>(maxW, g, lds, st, a);
            else launch_band_rb<false, false>(maxW, g, lds, st, a);
        }
        if (hipGetLastError() != hipSuccess) return false;
    }
    return true;
}

}  // namespace jp2hip
