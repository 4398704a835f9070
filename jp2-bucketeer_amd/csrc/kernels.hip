// kernels.hip -- the gfx950 encode path of libjp2hip.
//
// Stage map (reference stage: kdu_compress invoked at
// KakaduConverter.java:61-71):
//   k_ingest     S1+S2  TIFF strips in HBM -> tile-component planes, level
//                       shift, RCT (int) / ICT (fp32)
//   k_dwt_vert   S3     one decomposition level, columns (LDS strip)
//   k_dwt_horz   S3     one decomposition level, rows (LDS rows)
//   k_quant      S4     deadzone quantiser + bit-plane masks via wave ballot
//   k_t1         S5     EBCOT tier-1 + MQ coder, one lane per code-block,
//                       bit-parallel (64-bit row mask) context modelling
//   k_hull/k_select S6  PCRD-opt convex hulls + global slope thresholds
//   k_compact           gather the included bytes for the D2H copy
// Tier-2 (S7/S8) runs on host threads (t2.cpp).
//
// Floating point: built with -ffp-contract=off; every 9/7 / ICT expression is
// written in the same order as the oracle so the lossy path is bit-exact.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gpu_encoder.h"

namespace jp2hip {

#define HIPCHECK(x)                                                                    \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            err = std::string(#x) + ": " + hipGetErrorString(e_);                      \
            return false;                                                              \
        }                                                                              \
    } while (0)

// --------------------------------------------------------------------------
// S1 + S2: ingest
// --------------------------------------------------------------------------
struct IngestArgs {
    const uint8_t *src;
    const uint64_t *strip_off;
    int rps, w, h, nc, bits, planar, big_endian, mct, reversible;
    int ntx, tile_w, tile_h, plane_w, plane_h, spp_strips;  // strips per plane
    void *coef;
};

__device__ __forceinline__ int32_t read_sample(const IngestArgs &a, int x, int y, int c) {
    int strip = y / a.rps;
    size_t off;
    if (a.planar == 2) {
        off = a.strip_off[(size_t)c * a.spp_strips + strip] +
              ((size_t)(y - strip * a.rps) * a.w + x) * (a.bits >> 3);
    } else {
        off = a.strip_off[strip] + (((size_t)(y - strip * a.rps) * a.w + x) * a.nc + c) * (a.bits >> 3);
    }
    if (a.bits == 8) return (int32_t)a.src[off];
    uint32_t b0 = a.src[off], b1 = a.src[off + 1];
    return (int32_t)(a.big_endian ? ((b0 << 8) | b1) : (b0 | (b1 << 8)));
}

__global__ void __launch_bounds__(256) k_ingest(IngestArgs a) {
    int x = blockIdx.x * 64 + (threadIdx.x & 63);
    int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= a.w || y >= a.h) return;
    int32_t off = 1 << (a.bits - 1);
    int32_t s[4];
#pragma unroll
    for (int c = 0; c < 4; c++) s[c] = (c < a.nc) ? read_sample(a, x, y, c) - off : 0;
    int tx = x / a.tile_w, ty = y / a.tile_h;
    size_t plane = (size_t)a.plane_w * a.plane_h;
    size_t base = ((size_t)(ty * a.ntx + tx) * a.nc) * plane + (size_t)(y - ty * a.tile_h) * a.plane_w +
                  (x - tx * a.tile_w);
    bool domct = a.mct && a.nc >= 3;
    if (a.reversible) {
        int32_t *o = (int32_t *)a.coef;
        int32_t v[4] = {s[0], s[1], s[2], s[3]};
        if (domct) {
            v[0] = (s[0] + 2 * s[1] + s[2]) >> 2;
            v[1] = s[2] - s[1];
            v[2] = s[0] - s[1];
        }
#pragma unroll
        for (int c = 0; c < 4; c++)
            if (c < a.nc) o[base + (size_t)c * plane] = v[c];
    } else {
        float *o = (float *)a.coef;
        float f[4] = {(float)s[0], (float)s[1], (float)s[2], (float)s[3]};
        if (domct) {
            float R = f[0], G = f[1], B = f[2];
            float y0 = 0.299f * R; y0 = y0 + 0.587f * G; y0 = y0 + 0.114f * B;
            float cb = -0.16875f * R; cb = cb - 0.33126f * G; cb = cb + 0.5f * B;
            float cr = 0.5f * R; cr = cr - 0.41869f * G; cr = cr - 0.08131f * B;
            f[0] = y0; f[1] = cb; f[2] = cr;
        }
#pragma unroll
        for (int c = 0; c < 4; c++)
            if (c < a.nc) o[base + (size_t)c * plane] = f[c];
    }
}

// --------------------------------------------------------------------------
// S3: DWT.  Lifting per Annex F; symmetric extension; even start everywhere.
// --------------------------------------------------------------------------
#define A97 (-1.586134342059924f)
#define B97 (-0.052980118572961f)
#define G97 (0.882911075530934f)
#define D97 (0.443506852043971f)
#define K97 (1.230174104914001f)
#define INVK97 (0.8128930661159609f)

// In-LDS lifting over n samples at x[i*stride], executed by `nthr` threads
// with thread index t; `lines` independent signals at base offsets line*lstride.
template <bool REV>
__device__ __forceinline__ void lift_lines(void *buf, int n, int lines, int stride, int lstride,
                                           int t, int nthr) {
    if (n < 2) return;
    int nodd = n / 2, neven = (n + 1) / 2;
    if (REV) {
        int32_t *x = (int32_t *)buf;
        for (int it = t; it < nodd * lines; it += nthr) {
            int line = it / nodd, i = 2 * (it - line * nodd) + 1;
            int32_t *p = x + line * lstride;
            int32_t l = p[(i - 1) * stride], r = (i + 1 < n) ? p[(i + 1) * stride] : l;
            p[i * stride] -= (l + r) >> 1;
        }
        __syncthreads();
        for (int it = t; it < neven * lines; it += nthr) {
            int line = it / neven, i = 2 * (it - line * neven);
            int32_t *p = x + line * lstride;
            int32_t l = (i > 0) ? p[(i - 1) * stride] : p[(i + 1) * stride];
            int32_t r = (i + 1 < n) ? p[(i + 1) * stride] : p[(i - 1) * stride];
            p[i * stride] += (l + r + 2) >> 2;
        }
        __syncthreads();
    } else {
        float *x = (float *)buf;
        const float coef[4] = {A97, B97, G97, D97};
#pragma unroll
        for (int step = 0; step < 4; step++) {
            bool odd = (step & 1) == 0;
            int cnt = odd ? nodd : neven;
            float cf = coef[step];
            for (int it = t; it < cnt * lines; it += nthr) {
                int line = it / cnt, j = it - line * cnt;
                int i = odd ? 2 * j + 1 : 2 * j;
                float *p = x + line * lstride;
                float l = (i > 0) ? p[(i - 1) * stride] : p[(i + 1) * stride];
                float r = (i + 1 < n) ? p[(i + 1) * stride] : p[(i - 1) * stride];
                float tt = l + r;
                tt = cf * tt;
                p[i * stride] = p[i * stride] + tt;
            }
            __syncthreads();
        }
    }
}

struct DwtArgs {
    void *coef;
    const int32_t *tc_w, *tc_h;
    int plane_w, plane_h, level;  // level d >= 1 being produced
    int cw;                       // columns per strip (vertical kernel)
};

// Columns: one workgroup = `cw` columns x all rows of the current region.
template <bool REV>
__global__ void __launch_bounds__(256) k_dwt_vert(DwtArgs a) {
    extern __shared__ int32_t lds[];
    int tc = blockIdx.y;
    int sh = a.level - 1;
    int W = (a.tc_w[tc] + (1 << sh) - 1) >> sh, H = (a.tc_h[tc] + (1 << sh) - 1) >> sh;
    int x0 = blockIdx.x * a.cw;
    if (x0 >= W) return;
    int ncol = min(a.cw, W - x0);
    int ld = a.cw + 1;
    int32_t *g = (int32_t *)a.coef + (size_t)tc * a.plane_w * a.plane_h + x0;
    for (int it = threadIdx.x; it < H * a.cw; it += blockDim.x) {
        int y = it / a.cw, c = it - y * a.cw;
        if (c < ncol) lds[y * ld + c] = g[(size_t)y * a.plane_w + c];
    }
    __syncthreads();
    lift_lines<REV>(lds, H, ncol, ld, 1, threadIdx.x, blockDim.x);
    int nl = (H + 1) / 2;
    for (int it = threadIdx.x; it < H * a.cw; it += blockDim.x) {
        int y = it / a.cw, c = it - y * a.cw;
        if (c >= ncol) continue;
        int src = (y < nl) ? 2 * y : 2 * (y - nl) + 1;
        int32_t v = lds[src * ld + c];
        if (!REV && H > 1) {
            float f = __int_as_float(v);
            f = (y < nl) ? f * INVK97 : f * K97;
            v = __float_as_int(f);
        }
        g[(size_t)y * a.plane_w + c] = v;
    }
}

// Rows: one workgroup = 4 rows of the current region.
template <bool REV>
__global__ void __launch_bounds__(256) k_dwt_horz(DwtArgs a) {
    extern __shared__ int32_t lds[];
    constexpr int ROWS = 4;
    int tc = blockIdx.y;
    int sh = a.level - 1;
    int W = (a.tc_w[tc] + (1 << sh) - 1) >> sh, H = (a.tc_h[tc] + (1 << sh) - 1) >> sh;
    int y0 = blockIdx.x * ROWS;
    if (y0 >= H) return;
    int nrow = min(ROWS, H - y0);
    int ld = W + 1;
    int32_t *g = (int32_t *)a.coef + (size_t)tc * a.plane_w * a.plane_h + (size_t)y0 * a.plane_w;
    for (int it = threadIdx.x; it < nrow * W; it += blockDim.x) {
        int r = it / W, x = it - r * W;
        lds[r * ld + x] = g[(size_t)r * a.plane_w + x];
    }
    __syncthreads();
    lift_lines<REV>(lds, W, nrow, 1, ld, threadIdx.x, blockDim.x);
    int nl = (W + 1) / 2;
    for (int it = threadIdx.x; it < nrow * W; it += blockDim.x) {
        int r = it / W, x = it - r * W;
        int src = (x < nl) ? 2 * x : 2 * (x - nl) + 1;
        int32_t v = lds[r * ld + src];
        if (!REV && W > 1) {
            float f = __int_as_float(v);
            f = (x < nl) ? f * INVK97 : f * K97;
            v = __float_as_int(f);
        }
        g[(size_t)r * a.plane_w + x] = v;
    }
}

// --------------------------------------------------------------------------
// Distortion bookkeeping (identical integer definition in the oracle):
// squared error in half-units of mid-point reconstruction from plane p up.
// --------------------------------------------------------------------------
__device__ __forceinline__ int64_t dist_at(uint32_t v, int p, bool lossless) {
    int64_t t2 = 2 * (int64_t)v + (lossless ? 0 : 1);
    int64_t r2 = 0;
    if ((v >> p) != 0) {
        r2 = 2 * (int64_t)((v >> p) << p);
        if (!(lossless && p == 0)) r2 += (int64_t)1 << p;
    }
    int64_t e = t2 - r2;
    return e * e;
}
__device__ __forceinline__ int64_t dist_gain(uint32_t v, int p, bool lossless) {
    return dist_at(v, p + 1, lossless) - dist_at(v, p, lossless);
}

__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        int lo = __shfl_xor((int)(uint32_t)v, o, 64);
        int hi = __shfl_xor((int)(uint32_t)((uint64_t)v >> 32), o, 64);
        v += (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
    }
    return v;
}

// --------------------------------------------------------------------------
// S4: quantisation + bit-planes.  One wavefront per code-block; lane = column.
// Layout per block (uint64 words): B[p][64 rows] for p < Mb, then
// S[p][64 rows] = OR_{q>=p} B[q], then sign[64 rows].
// --------------------------------------------------------------------------
struct QuantArgs {
    const BlockDesc *blocks;
    const void *coef;
    int plane_w, plane_h, reversible;
    uint64_t *bp;
    int32_t *sm;
    uint8_t *P;
    int64_t *dref, *dsig;  // [block][32]
};

__global__ void __launch_bounds__(64) k_quant(QuantArgs a) {
    int b = blockIdx.x;
    BlockDesc d = a.blocks[b];
    int lane = threadIdx.x;
    bool act = lane < d.w;
    const int32_t *src = (const int32_t *)a.coef + (size_t)d.tc * a.plane_w * a.plane_h +
                         (size_t)d.y0 * a.plane_w + d.x0;
    int32_t *sm = a.sm + d.sm_off;
    uint32_t vmax = 0;
    uint32_t lim = (1u << d.Mb) - 1u;
    for (int y = 0; y < d.h; y++) {
        if (!act) continue;
        int32_t raw = src[(size_t)y * a.plane_w + lane];
        uint32_t v, s;
        if (a.reversible) {
            s = raw < 0;
            v = (uint32_t)(raw < 0 ? -raw : raw);
        } else {
            float cf = __int_as_float(raw);
            s = cf < 0.0f;
            float t = fabsf(cf) * d.inv_delta;
            v = (uint32_t)floorf(t);
        }
        if (v > lim) v = lim;
        sm[y * 64 + lane] = (int32_t)((s << 31) | v);
        vmax = max(vmax, v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
    int P = vmax ? 32 - __clz(vmax) : 0;
    if (lane == 0) a.P[b] = (uint8_t)P;
    __syncthreads();  // sm visible to the wave (same lanes re-read their own column anyway)
    uint64_t *B = a.bp + d.bp_off;
    uint64_t *S = B + (size_t)d.Mb * 64;
    uint64_t *SG = B + (size_t)2 * d.Mb * 64;
    for (int y = 0; y < d.h; y++) {
        uint32_t word = act ? (uint32_t)sm[y * 64 + lane] : 0u;
        uint32_t v = word & 0x7FFFFFFFu;
        uint64_t myB = 0, myS = 0;
        for (int p = 0; p < P; p++) {
            uint64_t bm = __ballot((v >> p) & 1u);
            uint64_t sm2 = __ballot((v >> p) != 0u);
            if (lane == p) { myB = bm; myS = sm2; }
        }
        uint64_t sg = __ballot(word >> 31);
        if (lane < P) {
            B[(size_t)lane * 64 + y] = myB;
            S[(size_t)lane * 64 + y] = myS;
        }
        if (lane == 63) SG[y] = sg;
    }
    bool lossless = a.reversible != 0;
    for (int p = 0; p < P; p++) {
        int64_t ref = 0, sig = 0;
        if (act) {
            for (int y = 0; y < d.h; y++) {
                uint32_t v = (uint32_t)sm[y * 64 + lane] & 0x7FFFFFFFu;
                uint32_t hi = v >> p;
                if (hi == 0) continue;
                int64_t g = dist_gain(v, p, lossless);
                if (hi == 1) sig += g;
                else ref += g;
            }
        }
        ref = wave_sum64(ref);
        sig = wave_sum64(sig);
        if (lane == 0) {
            a.dref[(size_t)b * 32 + p] = ref;
            a.dsig[(size_t)b * 32 + p] = sig;
        }
    }
}

// --------------------------------------------------------------------------
// S5: EBCOT tier-1 (Annex D) + MQ coder (Annex C).
//
// One lane encodes one code-block.  Significance state lives in 64-bit row
// masks (bit c = column c); a stripe (4 rows) is modelled with whole-row
// bit operations and only coded samples are visited.  SPP membership is the
// least fixed point of the causal neighbourhood rule, found by iterating the
// stripe's mask equations; MRP and CUP contexts are closed-form because the
// significance after CUP of plane p is exactly S[p].
// --------------------------------------------------------------------------
enum { CX_RL = 17, CX_UNI = 18 };

__device__ __forceinline__ int zc_ctx(int band, int pat) {
    int UL = pat & 1, U = (pat >> 1) & 1, UR = (pat >> 2) & 1, Lf = (pat >> 3) & 1;
    int Rt = (pat >> 4) & 1, DL = (pat >> 5) & 1, D = (pat >> 6) & 1, DR = (pat >> 7) & 1;
    int h = Lf + Rt, v = U + D, dg = UL + UR + DL + DR;
    if (band == 1) { int t = h; h = v; v = t; }
    if (band == 3) {
        int hv = h + v;
        if (dg >= 3) return 8;
        if (dg == 2) return hv >= 1 ? 7 : 6;
        if (dg == 1) return hv >= 2 ? 5 : (hv == 1 ? 4 : 3);
        return hv >= 2 ? 2 : (hv == 1 ? 1 : 0);
    }
    if (h == 2) return 8;
    if (h == 1) return v >= 1 ? 7 : (dg >= 1 ? 6 : 5);
    if (v == 2) return 4;
    if (v == 1) return 3;
    if (dg >= 2) return 2;
    return dg == 1 ? 1 : 0;
}

// pattern: Lsig Lneg Rsig Rneg Usig Uneg Dsig Dneg -> (ctx << 1) | xorbit
__device__ __forceinline__ int sc_lut(int pat) {
    auto contrib = [](int sig, int neg) { return sig ? (neg ? -1 : 1) : 0; };
    int hc = contrib(pat & 1, (pat >> 1) & 1) + contrib((pat >> 2) & 1, (pat >> 3) & 1);
    int vc = contrib((pat >> 4) & 1, (pat >> 5) & 1) + contrib((pat >> 6) & 1, (pat >> 7) & 1);
    hc = hc < -1 ? -1 : (hc > 1 ? 1 : hc);
    vc = vc < -1 ? -1 : (vc > 1 ? 1 : vc);
    int ctx, xr;
    if (hc == 1) { xr = 0; ctx = vc == 1 ? 13 : (vc == 0 ? 12 : 11); }
    else if (hc == 0) { xr = vc == -1; ctx = vc == 0 ? 9 : 10; }
    else { xr = 1; ctx = vc == 1 ? 11 : (vc == 0 ? 12 : 13); }
    return (ctx << 1) | xr;
}

__constant__ uint16_t c_qe[47] = {
    0x5601, 0x3401, 0x1801, 0x0AC1, 0x0521, 0x0221, 0x5601, 0x5401, 0x4801, 0x3801, 0x3001, 0x2401,
    0x1C01, 0x1601, 0x5601, 0x5401, 0x5101, 0x4801, 0x3801, 0x3401, 0x3001, 0x2801, 0x2401, 0x2201,
    0x1C01, 0x1801, 0x1601, 0x1401, 0x1201, 0x1101, 0x0AC1, 0x09C1, 0x08A1, 0x0521, 0x0441, 0x02A1,
    0x0221, 0x0141, 0x0111, 0x0085, 0x0049, 0x0025, 0x0015, 0x0009, 0x0005, 0x0001, 0x5601};
__constant__ uint8_t c_nmps[47] = {1,  2,  3,  4,  5,  38, 7,  8,  9,  10, 11, 12, 13, 29, 15, 16,
                                   17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32,
                                   33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 45, 46};
__constant__ uint8_t c_nlps[47] = {1,  6,  9,  12, 29, 33, 6,  14, 14, 14, 17, 18, 20, 21, 14, 14,
                                   15, 16, 17, 18, 19, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29,
                                   30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 46};

struct Mq {
    uint32_t C, A, B;
    int CT, bp, cap;
    uint8_t *out;
};

__device__ __forceinline__ void mq_byteout(Mq &m) {
    uint32_t B = m.B;
    if (B != 0xFF && m.C >= 0x8000000u) {  // carry into the pending byte
        B++;
        m.C &= 0x7FFFFFFu;
    }
    if (m.bp >= 0 && m.bp < m.cap) m.out[m.bp] = (uint8_t)B;
    m.bp++;
    if (B == 0xFF) {
        m.B = m.C >> 20;
        m.C &= 0xFFFFFu;
        m.CT = 7;
    } else {
        m.B = m.C >> 19;
        m.C &= 0x7FFFFu;
        m.CT = 8;
    }
}

__device__ __forceinline__ void mq_encode(Mq &m, uint8_t *cst, const uint32_t *tab, int d) {
    uint32_t st = *cst;
    uint32_t t = tab[st >> 1];
    uint32_t qe = t & 0xFFFFu;
    uint32_t mps = st & 1u;
    m.A -= qe;
    if ((uint32_t)d == mps) {
        if (m.A & 0x8000u) {
            m.C += qe;
            return;
        }
        if (m.A < qe) m.A = qe;
        else m.C += qe;
        st = (((t >> 16) & 63u) << 1) | mps;
    } else {
        if (m.A < qe) m.C += qe;
        else m.A = qe;
        mps ^= (t >> 28) & 1u;
        st = (((t >> 22) & 63u) << 1) | mps;
    }
    *cst = (uint8_t)st;
    int n = __clz(m.A) - 16;
    while (n > 0) {
        int s = min(n, m.CT);
        m.A <<= s;
        m.C <<= s;
        m.CT -= s;
        n -= s;
        if (m.CT == 0) mq_byteout(m);
    }
}

__device__ __forceinline__ int mq_flush(Mq &m) {
    uint32_t tempc = m.C + m.A;
    m.C |= 0xFFFFu;
    if (m.C >= tempc) m.C -= 0x8000u;
    m.C <<= m.CT;
    mq_byteout(m);
    m.C <<= m.CT;
    mq_byteout(m);
    if (m.B != 0xFF) {
        if (m.bp >= 0 && m.bp < m.cap) m.out[m.bp] = (uint8_t)m.B;
        m.bp++;
    }
    return m.bp;
}

__device__ __forceinline__ uint32_t bit(uint64_t m, int c) { return (uint32_t)(m >> c) & 1u; }

// 8-neighbour significance pattern of (row with masks) at column c.
// up: UPb (UL,U) UPa (UR); mid: MIDb (L) MIDa (R); down: DNb (DL) DNa (D,DR)
__device__ __forceinline__ int pattern8(uint64_t UPb, uint64_t UPa, uint64_t MIDb, uint64_t MIDa,
                                        uint64_t DNb, uint64_t DNa, int c) {
    return (int)(bit(UPb << 1, c) | (bit(UPb, c) << 1) | (bit(UPa >> 1, c) << 2) |
                 (bit(MIDb << 1, c) << 3) | (bit(MIDa >> 1, c) << 4) | (bit(DNb << 1, c) << 5) |
                 (bit(DNa, c) << 6) | (bit(DNa >> 1, c) << 7));
}
__device__ __forceinline__ int pattern_sign(uint64_t UPb, uint64_t MIDb, uint64_t MIDa, uint64_t DNa,
                                            uint64_t sgU, uint64_t sgM, uint64_t sgD, int c) {
    return (int)(bit(MIDb << 1, c) | (bit(sgM << 1, c) << 1) | (bit(MIDa >> 1, c) << 2) |
                 (bit(sgM >> 1, c) << 3) | (bit(UPb, c) << 4) | (bit(sgU, c) << 5) |
                 (bit(DNa, c) << 6) | (bit(sgD, c) << 7));
}
__device__ __forceinline__ uint64_t nbhd(uint64_t UPb, uint64_t UPa, uint64_t MIDb, uint64_t MIDa,
                                         uint64_t DNb, uint64_t DNa) {
    return (UPb << 1) | UPb | (UPa >> 1) | (MIDb << 1) | (MIDa >> 1) | (DNb << 1) | DNa | (DNa >> 1);
}

struct T1Args {
    const BlockDesc *blocks;
    const int32_t *order;
    int nblocks;
    const uint64_t *bp;
    const int32_t *sm;
    const int64_t *dref, *dsig;
    const uint8_t *P;
    uint8_t *out;
    int32_t *rates;  // [block][kMaxPasses]
    int64_t *dists;  // [block][kMaxPasses]
    uint8_t *npasses;
    int32_t *lengths;
    int lossless;
    int *err;
};

// Row-mask helpers for stripe s.  Index i in 0..5 = rows r0-1 .. r0+4.
#define ROWS6(dst, expr)                     \
    _Pragma("unroll") for (int i = 0; i < 6; i++) { \
        int r = r0 - 1 + i;                   \
        dst[i] = (r >= 0 && r < h) ? (expr) : 0ull; \
    }

__global__ void __launch_bounds__(64) k_t1(T1Args a) {
    __shared__ uint64_t Nsh[64 * 64];
    __shared__ uint8_t cxs[19 * 64];
    __shared__ uint8_t lzc[4 * 256];
    __shared__ uint8_t lsc[256];
    __shared__ uint32_t mqt[48];
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) lzc[i] = (uint8_t)zc_ctx(i >> 8, i & 255);
    for (int i = lane; i < 256; i += 64) lsc[i] = (uint8_t)sc_lut(i);
    if (lane < 47)
        mqt[lane] = (uint32_t)c_qe[lane] | ((uint32_t)c_nmps[lane] << 16) |
                    ((uint32_t)c_nlps[lane] << 22) |
                    ((uint32_t)(lane == 0 || lane == 6 || lane == 14) << 28);
    __syncthreads();
    const int gi = blockIdx.x * 64 + lane;
    if (gi >= a.nblocks) return;
    const int b = a.order[gi];
    const BlockDesc d = a.blocks[b];
    const int P = a.P[b];
    if (P == 0) {
        a.npasses[b] = 0;
        a.lengths[b] = 0;
        return;
    }
    const bool lossless = a.lossless != 0;
    const int w = d.w, h = d.h, Mb = d.Mb;
    const uint64_t V = (w >= 64) ? ~0ull : ((1ull << w) - 1ull);
    const uint64_t *BP = a.bp + d.bp_off;
    const uint64_t *SP = BP + (size_t)Mb * 64;
    const uint64_t *SGp = BP + (size_t)2 * Mb * 64;
    const int32_t *SM = a.sm + d.sm_off;
    const uint8_t *zl = lzc + d.band * 256;
    uint8_t *cx = cxs + lane;
#pragma unroll
    for (int k = 0; k < 19; k++) cx[k * 64] = 0;
    cx[0] = 4 << 1;
    cx[CX_RL * 64] = 3 << 1;
    cx[CX_UNI * 64] = 46 << 1;
    Mq m;
    m.C = 0; m.A = 0x8000; m.B = 0; m.CT = 12; m.bp = -1;
    m.cap = (int)d.out_cap;
    m.out = a.out + d.out_off;
    int32_t *R = a.rates + (size_t)b * kMaxPasses;
    int64_t *D = a.dists + (size_t)b * kMaxPasses;
    int np = 0;
    uint64_t *Ncol = Nsh + lane;  // Ncol[r * 64]
    const int nstripes = (h + 3) >> 2;

    for (int p = P - 1; p >= 0; --p) {
        const uint64_t *Bp = BP + (size_t)p * 64;
        const uint64_t *S0p = SP + (size_t)p * 64;
        const bool has1 = p + 1 < P, has2 = p + 2 < P;
        const uint64_t *S1p = SP + (size_t)(p + 1) * 64;
        const uint64_t *S2p = SP + (size_t)(p + 2) * 64;
        int64_t dspp = 0;
        if (p < P - 1) {
            // ---------------- significance propagation ----------------
            for (int s = 0; s < nstripes; s++) {
                const int r0 = s * 4, nr = min(4, h - r0);
                uint64_t s1[6], sg[6], bt[4], n[4] = {0, 0, 0, 0}, mem[4];
                ROWS6(s1, has1 ? S1p[r] : 0ull);
                ROWS6(sg, SGp[r]);
#pragma unroll
                for (int k = 0; k < 4; k++) bt[k] = (k < nr) ? Bp[r0 + k] : 0ull;
                const uint64_t bfprev = (r0 > 0) ? (s1[0] | Ncol[(r0 - 1) * 64]) : 0ull;
                for (;;) {
                    bool changed = false;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        if (k >= nr) { mem[k] = 0; continue; }
                        uint64_t UPb = (k == 0) ? bfprev : (s1[k] | n[k - 1]);
                        uint64_t UPa = (k == 0) ? bfprev : s1[k];
                        uint64_t MIDb = s1[k + 1] | n[k], MIDa = s1[k + 1];
                        uint64_t DNb = (k == 3) ? s1[5] : (s1[k + 2] | n[k + 1]);
                        uint64_t DNa = s1[k + 2];
                        mem[k] = ~s1[k + 1] & V & nbhd(UPb, UPa, MIDb, MIDa, DNb, DNa);
                        uint64_t nn = mem[k] & bt[k];
                        if (nn != n[k]) { n[k] = nn; changed = true; }
                    }
                    if (!changed) break;
                }
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (k < nr) Ncol[(r0 + k) * 64] = n[k];
                uint64_t colmask = mem[0] | mem[1] | mem[2] | mem[3];
                while (colmask) {
                    const int c = __ffsll((unsigned long long)colmask) - 1;
                    colmask &= colmask - 1;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        if (k >= nr || !bit(mem[k], c)) continue;
                        uint64_t UPb = (k == 0) ? bfprev : (s1[k] | n[k - 1]);
                        uint64_t UPa = (k == 0) ? bfprev : s1[k];
                        uint64_t MIDb = s1[k + 1] | n[k], MIDa = s1[k + 1];
                        uint64_t DNb = (k == 3) ? s1[5] : (s1[k + 2] | n[k + 1]);
                        uint64_t DNa = s1[k + 2];
                        int pat = pattern8(UPb, UPa, MIDb, MIDa, DNb, DNa, c);
                        int bv = (int)bit(bt[k], c);
                        mq_encode(m, cx + zl[pat] * 64, mqt, bv);
                        if (bv) {
                            int sp = lsc[pattern_sign(UPb, MIDb, MIDa, DNa, sg[k], sg[k + 1], sg[k + 2], c)];
                            uint32_t word = (uint32_t)SM[(r0 + k) * 64 + c];
                            mq_encode(m, cx + (sp >> 1) * 64, mqt, (int)((word >> 31) ^ (uint32_t)(sp & 1)));
                            dspp += dist_gain(word & 0x7FFFFFFFu, p, lossless);
                        }
                    }
                }
            }
            R[np] = m.bp + 3;
            D[np] = dspp;
            np++;
            // ---------------- magnitude refinement ----------------
            for (int s = 0; s < nstripes; s++) {
                const int r0 = s * 4, nr = min(4, h - r0);
                uint64_t post[6], bt[4], mem[4], fr[4];
                ROWS6(post, S1p[r] | Ncol[r * 64]);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    bool in = k < nr;
                    bt[k] = in ? Bp[r0 + k] : 0ull;
                    uint64_t s1k = in ? S1p[r0 + k] : 0ull;
                    mem[k] = s1k & V;
                    fr[k] = s1k & ~((in && has2) ? S2p[r0 + k] : 0ull);
                }
                uint64_t colmask = mem[0] | mem[1] | mem[2] | mem[3];
                while (colmask) {
                    const int c = __ffsll((unsigned long long)colmask) - 1;
                    colmask &= colmask - 1;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        if (k >= nr || !bit(mem[k], c)) continue;
                        int ctx;
                        if (bit(fr[k], c)) {
                            int pat = pattern8(post[k], post[k], post[k + 1], post[k + 1], post[k + 2],
                                               post[k + 2], c);
                            ctx = pat ? 15 : 14;
                        } else {
                            ctx = 16;
                        }
                        mq_encode(m, cx + ctx * 64, mqt, (int)bit(bt[k], c));
                    }
                }
            }
            R[np] = m.bp + 3;
            D[np] = a.dref[(size_t)b * 32 + p];
            np++;
        }
        // ---------------- cleanup ----------------
        const bool spp = p < P - 1;
        for (int s = 0; s < nstripes; s++) {
            const int r0 = s * 4, nr = min(4, h - r0);
            uint64_t s1[6], post[6], s0[6], sg[6], bt[4], mem[4];
            ROWS6(s1, has1 ? S1p[r] : 0ull);
            ROWS6(post, s1[i] | (spp ? Ncol[r * 64] : 0ull));
            ROWS6(s0, S0p[r]);
            ROWS6(sg, SGp[r]);
#pragma unroll
            for (int k = 0; k < 4; k++) bt[k] = (k < nr) ? Bp[r0 + k] : 0ull;
            // SPP membership with the final new-significance masks
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if (k >= nr) { mem[k] = 0; continue; }
                uint64_t c_spp = 0;
                if (spp) {
                    uint64_t UPb = post[k], UPa = (k == 0) ? post[0] : s1[k];
                    uint64_t MIDb = post[k + 1], MIDa = s1[k + 1];
                    uint64_t DNb = (k == 3) ? s1[5] : post[k + 2];
                    uint64_t DNa = s1[k + 2];
                    c_spp = ~s1[k + 1] & V & nbhd(UPb, UPa, MIDb, MIDa, DNb, DNa);
                }
                mem[k] = ~s1[k + 1] & ~c_spp & V;
            }
            uint64_t rl = 0;
            if (nr == 4) {
                uint64_t z = (s0[0] << 1) | s0[0] | (s0[0] >> 1) |
                             ((s0[1] | s0[2] | s0[3] | s0[4]) << 1) |
                             ((post[1] | post[2] | post[3] | post[4]) >> 1) |
                             (post[5] << 1) | post[5] | (post[5] >> 1);
                rl = mem[0] & mem[1] & mem[2] & mem[3] & ~z;
            }
            uint64_t colmask = mem[0] | mem[1] | mem[2] | mem[3];
            while (colmask) {
                const int c = __ffsll((unsigned long long)colmask) - 1;
                colmask &= colmask - 1;
                int kstart = 0;
                if (bit(rl, c)) {
                    int r = 4;
#pragma unroll
                    for (int k = 3; k >= 0; k--)
                        if (bit(bt[k], c)) r = k;
                    if (r == 4) {
                        mq_encode(m, cx + CX_RL * 64, mqt, 0);
                        continue;
                    }
                    mq_encode(m, cx + CX_RL * 64, mqt, 1);
                    mq_encode(m, cx + CX_UNI * 64, mqt, r >> 1);
                    mq_encode(m, cx + CX_UNI * 64, mqt, r & 1);
                    // sign of sample r: neighbours per the before/after rule
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        if (k != r) continue;
                        uint64_t UPb = s0[k];
                        uint64_t MIDb = s0[k + 1], MIDa = post[k + 1];
                        uint64_t DNa = post[k + 2];
                        int sp = lsc[pattern_sign(UPb, MIDb, MIDa, DNa, sg[k], sg[k + 1], sg[k + 2], c)];
                        uint32_t word = (uint32_t)SM[(r0 + k) * 64 + c];
                        mq_encode(m, cx + (sp >> 1) * 64, mqt, (int)((word >> 31) ^ (uint32_t)(sp & 1)));
                    }
                    kstart = r + 1;
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (k < kstart || k >= nr || !bit(mem[k], c)) continue;
                    uint64_t UPb = s0[k], UPa = (k == 0) ? s0[0] : post[k];
                    uint64_t MIDb = s0[k + 1], MIDa = post[k + 1];
                    uint64_t DNb = (k == 3) ? post[5] : s0[k + 2];
                    uint64_t DNa = post[k + 2];
                    int pat = pattern8(UPb, UPa, MIDb, MIDa, DNb, DNa, c);
                    int bv = (int)bit(bt[k], c);
                    mq_encode(m, cx + zl[pat] * 64, mqt, bv);
                    if (bv) {
                        int sp = lsc[pattern_sign(UPb, MIDb, MIDa, DNa, sg[k], sg[k + 1], sg[k + 2], c)];
                        uint32_t word = (uint32_t)SM[(r0 + k) * 64 + c];
                        mq_encode(m, cx + (sp >> 1) * 64, mqt, (int)((word >> 31) ^ (uint32_t)(sp & 1)));
                    }
                }
            }
        }
        R[np] = m.bp + 3;
        D[np] = a.dsig[(size_t)b * 32 + p] - dspp;
        np++;
    }
    const int len = mq_flush(m);
    if (len > m.cap) {
        atomicOr(a.err, 1);
    }
    R[np - 1] = len;
    for (int i = 0; i < np; i++) {
        int r = min(R[i], len);
        if (r > 1 && r <= m.cap && m.out[r - 1] == 0xFF) r--;
        R[i] = r;
    }
    a.npasses[b] = (uint8_t)np;
    a.lengths[b] = len;
}

// --------------------------------------------------------------------------
// S6: PCRD-opt.  Hull per block (thread per block), then one workgroup
// finds, for every layer at once, the smallest slope key whose total rate
// fits the layer budget (63-step bisection over the key space).
// --------------------------------------------------------------------------
struct HullArgs {
    int nblocks;
    const uint8_t *npasses;
    const int32_t *rates;
    const int64_t *dists;
    const double *weight;
    uint8_t *nhull;
    uint8_t *hpass;   // [block][kMaxPasses+1]
    uint64_t *hkey;   // [block][kMaxPasses+1]
};

__global__ void __launch_bounds__(256) k_hull(HullArgs a) {
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.nblocks) return;
    int np = a.npasses[b];
    const int32_t *R = a.rates + (size_t)b * kMaxPasses;
    const int64_t *Dd = a.dists + (size_t)b * kMaxPasses;
    uint8_t *hp = a.hpass + (size_t)b * (kMaxPasses + 1);
    uint64_t *hk = a.hkey + (size_t)b * (kMaxPasses + 1);
    double wgt = a.weight[b];
    int64_t D[kMaxPasses + 1];
    double sl[kMaxPasses + 1];
    D[0] = 0;
    for (int n = 1; n <= np; n++) D[n] = D[n - 1] + Dd[n - 1];
    int nh = 1;
    hp[0] = 0;
    sl[0] = 0.0;
    for (int n = 1; n <= np; n++) {
        for (;;) {
            int hh = hp[nh - 1];
            int64_t dD = D[n] - D[hh];
            int32_t dR = R[n - 1] - (hh ? R[hh - 1] : 0);
            if (dD <= 0) break;
            if (dR <= 0) { nh--; continue; }
            double s = (double)dD * wgt / (double)dR;
            if (nh >= 2 && s >= sl[nh - 1]) { nh--; continue; }
            hp[nh] = (uint8_t)n;
            sl[nh] = s;
            nh++;
            break;
        }
    }
    for (int i = 0; i < nh; i++) hk[i] = (uint64_t)__double_as_longlong(sl[i]);
    a.nhull[b] = (uint8_t)nh;
}

struct SelectArgs {
    int nblocks, layers, lossless;
    const uint8_t *nhull;
    const uint8_t *hpass;
    const uint64_t *hkey;
    const uint8_t *npasses;
    const int32_t *rates;
    const int64_t *budget;  // [layers]
    uint8_t *nl;            // [block][layers]
    int32_t *lrate;         // [block][layers]
};

// rate of block b at the last hull point whose key >= K
__device__ __forceinline__ int hull_pick(const SelectArgs &a, int b, uint64_t K) {
    int nh = a.nhull[b];
    const uint64_t *hk = a.hkey + (size_t)b * (kMaxPasses + 1);
    // keys strictly decrease with the hull index (i >= 1)
    int lo = 1, hi = nh;  // find first i in [1,nh) with hk[i] < K
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (hk[mid] >= K) lo = mid + 1;
        else hi = mid;
    }
    return lo - 1;  // hull index (0 = nothing)
}

__global__ void __launch_bounds__(1024) k_select(SelectArgs a) {
    __shared__ uint64_t lo[kMaxLayers], hi[kMaxLayers];
    __shared__ int64_t part[32][kMaxLayers];
    const int L = a.layers;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid < L) { lo[tid] = 0; hi[tid] = 0x7FF0000000000000ull; }
    __syncthreads();
    for (int it = 0; it < 64; it++) {
        int64_t acc[kMaxLayers];
        uint64_t mid[kMaxLayers];
        for (int l = 0; l < L; l++) { acc[l] = 0; mid[l] = lo[l] + ((hi[l] - lo[l]) >> 1); }
        for (int b = tid; b < a.nblocks; b += blockDim.x) {
            const int32_t *R = a.rates + (size_t)b * kMaxPasses;
            const uint8_t *hp = a.hpass + (size_t)b * (kMaxPasses + 1);
            for (int l = 0; l < L; l++) {
                int hi2 = hull_pick(a, b, mid[l]);
                int n = hp[hi2];
                acc[l] += n ? R[n - 1] : 0;
            }
        }
        for (int l = 0; l < L; l++) {
            int64_t v = wave_sum64(acc[l]);
            if (lane == 0) part[wv][l] = v;
        }
        __syncthreads();
        if (tid < L) {
            int64_t s = 0;
            for (int q = 0; q < (int)(blockDim.x >> 6); q++) s += part[q][tid];
            if (lo[tid] < hi[tid]) {
                uint64_t md = lo[tid] + ((hi[tid] - lo[tid]) >> 1);
                if (s <= a.budget[tid]) hi[tid] = md;
                else lo[tid] = md + 1;
            }
        }
        __syncthreads();
    }
    for (int b = tid; b < a.nblocks; b += blockDim.x) {
        const int32_t *R = a.rates + (size_t)b * kMaxPasses;
        const uint8_t *hp = a.hpass + (size_t)b * (kMaxPasses + 1);
        for (int l = 0; l < L; l++) {
            int n;
            if (a.lossless && l == L - 1) n = a.npasses[b];
            else n = hp[hull_pick(a, b, hi[l])];
            a.nl[(size_t)b * L + l] = (uint8_t)n;
            a.lrate[(size_t)b * L + l] = n ? R[n - 1] : 0;
        }
    }
}

// gather included bytes: one workgroup per block
__global__ void __launch_bounds__(256) k_compact(const BlockDesc *blocks, const uint8_t *src,
                                                 const uint64_t *dst_off, const int32_t *len,
                                                 uint8_t *dst) {
    int b = blockIdx.x;
    const uint8_t *s = src + blocks[b].out_off;
    uint8_t *o = dst + dst_off[b];
    int n = len[b];
    for (int i = threadIdx.x; i < n; i += blockDim.x) o[i] = s[i];
}

// --------------------------------------------------------------------------
// Device pipeline
// --------------------------------------------------------------------------
template <typename T>
static bool ensure(DevBuf &b, size_t count, std::string &err) {
    size_t bytes = count * sizeof(T);
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return true;
    if (b.ptr) (void)hipFree(b.ptr);
    b.ptr = nullptr;
    b.bytes = 0;
    size_t alloc = bytes + bytes / 8;
    hipError_t e = hipMalloc(&b.ptr, alloc);
    if (e != hipSuccess) {
        err = std::string("hipMalloc(") + std::to_string(alloc) + "): " + hipGetErrorString(e);
        return false;
    }
    b.bytes = alloc;
    return true;
}

GpuEncoder::~GpuEncoder() {
    DevBuf *all[] = {&coef, &blocks, &order, &bp, &sm, &P, &dref, &dsig, &t1out, &rates, &dists,
                     &npasses, &lengths, &weight, &nhull, &hpass, &hkey, &budget, &nl, &lrate,
                     &dstoff, &packed, &err, &tcw, &tch, &strips, &src};
    for (DevBuf *b : all)
        if (b->ptr) (void)hipFree(b->ptr);
    if (stream) (void)hipStreamDestroy(stream);
    for (int i = 0; i < kNumEvents; i++)
        if (ev[i]) (void)hipEventDestroy(ev[i]);
    if (h_packed) (void)hipHostFree(h_packed);
}

bool GpuEncoder::init(int dev, std::string &err) {
    device = dev;
    HIPCHECK(hipSetDevice(dev));
    HIPCHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    for (int i = 0; i < kNumEvents; i++) HIPCHECK(hipEventCreate(&ev[i]));
    return true;
}

bool GpuEncoder::upload_source(const void *host, size_t len, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    if (!ensure<uint8_t>(src, len, err)) return false;
    HIPCHECK(hipMemcpyAsync(src.ptr, host, len, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    return true;
}

bool GpuEncoder::dump(const char *dir, const char *name, const DevBuf &b, size_t bytes,
                      std::string &err) {
    std::vector<uint8_t> h(bytes);
    HIPCHECK(hipStreamSynchronize(stream));
    if (bytes) HIPCHECK(hipMemcpy(h.data(), b.ptr, bytes, hipMemcpyDeviceToHost));
    std::string path = std::string(dir) + "/" + name;
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) { err = "cannot write dump " + path; return false; }
    fwrite(h.data(), 1, bytes, f);
    fclose(f);
    return true;
}

bool GpuEncoder::run_front(const void *d_src, const jp2hip_layout &lay, const Plan &plan,
                           bool profile, StageTimes &st, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    const int nb = (int)plan.blocks.size();
    const bool rev = plan.rc.reversible != 0;
    size_t plane = (size_t)plan.plane_w * plan.plane_h;
    if (!ensure<int32_t>(coef, plane * plan.ntc, err)) return false;
    if (!ensure<BlockDesc>(blocks, nb, err)) return false;
    if (!ensure<int32_t>(order, nb, err)) return false;
    if (!ensure<uint64_t>(bp, plan.bp_words, err)) return false;
    if (!ensure<int32_t>(sm, plan.sm_words, err)) return false;
    if (!ensure<uint8_t>(P, nb, err)) return false;
    if (!ensure<int64_t>(dref, (size_t)nb * 32, err)) return false;
    if (!ensure<int64_t>(dsig, (size_t)nb * 32, err)) return false;
    if (!ensure<uint8_t>(t1out, plan.out_bytes, err)) return false;
    if (!ensure<int32_t>(rates, (size_t)nb * kMaxPasses, err)) return false;
    if (!ensure<int64_t>(dists, (size_t)nb * kMaxPasses, err)) return false;
    if (!ensure<uint8_t>(npasses, nb, err)) return false;
    if (!ensure<int32_t>(lengths, nb, err)) return false;
    if (!ensure<double>(weight, nb, err)) return false;
    if (!ensure<uint8_t>(nhull, nb, err)) return false;
    if (!ensure<uint8_t>(hpass, (size_t)nb * (kMaxPasses + 1), err)) return false;
    if (!ensure<uint64_t>(hkey, (size_t)nb * (kMaxPasses + 1), err)) return false;
    if (!ensure<int64_t>(budget, kMaxLayers, err)) return false;
    if (!ensure<uint8_t>(nl, (size_t)nb * plan.rc.layers, err)) return false;
    if (!ensure<int32_t>(lrate, (size_t)nb * plan.rc.layers, err)) return false;
    if (!ensure<int>(this->err, 4, err)) return false;
    if (!ensure<int32_t>(tcw, plan.ntc, err)) return false;
    if (!ensure<int32_t>(tch, plan.ntc, err)) return false;
    if (!ensure<uint64_t>(strips, lay.nstrips, err)) return false;

    HIPCHECK(hipMemcpyAsync(blocks.ptr, plan.blocks.data(), sizeof(BlockDesc) * nb, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipMemcpyAsync(order.ptr, plan.t1_order.data(), sizeof(int32_t) * nb, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipMemcpyAsync(weight.ptr, plan.weight.data(), sizeof(double) * nb, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipMemcpyAsync(tcw.ptr, plan.tc_w.data(), sizeof(int32_t) * plan.ntc, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipMemcpyAsync(tch.ptr, plan.tc_h.data(), sizeof(int32_t) * plan.ntc, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipMemcpyAsync(strips.ptr, lay.strip_offsets, sizeof(uint64_t) * lay.nstrips, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipMemsetAsync(this->err.ptr, 0, sizeof(int), stream));

    HIPCHECK(hipEventRecord(ev[0], stream));
    // S1+S2
    IngestArgs ia;
    ia.src = (const uint8_t *)d_src;
    ia.strip_off = (const uint64_t *)strips.ptr;
    ia.rps = lay.rows_per_strip;
    ia.w = plan.w; ia.h = plan.h; ia.nc = plan.nc; ia.bits = plan.bits;
    ia.planar = lay.planar; ia.big_endian = lay.big_endian;
    ia.mct = plan.rc.mct; ia.reversible = plan.rc.reversible;
    ia.ntx = plan.ntx; ia.tile_w = plan.rc.tile_w; ia.tile_h = plan.rc.tile_h;
    ia.plane_w = plan.plane_w; ia.plane_h = plan.plane_h;
    ia.spp_strips = (plan.h + lay.rows_per_strip - 1) / lay.rows_per_strip;
    ia.coef = coef.ptr;
    dim3 gi((plan.w + 63) / 64, (plan.h + 3) / 4);
    hipLaunchKernelGGL(k_ingest, gi, dim3(256), 0, stream, ia);
    HIPCHECK(hipGetLastError());
    const char *dd = getenv("JP2HIP_DUMP_DIR");
    if (dd && !dump(dd, "ingest.bin", coef, plane * plan.ntc * 4, err)) return false;
    HIPCHECK(hipEventRecord(ev[1], stream));
    // S3
    for (int lv = 1; lv <= plan.rc.levels; lv++) {
        DwtArgs da;
        da.coef = coef.ptr;
        da.tc_w = (const int32_t *)tcw.ptr;
        da.tc_h = (const int32_t *)tch.ptr;
        da.plane_w = plan.plane_w;
        da.plane_h = plan.plane_h;
        da.level = lv;
        int maxW = (plan.plane_w + (1 << (lv - 1)) - 1) >> (lv - 1);
        int maxH = (plan.plane_h + (1 << (lv - 1)) - 1) >> (lv - 1);
        int cw = std::max(1, std::min(64, 8192 / std::max(1, maxH)));
        da.cw = cw;
        size_t lds_v = (size_t)maxH * (cw + 1) * 4;
        dim3 gv((maxW + cw - 1) / cw, plan.ntc);
        if (rev) hipLaunchKernelGGL(k_dwt_vert<true>, gv, dim3(256), lds_v, stream, da);
        else hipLaunchKernelGGL(k_dwt_vert<false>, gv, dim3(256), lds_v, stream, da);
        HIPCHECK(hipGetLastError());
        size_t lds_h = (size_t)4 * (maxW + 1) * 4;
        dim3 gh((maxH + 3) / 4, plan.ntc);
        if (rev) hipLaunchKernelGGL(k_dwt_horz<true>, gh, dim3(256), lds_h, stream, da);
        else hipLaunchKernelGGL(k_dwt_horz<false>, gh, dim3(256), lds_h, stream, da);
        HIPCHECK(hipGetLastError());
    }
    HIPCHECK(hipEventRecord(ev[2], stream));
    if (dd && !dump(dd, "dwt.bin", coef, plane * plan.ntc * 4, err)) return false;
    // S4
    QuantArgs qa;
    qa.blocks = (const BlockDesc *)blocks.ptr;
    qa.coef = coef.ptr;
    qa.plane_w = plan.plane_w; qa.plane_h = plan.plane_h;
    qa.reversible = plan.rc.reversible;
    qa.bp = (uint64_t *)bp.ptr;
    qa.sm = (int32_t *)sm.ptr;
    qa.P = (uint8_t *)P.ptr;
    qa.dref = (int64_t *)dref.ptr;
    qa.dsig = (int64_t *)dsig.ptr;
    if (nb) hipLaunchKernelGGL(k_quant, dim3(nb), dim3(64), 0, stream, qa);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(ev[3], stream));
    // S5
    T1Args ta;
    ta.blocks = (const BlockDesc *)blocks.ptr;
    ta.order = (const int32_t *)order.ptr;
    ta.nblocks = nb;
    ta.bp = (const uint64_t *)bp.ptr;
    ta.sm = (const int32_t *)sm.ptr;
    ta.dref = (const int64_t *)dref.ptr;
    ta.dsig = (const int64_t *)dsig.ptr;
    ta.P = (const uint8_t *)P.ptr;
    ta.out = (uint8_t *)t1out.ptr;
    ta.rates = (int32_t *)rates.ptr;
    ta.dists = (int64_t *)dists.ptr;
    ta.npasses = (uint8_t *)npasses.ptr;
    ta.lengths = (int32_t *)lengths.ptr;
    ta.lossless = plan.rc.reversible;
    ta.err = (int *)this->err.ptr;
    if (nb) hipLaunchKernelGGL(k_t1, dim3((nb + 63) / 64), dim3(64), 0, stream, ta);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(ev[4], stream));
    // S6a hulls
    HullArgs ha;
    ha.nblocks = nb;
    ha.npasses = (const uint8_t *)npasses.ptr;
    ha.rates = (const int32_t *)rates.ptr;
    ha.dists = (const int64_t *)dists.ptr;
    ha.weight = (const double *)weight.ptr;
    ha.nhull = (uint8_t *)nhull.ptr;
    ha.hpass = (uint8_t *)hpass.ptr;
    ha.hkey = (uint64_t *)hkey.ptr;
    if (nb) hipLaunchKernelGGL(k_hull, dim3((nb + 255) / 256), dim3(256), 0, stream, ha);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(ev[5], stream));
    // totals needed on the host for the budgets
    h_lengths.resize(nb);
    h_npasses.resize(nb);
    h_P.resize(nb);
    HIPCHECK(hipMemcpyAsync(h_P.data(), P.ptr, nb, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipMemcpyAsync(h_lengths.data(), lengths.ptr, sizeof(int32_t) * nb, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipMemcpyAsync(h_npasses.data(), npasses.ptr, nb, hipMemcpyDeviceToHost, stream));
    int herr = 0;
    HIPCHECK(hipMemcpyAsync(&herr, this->err.ptr, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    if (herr) {
        err = "tier-1 output capacity exceeded";
        return false;
    }
    if (dd) {
        if (!dump(dd, "blocks.bin", blocks, sizeof(BlockDesc) * nb, err)) return false;
        if (!dump(dd, "sm.bin", sm, plan.sm_words * 4, err)) return false;
        if (!dump(dd, "P.bin", P, nb, err)) return false;
        if (!dump(dd, "t1out.bin", t1out, plan.out_bytes, err)) return false;
        if (!dump(dd, "lengths.bin", lengths, (size_t)nb * 4, err)) return false;
        if (!dump(dd, "npasses.bin", npasses, nb, err)) return false;
        if (!dump(dd, "rates.bin", rates, (size_t)nb * kMaxPasses * 4, err)) return false;
        if (!dump(dd, "dists.bin", dists, (size_t)nb * kMaxPasses * 8, err)) return false;
        if (!dump(dd, "dref.bin", dref, (size_t)nb * 32 * 8, err)) return false;
        if (!dump(dd, "dsig.bin", dsig, (size_t)nb * 32 * 8, err)) return false;
        if (!dump(dd, "bp.bin", bp, plan.bp_words * 8, err)) return false;
    }
    if (profile) {
        float t;
        HIPCHECK(hipEventElapsedTime(&t, ev[0], ev[1])); st.ingest = t;
        HIPCHECK(hipEventElapsedTime(&t, ev[1], ev[2])); st.dwt = t;
        HIPCHECK(hipEventElapsedTime(&t, ev[2], ev[3])); st.quant = t;
        HIPCHECK(hipEventElapsedTime(&t, ev[3], ev[4])); st.t1 = t;
        HIPCHECK(hipEventElapsedTime(&t, ev[4], ev[5])); st.pcrd = t;
    }
    return true;
}

bool GpuEncoder::select(const Plan &plan, const std::vector<int64_t> &budgets,
                        std::vector<uint8_t> &h_nl, std::vector<int32_t> &h_lrate, bool profile,
                        StageTimes &st, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    const int nb = (int)plan.blocks.size();
    const int L = plan.rc.layers;
    HIPCHECK(hipMemcpyAsync(budget.ptr, budgets.data(), sizeof(int64_t) * L, hipMemcpyHostToDevice, stream));
    SelectArgs sa;
    sa.nblocks = nb;
    sa.layers = L;
    sa.lossless = plan.rc.rate_bpp <= 0.0;
    sa.nhull = (const uint8_t *)nhull.ptr;
    sa.hpass = (const uint8_t *)hpass.ptr;
    sa.hkey = (const uint64_t *)hkey.ptr;
    sa.npasses = (const uint8_t *)npasses.ptr;
    sa.rates = (const int32_t *)rates.ptr;
    sa.budget = (const int64_t *)budget.ptr;
    sa.nl = (uint8_t *)nl.ptr;
    sa.lrate = (int32_t *)lrate.ptr;
    HIPCHECK(hipEventRecord(ev[6], stream));
    if (nb) hipLaunchKernelGGL(k_select, dim3(1), dim3(1024), 0, stream, sa);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(ev[7], stream));
    h_nl.resize((size_t)nb * L);
    h_lrate.resize((size_t)nb * L);
    HIPCHECK(hipMemcpyAsync(h_nl.data(), nl.ptr, h_nl.size(), hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipMemcpyAsync(h_lrate.data(), lrate.ptr, sizeof(int32_t) * h_lrate.size(), hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    if (profile) {
        float t;
        HIPCHECK(hipEventElapsedTime(&t, ev[6], ev[7]));
        st.pcrd += t;
    }
    return true;
}

bool GpuEncoder::gather(const Plan &plan, const std::vector<int32_t> &final_len,
                        const std::vector<uint64_t> &offsets, uint64_t total, const uint8_t **host_data,
                        bool profile, StageTimes &st, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    const int nb = (int)plan.blocks.size();
    if (!ensure<uint64_t>(dstoff, nb, err)) return false;
    if (!ensure<uint8_t>(packed, total, err)) return false;
    if (!ensure<int32_t>(lengths, nb, err)) return false;
    if (h_packed_cap < total) {
        if (h_packed) (void)hipHostFree(h_packed);
        h_packed = nullptr;
        h_packed_cap = 0;
        size_t cap = total + total / 4 + 4096;
        HIPCHECK(hipHostMalloc((void **)&h_packed, cap, hipHostMallocDefault));
        h_packed_cap = cap;
    }
    HIPCHECK(hipEventRecord(ev[8], stream));
    HIPCHECK(hipMemcpyAsync(dstoff.ptr, offsets.data(), sizeof(uint64_t) * nb, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipMemcpyAsync(lengths.ptr, final_len.data(), sizeof(int32_t) * nb, hipMemcpyHostToDevice, stream));
    if (nb) hipLaunchKernelGGL(k_compact, dim3(nb), dim3(256), 0, stream, (const BlockDesc *)blocks.ptr,
                               (const uint8_t *)t1out.ptr, (const uint64_t *)dstoff.ptr,
                               (const int32_t *)lengths.ptr, (uint8_t *)packed.ptr);
    HIPCHECK(hipGetLastError());
    if (total) HIPCHECK(hipMemcpyAsync(h_packed, packed.ptr, total, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipEventRecord(ev[9], stream));
    HIPCHECK(hipStreamSynchronize(stream));
    if (profile) {
        float t;
        HIPCHECK(hipEventElapsedTime(&t, ev[8], ev[9]));
        st.d2h += t;
    }
    *host_data = h_packed;
    return true;
}

bool GpuEncoder::t1_total_bytes(int64_t &bytes, int64_t &passes) const {
    bytes = 0;
    passes = 0;
    for (size_t i = 0; i < h_lengths.size(); i++) {
        bytes += h_lengths[i];
        passes += h_npasses[i];
    }
    return true;
}

}  // namespace jp2hip
