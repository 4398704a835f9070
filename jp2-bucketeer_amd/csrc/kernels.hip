// kernels.hip -- the gfx950 encode path of libjp2hip.
//
// Stage map (reference stage: kdu_compress invoked at
// KakaduConverter.java:61-71):
//   (dwt.hip)    S1-S3  TIFF strips in HBM -> level shift, RCT (int) / ICT
//                       (fp32) fused into DWT level 1; LDS-staged levels
//   k_ingest     S1+S2  stand-alone ingest, used only when levels == 0
//   k_quant      S4     deadzone quantiser + bit-plane masks via wave ballot
//   (t1.hip)     S5     EBCOT tier-1: context modelling + MQ coder
//   k_hull/k_select S6  PCRD-opt convex hulls + global slope thresholds
//   k_compact           gather the included bytes for the D2H copy
// Tier-2 (S7/S8) runs on host threads (t2.cpp).
//
// Floating point: built with -ffp-contract=off; every 9/7 / ICT expression is
// written in the same order as the oracle so the lossy path is bit-exact.
#include <hip/hip_runtime.h>

#include <chrono>
#include <thread>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "device_common.h"
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
    int row0;  // image row of local row 0 (tile-split bands)
    void *coef;
    float inv;     // no decomposition: the one band's quantiser (QuantTab [0][0])
    uint32_t lim;
    int q16;
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
    for (int c = 0; c < 4; c++) s[c] = (c < a.nc) ? read_sample(a, x, a.row0 + y, c) - off : 0;
    int tx = x / a.tile_w, ty = y / a.tile_h;
    size_t plane = (size_t)a.plane_w * a.plane_h;
    size_t base = ((size_t)(ty * a.ntx + tx) * a.nc) * plane + (size_t)(y - ty * a.tile_h) * a.plane_w +
                  (x - tx * a.tile_w);
    bool domct = a.mct && a.nc >= 3;
    // the samples are the final coefficients: quantisation indices, as the
    // DWT writes them (dwt.hip)
    auto put = [&](int c, uint32_t q) {
        if (a.q16) ((uint16_t *)a.coef)[base + (size_t)c * plane] = (uint16_t)q;
        else ((uint32_t *)a.coef)[base + (size_t)c * plane] = q;
    };
    if (a.reversible) {
        int32_t v[4] = {s[0], s[1], s[2], s[3]};
        if (domct) {
            v[0] = (s[0] + 2 * s[1] + s[2]) >> 2;
            v[1] = s[2] - s[1];
            v[2] = s[0] - s[1];
        }
#pragma unroll
        for (int c = 0; c < 4; c++)
            if (c < a.nc) put(c, quant_sm<true>(v[c], a.inv, a.lim, a.q16 ? 15 : 31));
    } else {
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
            if (c < a.nc) put(c, quant_sm<false>(__float_as_int(f[c]), a.inv, a.lim, a.q16 ? 15 : 31));
    }
}

// --------------------------------------------------------------------------
// S1a: compressed strips (TIFF 6.0 sections 9, 13, 14; Deflate per the TIFF
// Technical Notes).  The strips of an LZW, Deflate or PackBits TIFF are
// decoded in HBM before ingest: one lane per strip (each strip is an
// independent byte stream), output strip s at s * stride of a
// staging buffer, so ingest then reads an uncompressed layout.  Horizontal
// differencing (Predictor 2) is undone afterwards, one lane per row.
// --------------------------------------------------------------------------

// LZW, MSB-first codes of 9..12 bits with TIFF's early width change; the
// string of table entry k is (start, length) inside the strip's own output
// (entry k = string(prev) + first byte of the next string, which is exactly
// where the decoder wrote them), so decoding is copying, as in LZ77.
// One strip per single-lane workgroup: a strip's decode is one serial chain,
// so strips must not share a wave (divergent lanes run each other's paths);
// the 4096-entry string table lives in LDS, and a string is copied 8 bytes
// of independent loads at a time.
__global__ void __launch_bounds__(64) k_unlzw(UnpackArgs a) {
    __shared__ uint2 tab[4096];
    const int s = blockIdx.x;
    if (s >= a.nstrips || threadIdx.x || (a.only && !a.only[s])) return;
    const uint8_t *in = a.src + a.off[s];
    const uint64_t n = a.cnt[s], cap = strip_out_bytes(a, s);
    uint8_t *out = a.dst + (uint64_t)s * a.stride;
    uint64_t ip = 0, pos = 0, acc = 0, prev_pos = 0;
    int nbits = 0, width = 9, next = 258;
    uint32_t prev_len = 0;
    bool bad = false;
    if (n >= 2 && in[0] == 0 && (in[1] & 1)) {  // pre-TIFF 6.0 (LSB-first) LZW, as libtiff detects it
        atomicOr(a.err, 4);
        return;
    }
    for (;;) {
        if (pos >= cap) break;  // strip complete: trailing codes are ignored (libtiff stops here too)
        if (nbits < width) {  // top up to >= 32 bits with independent byte loads
            if (ip + 4 <= n) {
                const uint32_t w4 = ((uint32_t)in[ip] << 24) | ((uint32_t)in[ip + 1] << 16) |
                                    ((uint32_t)in[ip + 2] << 8) | in[ip + 3];
                acc = (acc << 32) | w4;
                ip += 4;
                nbits += 32;
            } else {
                while (nbits < width && ip < n) { acc = (acc << 8) | in[ip++]; nbits += 8; }
            }
        }
        if (nbits < width) break;  // input exhausted: treat as end of information
        const int code = (int)((acc >> (nbits - width)) & ((1u << width) - 1u));
        nbits -= width;
        if (code == 257) break;
        if (code == 256) { width = 9; next = 258; prev_len = 0; continue; }
        const uint64_t cur = pos;
        uint32_t len;
        if (code < 256) {
            out[pos++] = (uint8_t)code;
            len = 1;
        } else {
            uint64_t from;
            bool kwk = false;  // string(prev) + its own first byte: the last byte is the first
            if (code < next) { const uint2 e = tab[code]; from = e.x; len = e.y; }
            else if (code == next && prev_len) { from = prev_pos; len = prev_len + 1; kwk = true; }
            else { bad = true; break; }
            if (pos + len > cap) {  // the strip ends inside this string: keep what fits
                for (uint64_t k = 0; pos + k < cap; k++) out[pos + k] = (kwk && k == len - 1) ? out[from] : out[from + k];
                pos = cap;
                break;
            }
            const uint32_t body = kwk ? len - 1 : len;  // source bytes all lie before pos
            uint32_t k = 0;
            for (; k + 8 <= body; k += 8) {
                uint8_t t[8];
#pragma unroll
                for (int j = 0; j < 8; j++) t[j] = out[from + k + j];
#pragma unroll
                for (int j = 0; j < 8; j++) out[pos + k + j] = t[j];
            }
            for (; k < body; k++) out[pos + k] = out[from + k];
            if (kwk) out[pos + body] = out[from];
            pos += len;
        }
        if (prev_len && next < 4096) {
            tab[next] = make_uint2((uint32_t)prev_pos, prev_len + 1);
            next++;
            if (next >= (1 << width) - 1 && width < 12) width++;
        }
        prev_pos = cur;
        prev_len = len;
    }
    if (bad || pos != cap) atomicOr(a.err, 2);
}

// PackBits: n in 0..127 copies n+1 literal bytes, -127..-1 repeats the next
// byte 1-n times, -128 is a no-op.  One strip per wave: every lane walks the
// same run headers (uniform control flow), and a run's bytes are written by
// the 64 lanes together.
__global__ void __launch_bounds__(64) k_unpackbits(UnpackArgs a) {
    const int s = blockIdx.x, lane = threadIdx.x;
    if (s >= a.nstrips) return;
    const uint8_t *in = a.src + a.off[s];
    const uint64_t n = a.cnt[s], cap = strip_out_bytes(a, s);
    uint8_t *out = a.dst + (uint64_t)s * a.stride;
    uint64_t ip = 0, pos = 0;
    bool bad = false;
    while (ip < n && pos < cap) {
        const int c = (int8_t)in[ip++];
        // a run past the strip's end is cut at cap (libtiff keeps what fits)
        if (c >= 0) {
            if (ip + c + 1 > n) { bad = true; break; }
            const uint64_t m = min((uint64_t)c + 1, cap - pos);
            for (uint64_t i = lane; i < m; i += 64) out[pos + i] = in[ip + i];
            ip += c + 1;
            pos += m;
        } else if (c != -128) {
            if (ip >= n) { bad = true; break; }
            const uint8_t v = in[ip++];
            const uint64_t m = min((uint64_t)(1 - c), cap - pos);
            for (uint64_t i = lane; i < m; i += 64) out[pos + i] = v;
            pos += m;
        }
    }
    if (lane == 0 && (bad || pos != cap)) atomicOr(a.err, 2);
}

// Deflate (RFC 1951) in a zlib wrapper (RFC 1950): TIFF compression 8
// (Adobe Deflate) and 32946 (the older Deflate code), in two phases.
//
// k_inflate, one wave per strip: a Huffman stream has no positions known
// before decoding it, so the symbol decode is one serial chain per strip.
// The wave runs it with wave-uniform control flow (the state in scalar
// registers) and keeps that chain short: it does not build the output.  Each
// output byte p gets a 32-bit link instead -- kLinkByte | value for a
// literal (or a stored-block byte), or the position of an earlier byte with
// the same value for a match byte (an overlapping match, dist < length,
// points before the match start: byte p0 + x -> p0 - dist + x mod dist) --
// written by the lanes with plain stores (no window, no read-back, no
// barrier).  Length and distance bases come from closed forms (scalar
// arithmetic), so a literal costs one table lookup and a match two.  The
// lanes are used where the work is parallel: the compressed bytes reach an LDS
// ring 1 KiB per vector load, one chunk ahead; the code tables are built by
// the lanes (ranks within a code length by ballot); a match's links and a
// stored block's bytes are written a lane per byte.
// k_inflate_links then resolves the links of every strip in parallel:
// pointer doubling (link[p] = link[link[p]], in place -- a link read while
// another thread rewrites it is still a valid link of the same value), then
// each byte follows what is left of its chain and is written out.
// kInfLanes is the wave width (the host build of tests/test_inflate_host.py
// runs the same text with one lane).
#ifndef JP2HIP_INF_LANES
#define JP2HIP_INF_LANES 64
#endif
constexpr int kInfLanes = JP2HIP_INF_LANES;
constexpr uint32_t kInChunkWords = 4 * kInfLanes;       // words per ring refill (16 bytes a lane)
constexpr uint32_t kInRingWords = 2 * (kInChunkWords > 16 ? kInChunkWords : 16);  // >= two chunks
constexpr int kInfLB = 12, kInfDB = 9;                  // direct-lookup bits: literal/length, distance
constexpr uint32_t kLinkByte = 0x80000000u;             // link of a byte whose value is known
// the literal/length direct lookup's entry for a longer code: bit 8 set like
// every non-literal's, so "literal" is one bit test (entries: len << 9 | sym)
constexpr uint32_t kInfNoFast = 0x100u;
constexpr int kLinkDoublings = 5;                       // pointer-doubling rounds before the chase

__constant__ uint8_t kInfClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// RFC 1951 3.2.5 in closed form: length code i = sym - 257 (0..28) and
// distance code d (0..29) -> (base, extra bits)
__device__ __forceinline__ uint32_t inf_len_extra(uint32_t i) { return i < 8u || i == 28u ? 0u : (i - 4u) >> 2; }
__device__ __forceinline__ uint32_t inf_len_base(uint32_t i) {
    return i == 28u ? 258u : (i < 8u ? 3u + i : ((4u + (i & 3u)) << inf_len_extra(i)) + 3u);
}
__device__ __forceinline__ uint32_t inf_dist_extra(uint32_t d) { return d < 4u ? 0u : (d >> 1) - 1u; }
__device__ __forceinline__ uint32_t inf_dist_base(uint32_t d) {
    return d < 4u ? d + 1u : ((2u + (d & 1u)) << inf_dist_extra(d)) + 1u;
}

__device__ __forceinline__ uint32_t inf_uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t inf_uni64(uint64_t v) {
    return ((uint64_t)inf_uni((uint32_t)(v >> 32)) << 32) | inf_uni((uint32_t)v);
}

struct InfShared {
    uint32_t ring[kInRingWords];          // compressed stream words
    uint16_t lfast[1 << kInfLB], dfast[1 << kInfDB];
    uint16_t lcnt[16], dcnt[16], lsym[288], dsym[32];
    uint8_t lens[320];
    uint32_t scr[64];                     // table-build scratch
};

// Bit reader over the strip's 16-byte-aligned words, fed from the LDS ring,
// addressed by absolute bit position P (bit 0 = bit 0 of the aligned base
// word; the stream starts at head_bits).  Words past the stream read as zero
// (never loaded): decoding runs on to the end of the strip's output or of the
// block, and a stream read past its end (P > end_bits) is reported corrupt at
// the end -- no per-read bookkeeping on the hot path.
struct InfIn {
    const uint32_t *w;                 // aligned base of the stream
    uint32_t nw;                       // words holding stream bytes
    uint64_t loaded;                   // words written to the ring
    uint64_t P;                        // next bit to read
    uint64_t head_bits, end_bits;      // where the stream starts / ends (bits)
    uint4 pre;                         // this lane's 16 bytes of the chunk after them
    uint32_t *ring;
    int lane;
    __device__ __forceinline__ uint4 chunk(uint64_t c) const {  // this lane's part of chunk c
        const uint64_t w0 = c * kInChunkWords + 4u * (uint32_t)lane;
        if (w0 + 4 <= nw) return *(const uint4 *)(w + w0);
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (w0 + 0 < nw) v.x = w[w0 + 0];
        if (w0 + 1 < nw) v.y = w[w0 + 1];
        if (w0 + 2 < nw) v.z = w[w0 + 2];
        return v;
    }
    __device__ __forceinline__ void top_up() {  // the prefetched chunk into the ring, the next one in flight
        const uint64_t c = loaded / kInChunkWords;
        ((uint4 *)ring)[(c * kInfLanes + (uint32_t)lane) % (kInRingWords / 4)] = pre;
        loaded += kInChunkWords;
        pre = chunk(c + 1);
    }
    // the ring holds at least 8 words (256 bits) from P's word on: called once
    // per window / symbol / code length (each reads < 64 bits from P)
    __device__ __forceinline__ void ensure() {
        const uint64_t k = P >> 5;
        if (k + 8 >= loaded) {
            if (k >= loaded) {  // a jump (past a stored block): restart the ring at P's chunk
                loaded = (k / kInChunkWords) * kInChunkWords;
                pre = chunk(loaded / kInChunkWords);
            }
            do top_up(); while (k + 8 >= loaded);  // (once per 1 KiB on the GPU)
            __builtin_amdgcn_wave_barrier();
            // wave-uniform, after the lane-dependent loads: the decode keeps
            // running on the scalar unit
            loaded = inf_uni64(loaded);
        }
    }
    __device__ __forceinline__ void init(const uint8_t *in, uint64_t n, uint32_t *r, int ln) {
        const uint64_t addr = (uint64_t)(uintptr_t)in, head = addr & 15;
        w = (const uint32_t *)(uintptr_t)(addr - head);
        nw = (uint32_t)((head + n + 3) >> 2);
        ring = r;
        lane = ln;
        loaded = 0;
        pre = chunk(0);
        head_bits = 8 * head;
        end_bits = 8 * (head + n);
        P = head_bits;
        ensure();
    }
    // n <= 32 bits at bit position q (wave-uniform; the ring must hold them)
    __device__ __forceinline__ uint32_t bits_at(uint64_t q, int n) const {
        const uint64_t k = q >> 5;
        const uint32_t lo = inf_uni(ring[k % kInRingWords]), hi = inf_uni(ring[(k + 1) % kInRingWords]);
        const uint32_t v = __builtin_amdgcn_alignbit(hi, lo, (uint32_t)(q & 31));
        return n >= 32 ? v : v & ((1u << n) - 1u);
    }
    __device__ __forceinline__ uint32_t get(int n) {  // n <= 32
        const uint32_t v = bits_at(P, n);
        P += (uint64_t)n;
        return v;
    }
    __device__ __forceinline__ uint64_t consumed() const { return P - head_bits; }
    __device__ __forceinline__ void align() { P = (P + 7) & ~7ull; }  // to the next byte
};

// Canonical code of a length-walk (codes longer than the direct lookup),
// from bit position q; returns the symbol and sets *len (0: invalid)
__device__ int inf_walk_at(const InfIn &b, uint64_t q, const uint16_t *cnt, const uint16_t *sym, int *len) {
    int code = 0, first = 0, index = 0;
    const uint32_t v = b.bits_at(q, 16);
    for (int l = 1; l <= 15; l++) {
        code |= (int)((v >> (l - 1)) & 1u);
        const int count = (int)inf_uni(cnt[l]);
        if (code - count < first) {
            *len = l;
            return (int)inf_uni(sym[index + (code - first)]);
        }
        index += count;
        first = (first + count) << 1;
        code <<= 1;
    }
    *len = 0;
    return -1;
}

// One symbol from P with the 2^FB-entry direct lookup (code-length tables)
template <int FB>
__device__ __forceinline__ int inf_decode(InfIn &b, const uint16_t *fast, const uint16_t *cnt, const uint16_t *sym) {
    const uint32_t e = inf_uni(fast[b.bits_at(b.P, FB)]);
    if (e) {
        b.P += e >> 9;
        return (int)(e & 511u);
    }
    int l;
    const int s = inf_walk_at(b, b.P, cnt, sym, &l);
    b.P += (uint64_t)l;
    return s;
}

// Canonical Huffman table from n code lengths, built by the lanes: 16
// per-length counts (LDS atomics), each length's first code and first symbol
// slot (one uniform pass over the 15 lengths), every symbol's rank among the
// lower-numbered symbols of its length (a ballot per length and chunk of
// kInfLanes symbols), then the symbols in code order and the 2^FB-entry
// direct lookup ((len << 9) | sym, 0: a longer code), a symbol per lane.
// `scr`: 64 words of LDS.  false: over-subscribed lengths (an incomplete
// code is accepted; its unused codes fail in inf_walk).
__device__ __forceinline__ uint32_t inf_ballot_below(bool p, int lane, uint32_t &tot) {
#if JP2HIP_INF_LANES > 1
    const uint64_t m = __ballot(p);
    tot = (uint32_t)__popcll(m);
    return (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
#else
    tot = p ? 1u : 0u;
    return 0u;
#endif
}
template <int FB, uint32_t EMPTY = 0u>
__device__ bool inf_build(uint16_t *cnt, uint16_t *sym, uint16_t *fast, const uint8_t *len, int n, int lane,
                          uint32_t *scr) {
    uint32_t *cl = scr, *offs = scr + 16, *next = scr + 32, *seen = scr + 48;
    for (int i = lane; i < 64; i += kInfLanes) scr[i] = 0u;
    const uint32_t e2 = EMPTY * 0x10001u;
    for (int i = lane; i < (1 << FB) / 8; i += kInfLanes) ((uint4 *)fast)[i] = make_uint4(e2, e2, e2, e2);
    __builtin_amdgcn_wave_barrier();
    for (int s = lane; s < n; s += kInfLanes)
        if (len[s]) atomicAdd(&cl[len[s]], 1u);
    __builtin_amdgcn_wave_barrier();
    int left = 1;
    uint32_t code = 0, off = 0;
    for (int l = 1; l < 16; l++) {
        const uint32_t c = inf_uni(cl[l]);
        left = (left << 1) - (int)c;
        if (lane == 0) {
            offs[l] = off;
            next[l] = code;
            cnt[l] = (uint16_t)c;
        }
        off += c;
        code = (code + c) << 1;
    }
    if (lane == 0) cnt[0] = 0;
    if (left < 0) return false;
    __builtin_amdgcn_wave_barrier();
    for (int s0 = 0; s0 < n; s0 += kInfLanes) {
        const int s = s0 + lane;
        const uint32_t l = s < n ? len[s] : 0u;
        uint32_t rank = 0;
        for (int q = 1; q < 16; q++) {
            uint32_t tot;
            const uint32_t below = inf_ballot_below(l == (uint32_t)q, lane, tot);
            if (tot) {
                if (l == (uint32_t)q) rank = seen[q] + below;
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) seen[q] += tot;
            }
        }
        if (l) {
            sym[offs[l] + rank] = (uint16_t)s;
            if ((int)l <= FB) {
                const uint32_t r = __builtin_bitreverse32(next[l] + rank) >> (32 - l);  // stream order: code MSB first
                for (uint32_t i = r; i < (1u << FB); i += 1u << l) fast[i] = (uint16_t)((l << 9) | (uint32_t)s);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    return true;
}

// The symbols of one Huffman block, a window of kInfLanes bit offsets at a
// time: lane l looks up the codes that would start at bit P + l (the
// literal/length table and the distance table, one LDS read each for the
// whole wave), then the walk follows the actual symbol boundaries through
// those lookups by readlane -- offset o, o + code length, ... -- with no
// memory access until the walk leaves the window.  Literals take a tight
// loop; a match's parts (length extra bits, distance code, distance extra
// bits) move to the next window whenever they start past this one.
// A run of literals is stored by the lanes that hold them (each lane's own
// table entry), at their ranks in the run; a match's links are stored by the
// lanes.
// Returns false on a corrupt stream; full = the strip is full.
__device__ __attribute__((noinline)) int inf_walk_slow(const InfIn &b, uint64_t q, const uint16_t *cnt,
                                                       const uint16_t *sym, int *len) {
    return inf_walk_at(b, q, cnt, sym, len);
}
__device__ bool inf_block(InfIn &b, InfShared &S, uint32_t *L, uint32_t cap, uint32_t &pos, bool &full, int lane) {
    uint32_t X = 0, Le = 0, De = 0, o = 0;
    // the window at P: this lane's 32 bits from P + lane and the two table
    // entries there
    auto window = [&]() {
        b.P += o;
        o = 0;
        b.ensure();
        const uint64_t q = b.P + (uint64_t)lane;
        const uint32_t kw = (uint32_t)(q >> 5) % kInRingWords;
        X = __builtin_amdgcn_alignbit(b.ring[(kw + 1) % kInRingWords], b.ring[kw], (uint32_t)(q & 31));
        Le = S.lfast[X & ((1u << kInfLB) - 1u)];
        De = S.dfast[X & ((1u << kInfDB) - 1u)];
    };
    window();
    for (;;) {
        // the walk's state is wave-uniform; say so (the compiler's divergence
        // analysis loses it through the stores of the lanes that hold literals)
        pos = inf_uni(pos);
        if (o >= (uint32_t)kInfLanes) {
            window();
            if (b.P > b.end_bits + 64) return false;  // far past the stream's end: truncated
        }
        // a run of literals inside this window: the walk only marks where
        // each starts (bit o of `run`); the lane at that offset already holds
        // the literal in its own table entry, and stores it at its rank in the
        // run (at most kInfLanes literals: each code is at least one bit)
        uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)Le, (int)o);
        if (!(e & 0x100u) && cap - pos >= (uint32_t)kInfLanes) {
            uint64_t run = 0;
            do {
                run |= 1ull << o;
                o += e >> 9;
                if (o >= (uint32_t)kInfLanes) break;
                e = (uint32_t)__builtin_amdgcn_readlane((int)Le, (int)o);
            } while (!(e & 0x100u));
            run = inf_uni64(run);
#if JP2HIP_INF_LANES > 1
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(run >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)run, 0u));
#else
            const uint32_t rank = 0u;
#endif
            if ((run >> lane) & 1ull) L[pos + rank] = kLinkByte | (Le & 255u);
            pos += (uint32_t)__popcll(run);
            if (o >= (uint32_t)kInfLanes) continue;
        } else if (!(e & 0x100u)) {  // near the strip's end: one literal at a time
            if (pos >= cap) {  // strip full: trailing data ignored
                full = true;
                b.P += o + (e >> 9);
                return true;
            }
            L[pos] = kLinkByte | (e & 255u);  // every lane stores the same word
            pos++;
            o += e >> 9;
            continue;
        }
        if (e == kInfNoFast) e = 0;  // (the walk below looks for 0)
        uint32_t cl = e >> 9, sy = e & 511u;
        if (!e) {  // a code longer than the direct lookup: walk it bit by bit
            int l;
            // (a call's results are per lane to the compiler: say they are uniform)
            const int ws = (int)inf_uni((uint32_t)inf_walk_slow(b, b.P + o, S.lcnt, S.lsym, &l));
            if (ws < 0) return false;
            cl = inf_uni((uint32_t)l);
            sy = (uint32_t)ws;
            if (sy < 256u) {  // (rare) a long literal code
                if (pos >= cap) {
                    full = true;
                    b.P += o + cl;
                    return true;
                }
                L[pos] = kLinkByte | sy;  // every lane stores the same word
                pos++;
                o += cl;
                continue;
            }
        }
        o += cl;
        if (sy == 256u) {  // end of block
            b.P += o;
            return true;
        }
        const uint32_t li = sy - 257u;
        if (li >= 29u) return false;
        if (o >= (uint32_t)kInfLanes) window();
        const uint32_t nl = inf_len_extra(li);
        uint32_t len = inf_len_base(li) + ((uint32_t)__builtin_amdgcn_readlane((int)X, (int)o) & ((1u << nl) - 1u));
        o += nl;
        if (o >= (uint32_t)kInfLanes) window();
        uint32_t ed = (uint32_t)__builtin_amdgcn_readlane((int)De, (int)o), dc = ed & 511u, dl = ed >> 9;
        if (!ed) {
            int l;
            const int ws = (int)inf_uni((uint32_t)inf_walk_slow(b, b.P + o, S.dcnt, S.dsym, &l));
            if (ws < 0) return false;
            dl = inf_uni((uint32_t)l);
            dc = (uint32_t)ws;
        }
        if (dc >= 30u) return false;
        o += dl;
        if (o >= (uint32_t)kInfLanes) window();
        const uint32_t nd = inf_dist_extra(dc);
        const uint32_t dist = inf_dist_base(dc) + ((uint32_t)__builtin_amdgcn_readlane((int)X, (int)o) & ((1u << nd) - 1u));
        o += nd;
        if (dist > pos) return false;
        bool cut = false;
        if (len > cap - pos) {  // the strip ends inside this match: keep what fits
            len = cap - pos;
            cut = true;
        }
        // each byte links to one before the match start (period dist when
        // the match overlaps itself)
        const uint32_t src = pos - dist;
        if (dist >= len) {
            for (uint32_t x = (uint32_t)lane; x < len; x += kInfLanes) L[pos + x] = src + x;
        } else {  // byte x repeats byte x mod dist before the match: one division per match
            uint32_t r = (uint32_t)lane % dist;
            const uint32_t step = (uint32_t)kInfLanes % dist;
            for (uint32_t x = (uint32_t)lane; x < len; x += kInfLanes) {
                L[pos + x] = src + r;
                r += step;
                r = r >= dist ? r - dist : r;
            }
        }
        pos += len;
        if (cut) {
            b.P += o;
            full = true;
            return true;
        }
    }
}

__global__ void __launch_bounds__(kInfLanes) k_inflate(UnpackArgs a) {
    __shared__ __attribute__((aligned(16))) InfShared S;
    const int s = blockIdx.x, lane = (int)threadIdx.x;
    if (s >= a.nstrips) return;
    // the strip's geometry as wave-uniform (scalar) values: everything the
    // decode derives from them stays scalar, and its branches too
    const uint8_t *in0 = a.src + inf_uni64(a.off[s]);
    const uint64_t n0 = inf_uni64(a.cnt[s]);
    const uint64_t cap64 = inf_uni64(strip_out_bytes(a, s));
    uint32_t *L = a.lnk + (uint64_t)s * a.stride;  // this strip's links
    if (cap64 >= (1ull << 31)) {  // a strip / tile of 2 GiB or more: not a TIFF the host parser accepts
        if (lane == 0) atomicOr(a.err, 2);
        return;
    }
    const uint32_t cap = (uint32_t)cap64;
    uint32_t pos = 0;
    const uint32_t h0 = inf_uni(n0 >= 1 ? in0[0] : 0u), h1 = inf_uni(n0 >= 2 ? in0[1] : 0u);
    bool bad = n0 < 2 || (h0 & 15) != 8 || (h0 >> 4) > 7 || ((h0 << 8) | h1) % 31 || (h1 & 0x20);
    InfIn b;
    b.init(in0, n0, S.ring, lane);
    b.P += 16;  // zlib CMF, FLG (checked above)
    bool last = false;
    while (!bad && !last) {
        b.ensure();
        last = b.get(1);
        const int type = (int)b.get(2);
        if (type == 0) {  // stored: to the byte boundary, LEN, ~LEN, then LEN bytes copied by the lanes
            b.align();
            uint32_t len = b.get(16);
            const uint32_t nlen = b.get(16);
            if (len != (~nlen & 0xFFFFu)) { bad = true; break; }
            const uint64_t at = b.consumed() / 8;  // the block's first byte in the stream
            if (at + len > n0) { bad = true; break; }     // truncated
            if (len > cap - pos) { len = cap - pos; last = true; }  // strip full: stop here
            for (uint32_t i = (uint32_t)lane; i < len; i += kInfLanes) L[pos + i] = kLinkByte | in0[at + i];
            pos += len;
            b.P += 8ull * len;
            continue;
        }
        if (type == 1) {  // fixed codes
            for (int i = lane; i < 318; i += kInfLanes)
                S.lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < 288 ? 8 : 5;
            __builtin_amdgcn_wave_barrier();
            inf_build<kInfLB, kInfNoFast>(S.lcnt, S.lsym, S.lfast, S.lens, 288, lane, S.scr);
            inf_build<kInfDB>(S.dcnt, S.dsym, S.dfast, S.lens + 288, 30, lane, S.scr);
        } else if (type == 2) {  // dynamic codes
            const int nlen = (int)b.get(5) + 257, ndist = (int)b.get(5) + 1, ncode = (int)b.get(4) + 4;
            if (nlen > 286 || ndist > 30) { bad = true; break; }
            b.ensure();
            for (int i = 0; i < 19; i++) {
                const uint32_t v = i < ncode ? b.get(3) : 0u;
                if (lane == 0) S.lens[kInfClOrder[i]] = (uint8_t)v;
            }
            __builtin_amdgcn_wave_barrier();
            if (!inf_build<7>(S.lcnt, S.lsym, S.lfast, S.lens, 19, lane, S.scr)) { bad = true; break; }
            int i = 0;
            while (i < nlen + ndist) {
                b.ensure();
                const int sy = inf_decode<7>(b, S.lfast, S.lcnt, S.lsym);
                if (sy < 0) { bad = true; break; }
                if (sy < 16) {
                    if (lane == 0) S.lens[i] = (uint8_t)sy;
                    i++;
                    continue;
                }
                uint32_t v = 0;
                int rep;
                if (sy == 16) {
                    if (i == 0) { bad = true; break; }
                    v = inf_uni(S.lens[i - 1]);
                    rep = 3 + (int)b.get(2);
                } else if (sy == 17) rep = 3 + (int)b.get(3);
                else rep = 11 + (int)b.get(7);
                if (i + rep > nlen + ndist) { bad = true; break; }
                for (int j = lane; j < rep; j += kInfLanes) S.lens[i + j] = (uint8_t)v;
                i += rep;
            }
            __builtin_amdgcn_wave_barrier();
            if (bad || inf_uni(S.lens[256]) == 0) { bad = true; break; }
            if (!inf_build<kInfLB, kInfNoFast>(S.lcnt, S.lsym, S.lfast, S.lens, nlen, lane, S.scr) ||
                !inf_build<kInfDB>(S.dcnt, S.dsym, S.dfast, S.lens + nlen, ndist, lane, S.scr)) {
                bad = true;
                break;
            }
        } else { bad = true; break; }
        __builtin_amdgcn_wave_barrier();
        bool full = false;
        if (!inf_block(b, S, L, cap, pos, full, lane)) { bad = true; break; }
        if (full) last = true;
    }
    bad = bad || b.P > b.end_bits;  // read past the end of the stream: truncated
    if (bad || pos != cap) {
        if (lane == 0) atomicOr(a.err, 2);
        // a strip that stopped short: its remaining links become known bytes
        // (0), so k_inflate_links never follows a stale or unwritten slot
        for (uint32_t i = pos + (uint32_t)lane; i < cap; i += kInfLanes) L[i] = kLinkByte;
    }
}

// Resolves every decoded strip's links (k_inflate) into its bytes: grid
// (chunks of kLinkChunk bytes, strips).  Rounds of pointer doubling first,
// one launch each (round < kLinkDoublings), then the last launch chases what
// is left of each chain and writes the bytes.  Links only point backwards
// within their strip, so every chain ends at a byte of known value.
constexpr int kLinkChunk = 4096;
__global__ void __launch_bounds__(256) k_inflate_links(UnpackArgs a, int chase) {
    const int s = blockIdx.y;
    const uint64_t cap64 = strip_out_bytes(a, s);
    if (cap64 >= (1ull << 31)) return;  // k_inflate refused the strip (error already set)
    const uint32_t cap = (uint32_t)cap64;
    uint32_t *L = a.lnk + (uint64_t)s * a.stride;
    uint8_t *out = a.dst + (uint64_t)s * a.stride;
    const uint32_t p0 = blockIdx.x * (uint32_t)kLinkChunk;
    // a well-formed link points strictly backwards; anything else (a corrupt
    // strip's slot) ends the chain, so every chase terminates in bounds
    for (uint32_t p = p0 + threadIdx.x; p < min(cap, p0 + (uint32_t)kLinkChunk); p += 256) {
        uint32_t v = L[p];
        if (!chase) {
            if (!(v & kLinkByte) && v < p) {
                const uint32_t u = L[v];
                if (u != v) L[p] = u;
            }
            continue;
        }
        uint32_t at = p;
        while (!(v & kLinkByte)) {
            if (v >= at) { v = kLinkByte; break; }
            at = v;
            v = L[v];
        }
        out[p] = (uint8_t)v;
    }
}

// Predictor 2: each sample adds the same component of the pixel to its left
// (modulo 2^bits, in the file's byte order for 16-bit samples).
__global__ void __launch_bounds__(256) k_unpredict(uint8_t *dst, int nrows, int rows_per_strip_buf, int rps, int h,
                                                    int per_plane, uint64_t stride, int w, int spp, int bits,
                                                    int big_endian) {
    const int r = blockIdx.x * 256 + threadIdx.x;  // global decoded row: strip * rps + row in strip
    if (r >= nrows) return;
    const int s = r / rows_per_strip_buf, y = r % rows_per_strip_buf;
    if ((s % per_plane) * rps + y >= h || y >= rps) return;
    const uint64_t rb = (uint64_t)w * spp * (bits >> 3);
    uint8_t *row = dst + (uint64_t)s * stride + (uint64_t)y * rb;
    if (bits == 8) {
        for (int i = spp; i < w * spp; i++) row[i] = (uint8_t)(row[i] + row[i - spp]);
    } else {
        auto rd = [&](int i) -> uint32_t {
            return big_endian ? ((uint32_t)row[2 * i] << 8) | row[2 * i + 1] : row[2 * i] | ((uint32_t)row[2 * i + 1] << 8);
        };
        for (int i = spp; i < w * spp; i++) {
            const uint32_t v = (rd(i) + rd(i - spp)) & 0xFFFFu;
            if (big_endian) { row[2 * i] = (uint8_t)(v >> 8); row[2 * i + 1] = (uint8_t)v; }
            else { row[2 * i] = (uint8_t)v; row[2 * i + 1] = (uint8_t)(v >> 8); }
        }
    }
}

// Tiled TIFF -> one row-major strip per plane: thread per pixel of a row.
// Tile t of plane p starts at base + (toff ? toff[t] : t * tstride).
__global__ void __launch_bounds__(256) k_untile(const uint8_t *base, const uint64_t *toff, uint64_t tstride, int w,
                                                 int h, int tw, int th, int across, int per_plane, int px_bytes,
                                                 uint8_t *out) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, p = blockIdx.z;
    if (x >= w) return;
    const int t = p * per_plane + (y / th) * across + x / tw;
    const uint8_t *src = base + (toff ? toff[t] : (uint64_t)t * tstride) +
                         ((uint64_t)(y % th) * tw + (x % tw)) * px_bytes;
    uint8_t *dst = out + (uint64_t)p * w * h * px_bytes + ((uint64_t)y * w + x) * px_bytes;
    for (int i = 0; i < px_bytes; i++) dst[i] = src[i];
}

// --------------------------------------------------------------------------
// S4: quantisation + bit-planes.  One wavefront per code-block; lane = column.
// Layout per block (uint64 words, lane c = column c, bit y = row y): B[p][64]
// for p < Mb, then sign[64].  (S[p] = OR_{q>=p} B[q], the significance state
// after plane p, is not stored: k_t1_cm3 walks the planes top-down and builds
// it as it goes.)
// --------------------------------------------------------------------------
constexpr int kZeroSpans = 9;
struct QuantArgs {
    const BlockDesc *blocks;
    const void *coef;
    int plane_w, plane_h, reversible;
    uint64_t *bp;
    int32_t *sm;
    uint8_t *P;
    int64_t *dref, *dsig;  // [block][32]
    uint32_t *est;         // [block][32] predicted coded size of plane p, 1/16 bit
    int max_mb;            // largest Mb of the plan (LDS: max_mb * 512 bytes per wave)
    int keep_sm;           // write the sign-magnitude copy of every block (debug dumps)
    int nblocks;
    // per-encode counters of later kernels, zeroed here (no memset launch):
    // dword spans, spread over the workgroups
    uint32_t *zero[kZeroSpans];
    uint32_t nzero[kZeroSpans];
};

constexpr int kQuantWaves = 2;  // code-blocks (waves) per workgroup
// The coefficient plane holds the quantisation indices the DWT wrote
// (sign-magnitude, 16-bit words when Q16: QuantTab::q16)
template <bool REV, bool Q16>
__global__ void __launch_bounds__(64 * kQuantWaves) k_quant(QuantArgs a) {
    extern __shared__ uint64_t lds_planes[];  // [wave][plane][lane], a.max_mb planes per wave
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.x * kQuantWaves + wv;
#pragma unroll
    for (int z = 0; z < kZeroSpans; z++)
        for (uint32_t i = blockIdx.x * 64 * kQuantWaves + threadIdx.x; i < a.nzero[z]; i += gridDim.x * 64 * kQuantWaves)
            a.zero[z][i] = 0u;
    if (b >= a.nblocks) return;
    uint64_t *planes = lds_planes + (size_t)wv * a.max_mb * 64;
    BlockDesc d = a.blocks[b];
    int lane = threadIdx.x & 63;
    bool act = lane < d.w;
    // the block's first row (wave-uniform: each row load is a scalar base +
    // the lane's column offset, no per-row address registers)
    const size_t e0 = (size_t)d.tc * a.plane_w * a.plane_h + (size_t)d.y0 * a.plane_w + d.x0;
    const int cl = act ? lane : 0;
    int32_t *sm = a.sm + d.sm_off + lane;
    // the sign-magnitude copy is read only by the 64-bit distortion path of
    // planes above 23 (below) and by the debug dumps
    const bool keep_sm = a.keep_sm || d.Mb > 24;
    uint32_t vmax = 0;
    // the lane's column stays in registers (sign | magnitude) for the
    // bit-plane and distortion passes: the indices are read from HBM once.
    // All 64 row loads are in flight at once; rows past the block end
    // re-read its last row and lanes past its width read column 0 -- values
    // of the block, so its maximum is unchanged -- and are cleared from the
    // bit-plane masks (`valid`), not row by row.
    uint32_t col[64];
    const int hm1 = d.h - 1;
    if constexpr (Q16) {
        const uint16_t *src = (const uint16_t *)a.coef + e0;
#pragma unroll
        for (int y = 0; y < 64; y++) col[y] = src[(size_t)min(y, hm1) * a.plane_w + cl];
    } else {
        const uint32_t *src = (const uint32_t *)a.coef + e0;
#pragma unroll
        for (int y = 0; y < 64; y++) col[y] = src[(size_t)min(y, hm1) * a.plane_w + cl];
    }
    // magnitudes in col[], the signs straight into the sign column (the sign
    // bit as stored: a -0.0 quantises to 0, and a zero's sign is never coded)
    constexpr int kSb = Q16 ? 15 : 31;
    uint32_t sg_lo = 0, sg_hi = 0;
#pragma unroll
    for (int y = 0; y < 64; y++) {
        const uint32_t raw = col[y];
        const uint32_t v = raw & ((1u << kSb) - 1u);
        if (y < 32) sg_lo |= (raw >> kSb) << y;
        else sg_hi |= (raw >> kSb) << (y - 32);
        col[y] = v;
        vmax = max(vmax, v);
    }
    const uint64_t hmask = d.h >= 64 ? ~0ull : ((1ull << d.h) - 1ull);
    const uint64_t valid = act ? hmask : 0ull;  // rows < h of columns < w
    const uint64_t sgcol = (((uint64_t)sg_hi << 32) | sg_lo) & valid;
    if (keep_sm) {
#pragma unroll
        for (int y = 0; y < 64; y++)
            if (y < d.h) sm[y * 64] = act ? (int32_t)(col[y] | (uint32_t)((sgcol >> y) & 1u) << 31) : 0;
    }
    // the magnitude bits of the block = those of the OR of its magnitudes
    // (a DPP reduction; uniform: P and the plane loop stay scalar)
    vmax = wave_or_u32(vmax);
    const int P = __builtin_amdgcn_readfirstlane(vmax ? 32 - __clz(vmax) : 0);
    if (lane == 0) a.P[b] = (uint8_t)P;
    // column masks (lane c, bit y = row y): BT[p][c] = bit p of the
    // column, then the sign column SGT[c] -- the layout the tier-1 context
    // modelling reads (t1.hip k_t1_cm3)
    uint64_t *BT = a.bp + d.bp_off;
    uint64_t *SGT = BT + (size_t)d.Mb * 64;
    SGT[lane] = sgcol;
    // every plane's column mask, kept in LDS for the distortion sums below.
    // Four planes at a time: a row's 4 bits are spread to the 4 bytes of a
    // word by one multiply (nib * 0x204081 & 0x01010101), so G[g] collects
    // rows 8g..8g+7 with plane p0+k in byte k; each plane's 64-bit mask is
    // then byte k of G[0..7], gathered by v_perm_b32 (4 ops per row group of
    // 4 planes instead of 2 per row and plane)
    for (int p0 = 0; p0 < P; p0 += 4) {
        uint32_t G[8];
#pragma unroll
        for (int g = 0; g < 8; g++) {
            uint32_t acc = 0;
#pragma unroll
            for (int i = 0; i < 8; i++)
                acc |= (__umul24(__builtin_amdgcn_ubfe(col[8 * g + i], (uint32_t)p0, 4u), 0x00204081u) & 0x01010101u) << i;
            G[g] = acc;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int p = p0 + k;
            if (p >= P) break;
            // bytes k of (G0, G1) and (G2, G3) -> low halves; the pair merged
            const uint32_t sel = (uint32_t)k | ((uint32_t)(k + 4) << 8) | 0x0C0C0000u;
            const uint32_t lo = __builtin_amdgcn_perm(G[1], G[0], sel) | (__builtin_amdgcn_perm(G[3], G[2], sel) << 16);
            const uint32_t hi = __builtin_amdgcn_perm(G[5], G[4], sel) | (__builtin_amdgcn_perm(G[7], G[6], sel) << 16);
            const uint64_t m = (((uint64_t)hi << 32) | lo) & valid;
            planes[p * 64 + lane] = m;
            BT[(size_t)p * 64 + lane] = m;
        }
    }
    constexpr bool lossless = REV;
    constexpr int dd = lossless ? 0 : 1;  // reconstruction offset, half-units
    const bool wcol = lane < d.w;
    uint64_t colS = 0;       // S[p+1] of this column
    uint32_t cnt_above = 0;  // |S[p+1]| over the block
    // Planes top-down.  Distortion decreases of plane p (oracle dist_gain,
    // half-units, d = reconstruction offset): a sample whose top bit is p
    // gains 2^p (12 v + 6d - 9 2^p); one significant above p, with l = v mod
    // 2^p, gains 2^p (4l + 2d - 2^p) if bit p is set, else 2^p (3 2^p - 4l -
    // 2d); lossless p = 0 gains 4 for a new sample and for a refined 0 bit,
    // nothing else.  The sums of v over new samples (N) and of +-l over
    // refined ones (R1: bit p set, R0: clear) come from the column masks:
    // sum_N v = sum_{q<=p} 2^q |N & B[q]|, sum_R +-l = sum_{q<p} 2^q (|R1 &
    // B[q]| - |R0 & B[q]|), int32 per lane up to p = 23.  The slope-prediction
    // counts (oracle plane_stats): significant samples, and insignificant
    // samples with a significant 8-neighbour.
    for (int p = P - 1; p >= 0; p--) {
        const uint64_t Bp = planes[p * 64 + lane];
        const uint64_t N = Bp & ~colS, R1 = colS & Bp;
        uint32_t nb1 = (uint32_t)__popcll(R1);  // refined samples with bit p set
        int64_t ref = 0, sig = 0;
        int32_t sv = 0, sl = 0;
        if (p <= 23) {
            sv = __popcll(N) << p;
            for (int q = 0; q < p; q++) {
                const uint64_t Bq = planes[q * 64 + lane];
                sv += __popcll(N & Bq) << q;
                sl += (2 * __popcll(R1 & Bq) - __popcll(colS & Bq)) * (1 << q);
            }
        } else {
            // 64-bit gains per row, the column re-read from the sign-magnitude
            // copy (never for <= 16-bit sources)
            for (int y = 0; y < d.h; y++) {
                const uint32_t v = (uint32_t)sm[y * 64] & 0x7FFFFFFFu;
                const uint32_t hi = v >> p;
                if (hi == 0) continue;
                const int64_t g = dist_gain(v, p, lossless);
                if (hi == 1) sig += g;
                else ref += g;
            }
        }
        colS |= Bp;
        // insignificant samples with a significant 8-neighbour (rows < h,
        // columns < w)
        // (DPP whole-wave shifts on every lane: lanes 0 / 63 receive 0)
        const uint64_t Lc = wave_shr1(colS), Rc = wave_shl1(colS);
        const uint64_t H = colS | Lc | Rc;
        uint32_t cN = wcol ? (uint32_t)__popcll((H | (H << 1) | (H >> 1)) & ~colS & hmask) : 0u;
        uint32_t cS = (uint32_t)__popcll(colS);
        // wave totals by DPP scans; cS and cN (<= 4096 each) share one scan
        {
            const uint32_t both = wave_sum_u32(cS | (cN << 16));
            cS = both & 0xFFFFu;
            cN = both >> 16;
            nb1 = wave_sum_u32(nb1);
        }
        if (p <= 23) {
            const int64_t SV = wave_sum64(sv), SL = wave_sum64(sl);
            const int64_t n1 = cS - cnt_above, nr1 = nb1, nr0 = cnt_above - nb1, q = (int64_t)1 << p;
            if (lossless && p == 0) {
                sig = 4 * n1;
                ref = 4 * nr0;
            } else {
                sig = q * (12 * SV + (6 * dd - 9 * q) * n1);
                ref = q * (4 * SL + nr1 * (2 * dd - q) + nr0 * (3 * q - 2 * dd));
            }
        } else {
            ref = wave_sum64(ref);
            sig = wave_sum64(sig);
        }
        if (lane == 0) {
            a.est[(size_t)b * 32 + p] = 16u * cnt_above + 56u * (cS - cnt_above) + 5u * cN;
            a.dref[(size_t)b * 32 + p] = ref;
            a.dsig[(size_t)b * 32 + p] = sig;
        }
        cnt_above = cS;
    }
}

// --------------------------------------------------------------------------
// S4b: slope prediction (rate-driven encodes; oracle/jp2_oracle.c
// predict_and_code).  kdu_compress "-rate" (KakaduConverter.java:44) stops
// its block coder at a predicted slope threshold instead of coding passes
// PCRD-opt will discard.  Plane p of a block has predicted slope
// pd * weight / est; est is histogrammed over 1/8-octave slope bins, the bin
// where the predicted size reaches the target fixes the cut, and planes more
// than kSkipMargin bins below it are not coded (pmin = lowest coded plane).
// All integer after the one IEEE division, so the oracle agrees bit for bit.
// --------------------------------------------------------------------------
__device__ __forceinline__ int slope_bin(double s) {
    if (!(s > 0.0)) return -1;
    const uint64_t k = (uint64_t)__double_as_longlong(s);
    const int b = (int)(k >> 49) - kSlopeBinBase;
    return b < 0 ? 0 : (b >= kSlopeBins ? kSlopeBins - 1 : b);
}
__device__ __forceinline__ int plane_bin(int64_t pd, double wgt, uint32_t est) {
    if (est == 0) return pd > 0 ? kSlopeBins - 1 : -1;
    return slope_bin((double)pd * wgt / (double)est);
}

struct PredictArgs {
    int nblocks;
    const uint8_t *P;
    const int64_t *dref, *dsig;
    const uint32_t *est;
    const double *weight;
    unsigned long long *hist;  // [kSlopeBins]
    int *kcut;
    uint8_t *pmin;
};

// Thread per block, its planes in a loop (a thread per (block, plane) slot
// left most lanes idle: 32 slots for ~12 planes); a workgroup covers
// kHistBlocks consecutive blocks, whose planes land in few bins, so it sums
// into an LDS histogram and flushes only the bins it touched.
constexpr int kHistBlocks = 1024;
__global__ void __launch_bounds__(256) k_plane_hist(PredictArgs a) {
    __shared__ unsigned long long lh[kSlopeBins];
    for (int i = threadIdx.x; i < kSlopeBins; i += 256) lh[i] = 0;
    __syncthreads();
    const int b0 = blockIdx.x * kHistBlocks;
    const int b1 = min(a.nblocks, b0 + kHistBlocks);
    for (int b = b0 + (int)threadIdx.x; b < b1; b += 256) {
        const int Pb = a.P[b];
        const double wb = a.weight[b];
        const size_t i0 = (size_t)b * 32;
        // the next plane's three loads in flight while this one is binned
        int64_t dd = Pb > 0 ? a.dref[i0] + a.dsig[i0] : 0;
        uint32_t e = Pb > 0 ? a.est[i0] : 0u;
        for (int p = 0; p < Pb; p++) {
            const int pn = min(p + 1, 31);
            const int64_t ddn = a.dref[i0 + pn] + a.dsig[i0 + pn];
            const uint32_t en = a.est[i0 + pn];
            const int k = plane_bin(dd, wb, e);
            if (k >= 0) atomicAdd(&lh[k], (unsigned long long)e);
            dd = ddn;
            e = en;
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kSlopeBins; k += 256)
        if (lh[k]) atomicAdd(&a.hist[k], lh[k]);
}

// kstar = #{k in [1, kSlopeBins) : sum_{j >= k} hist[j] >= goal} (the
// oracle's downward scan), kcut = kstar - kSkipMargin.  One wave; lane l owns
// bins [16 l, 16 l + 16).
__device__ __forceinline__ int plane_cut(const unsigned long long *hist, int64_t goal) {
    const int lane = threadIdx.x & 63;
    constexpr int kPer = kSlopeBins / 64;
    unsigned long long h[kPer], part = 0;
#pragma unroll
    for (int i = 0; i < kPer; i++) { h[i] = hist[lane * kPer + i]; part += h[i]; }
    // exclusive suffix sum over lanes: bins above this lane's range
    const uint64_t inc = wave_incl_scan64(part);
    const unsigned long long above =
        (uint64_t)__shfl((long long)inc, 63, 64) - inc;
    int cnt = 0;
    unsigned long long acc = above;
#pragma unroll
    for (int i = kPer - 1; i >= 0; i--) {
        acc += h[i];
        const int k = lane * kPer + i;
        cnt += (k >= 1 && acc >= (unsigned long long)goal) ? 1 : 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    return cnt - kSkipMargin;
}

// the lowest coded plane of each block, then its items in tier-1's work lists
// (every workgroup finds the cut from the histogram itself: no launch for it)
__global__ void __launch_bounds__(256) k_plane_pmin(PredictArgs a, T1ItemArgs ia, int64_t goal) {
    __shared__ int kcut;
    __shared__ ItemScratch sc;
    if (threadIdx.x < 64) {
        const int kc = plane_cut(a.hist, goal);
        if (threadIdx.x == 0) kcut = kc;
    }
    __syncthreads();
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = b < a.nblocks;
    const int P = in ? a.P[b] : 0;
    int pmin = P > 0 ? P - 1 : 0;
    if (in) {
        const int kc = kcut;
        const double wgt = a.weight[b];
        // planes 8 at a time: their loads in flight together
        bool found = false;
        for (int p0 = 0; p0 < P && !found; p0 += 8) {
            int64_t dd[8];
            uint32_t e[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const size_t i = (size_t)b * 32 + min(p0 + j, 31);
                dd[j] = a.dref[i] + a.dsig[i];
                e[j] = a.est[i];
            }
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (!found && p0 + j < P && plane_bin(dd[j], wgt, e[j]) >= kc) {
                    pmin = p0 + j;
                    found = true;
                }
        }
        a.pmin[b] = (uint8_t)pmin;
    }
    emit_t1_items<256>(ia, b, in, P, pmin, sc);
}

// --------------------------------------------------------------------------
// S6: PCRD-opt.  Hull per block (thread per block, k_hull), which also
// histograms every hull segment's bytes over kPcrdBins slope-key bins; then
// k_select finds each layer's threshold: the bin its budget falls in from the
// histogram, the exact key inside that bin by a radix select over the
// segments of that bin only (no sort of all segments).
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
    int64_t *hdist;   // [block][kMaxPasses+1] HullPt: the stack's distortion and rate at each point
    unsigned long long *hbytes;  // [group][kPcrdBins] segment bytes per slope bin (zeroed by k_quant)
    uint32_t *hcount;            // [group][kPcrdBins] segments per slope bin
    const int32_t *grp_b0;       // rate-control groups' block ranges (Plan::grp_b0): grid.y = group
    unsigned long long *gtot;    // [group] tier-1 bytes (lossless budgets; zeroed by k_quant)
    // the tier-1 totals of T2Summary (t1_bytes, coded_passes, decisions,
    // skipped; zeroed by k_quant), summed here once per encode instead of by
    // every rate iteration's totals
    const int32_t *lengths;
    const unsigned long long *acc;
    const uint8_t *pmin;
    T2Summary *sum;
};

// slope-key bin: monotone in the key (positive doubles order like their bits)
__device__ __forceinline__ int pcrd_bin(uint64_t key) {
    const int b = (int)(key >> 47) - kPcrdBinBase;
    return b < 0 ? 0 : (b >= kPcrdBins ? kPcrdBins - 1 : b);
}

// hull stack entry beside the output arrays (pass index, slope key): the
// cumulative distortion and the rate at the point, so a pop is one round
// trip (no pass-index -> rate chain)
struct HullPt {
    int64_t d;
    int32_t r, pad;
};
static_assert(sizeof(HullPt) == 16, "HullPt layout");

__device__ __forceinline__ void hull_one(const HullArgs &a, int b, uint32_t *lb, uint32_t *lc) {
    const int np = a.npasses[b];
    const int32_t *R = a.rates + (size_t)b * kMaxPasses;
    const int64_t *Dd = a.dists + (size_t)b * kMaxPasses;
    uint8_t *hp = a.hpass + (size_t)b * (kMaxPasses + 1);
    uint64_t *hk = a.hkey + (size_t)b * (kMaxPasses + 1);
    // the hull stack lives in the output arrays themselves plus hs, so the
    // lane keeps no per-pass arrays (no scratch memory); its top entry (key,
    // cumulative distortion, rate) also lives in registers, so only a pop
    // reads the stack back
    HullPt *hs = (HullPt *)a.hdist + (size_t)b * (kMaxPasses + 1);
    const double wgt = a.weight[b];
    int nh = 1;
    hp[0] = 0;
    hk[0] = 0;
    uint64_t tk = 0;
    int64_t td = 0;
    int32_t tr = 0;
    int64_t Dn = 0;
    // The workgroup's slope-bin histogram follows the stack: a push adds its
    // segment (key, bytes), a pop takes it back out, so what remains is the
    // final hull's segments (no pass over the hull afterwards)
    auto seg = [&](uint64_t key, int32_t bytes, int sign) {
        const int bn = pcrd_bin(key);
        atomicAdd(&lb[bn], (uint32_t)(sign * bytes));
        atomicAdd(&lc[bn], (uint32_t)sign);
    };
    // passes 8 at a time: their rate and distortion loads in flight together
    for (int n0 = 0; n0 < np; n0 += 8) {
        int32_t r8[8];
        int64_t d8[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int i = min(n0 + j, np - 1);
            r8[j] = R[i];
            d8[j] = Dd[i];
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int n = n0 + j + 1;
            if (n > np) break;
            const int32_t Rn = r8[j];
            Dn += d8[j];
            for (;;) {
                const int64_t dD = Dn - td;
                const int32_t dR = Rn - tr;
                bool pop = false;
                double s = 0.0;
                if (dD <= 0) break;
                if (dR <= 0) pop = true;
                else {
                    s = (double)dD * wgt / (double)dR;
                    pop = nh >= 2 && s >= __longlong_as_double((long long)tk);
                }
                if (pop) {
                    nh--;
                    const int32_t rpop = tr;
                    const uint64_t kpop = tk;
                    if (nh <= 1) {
                        tk = 0;
                        td = 0;
                        tr = 0;
                    } else {
                        const HullPt e = hs[nh - 1];
                        tk = hk[nh - 1];
                        td = e.d;
                        tr = e.r;
                    }
                    seg(kpop, rpop - tr, -1);
                    continue;
                }
                seg((uint64_t)__double_as_longlong(s), Rn - tr, 1);
                tk = (uint64_t)__double_as_longlong(s);
                td = Dn;
                tr = Rn;
                hp[nh] = (uint8_t)n;
                hk[nh] = tk;
                hs[nh].d = Dn;
                hs[nh].r = Rn;
                nh++;
                break;
            }
        }
    }
    a.nhull[b] = (uint8_t)nh;
}

constexpr int kHullThreads = 256;
__global__ void __launch_bounds__(kHullThreads) k_hull(HullArgs a) {
    // a workgroup's bytes per bin fit 32 bits (256 blocks of < 100 KB; the
    // pops' transient negatives wrap and cancel): 32 KB of LDS, not 48
    __shared__ uint32_t lb[kPcrdBins];
    __shared__ uint32_t lc[kPcrdBins];
    for (int i = threadIdx.x; i < kPcrdBins; i += kHullThreads) {
        lb[i] = 0;
        lc[i] = 0;
    }
    __syncthreads();
    const int g = blockIdx.y, gb1 = a.grp_b0[g + 1];
    const int b = a.grp_b0[g] + blockIdx.x * kHullThreads + threadIdx.x;
    if (a.grp_b0[g] + blockIdx.x * kHullThreads >= gb1) return;  // (the whole workgroup)
    int64_t tb = 0, tp = 0, nd = 0;
    bool sk = false;
    if (b < gb1) {
        hull_one(a, b, lb, lc);
        tb = a.lengths[b];
        tp = a.npasses[b];
        nd = (int64_t)(a.acc[b] & ((1ull << 40) - 1ull));  // decisions (k_t1_cm3)
        sk = a.pmin[b] > 0;
    }
    tb = wave_sum64(tb);
    tp = wave_sum64(tp);
    nd = wave_sum64(nd);
    sk = __any(sk);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&a.gtot[g], (unsigned long long)tb);
        atomicAdd((unsigned long long *)&a.sum->t1_bytes, (unsigned long long)tb);
        atomicAdd((unsigned long long *)&a.sum->coded_passes, (unsigned long long)tp);
        atomicAdd((unsigned long long *)&a.sum->decisions, (unsigned long long)nd);
        if (sk) atomicOr(&a.sum->skipped, 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kPcrdBins; i += kHullThreads)
        if (lc[i]) {
            atomicAdd(&a.hbytes[(size_t)g * kPcrdBins + i], (unsigned long long)lb[i]);
            atomicAdd(&a.hcount[(size_t)g * kPcrdBins + i], lc[i]);
        }
}


// Layer thresholds.  The oracle's rule (oracle/jp2_oracle.c select_threshold)
// is: walk hull segments in decreasing slope-key order, group equal keys, and
// take whole groups while the running byte total fits the budget.  With
// S(k) = bytes of the segments whose key >= k (non-increasing), that takes
// exactly the keys >= K' = min { k : S(k) <= budget } (split.cpp), and K' is
// one above the first key not taken -- the rule's Kc (Kdu-Layer-Info).
//
// Two launches, no sort:
//  1. every workgroup of both: suffix sums of the k_hull bin histogram; per
//     layer the bin b whose segments straddle the budget (S over the bins
//     above b fits, with b's bytes it does not);
//  2. k_select, thread per code-block: the hull segments whose key falls in
//     one of those bins are appended to that bin's candidate list;
//  3. k_select_resolve, a workgroup per layer: the largest key v with (bytes
//     above the bin) + (candidate bytes with key >= v) > budget is the first
//     key not taken, K' = v + 1.
// The list fill counters are zeroed by k_quant and left zero by
// k_select_resolve for the next k_select (the device rate loop runs several).
struct SelectArgs {
    const int *halt;  // device rate loop: nothing to do once it has stopped
    // device rate loop, first iteration: the budgets come from `init` (every
    // workgroup derives them), and k_select's workgroup 0 writes the loop's
    // state and budgets (what a separate init launch did)
    int init_on;
    RateState init;
    RateState *rs;
    int64_t *budget_w;
    int nblocks, layers;
    const uint8_t *nhull, *hpass;
    const uint64_t *hkey;
    const int32_t *rates;
    // rate-control groups (grid.y = group): block ranges, first candidate
    // slot (the bound on the hull segments of the groups before), and per
    // group: histogram kPcrdBins apart, budgets / thresholds kMaxLayers
    // apart, list fills kMaxLayers + 1 apart
    const int32_t *grp_b0;
    const uint32_t *grp_seg0;
    const unsigned long long *hbytes;
    const uint32_t *hcount;
    const int64_t *budget;
    // lossless: group g's layer-l budget is gtot[g] * frac[l] >> 16 (the
    // group's tier-1 bytes, k_hull), not budget[]
    int lossless;
    const unsigned long long *gtot;
    int32_t frac[kMaxLayers];
    uint64_t *lkey;   // candidate lists, capacity >= every hull segment
    uint32_t *lsize;
    uint32_t *ctl;    // [group][1 + i] fill of list i ([0] unused)
    uint64_t *K, *Kc;
    int64_t *dbg;     // debug builds: [0] lists, [1 + i] list sizes, [33 + l] rounds, [65 + l] survivors
};

// 256 threads a workgroup (4 waves): under load a 1 024-thread workgroup
// waits for 16 free wave slots on one CU
constexpr int kSelThreads = 256, kSelBrute = 64;
constexpr int kSelPer = kPcrdBins / kSelThreads;  // bins per thread in the scans
// k_select_resolve narrows a layer's key range 1 024 ways per round
constexpr int kResLog2 = 10, kResBins = 1 << kResLog2, kResPer = kResBins / kSelThreads;
// phase 1, run by every workgroup of both kernels (a few microseconds; no
// hand-off through memory): suffix sums of the bin histogram, per layer the
// bin and what it must supply, one candidate list per distinct bin
struct SelBins {
    uint64_t csfx[kSelThreads + 1];     // bytes of the bins >= kSelPer * t (t = 0 .. kSelThreads)
    uint64_t wsum[kSelThreads / 64 + 1];
    int lbin[kMaxLayers], lli[kMaxLayers];
    int64_t lneed[kMaxLayers];          // budget - bytes above the bin
    int list_bin[kMaxLayers];
    uint32_t list_off[kMaxLayers + 1];
    int nlist;
};
// The suffix sums are kept per thread chunk (kSelPer bins), 2 KB of LDS
// instead of a 32 KB table per bin (and no 4 KB bin -> list map): a layer's
// bin is found by a binary search over the chunks, then a walk down its
// chunk's bins (re-read from L2).
__device__ __forceinline__ void select_bins(const SelectArgs &a, SelBins &sh, int g) {
    const int tid = threadIdx.x, L = a.layers;
    const unsigned long long *hbytes = a.hbytes + (size_t)g * kPcrdBins;
    const uint32_t *hcount = a.hcount + (size_t)g * kPcrdBins;
    uint64_t *csfx = sh.csfx;
    int *lbin = sh.lbin, *lli = sh.lli, *list_bin = sh.list_bin;
    int64_t *lneed = sh.lneed;
    uint32_t *list_off = sh.list_off;
    {
        uint64_t s = 0;
#pragma unroll
        for (int i = 0; i < kSelPer; i++) s += hbytes[kSelPer * tid + i];
        uint64_t tot;
        const uint64_t pre = wg_excl_scan64<kSelThreads>(s, sh.wsum, tot);
        csfx[tid] = tot - pre;
        if (tid == 0) csfx[kSelThreads] = 0;
    }
    __syncthreads();
    if (tid < L) {
        // (a negative budget takes nothing, as 0 does: every segment has bytes)
        const int64_t B = a.init_on    ? (a.init.budget < 0 ? 0 : a.init.budget) >> (L - 1 - tid)
                          : a.lossless ? (int64_t)((a.gtot[g] * (unsigned long long)a.frac[tid]) >> 16)
                                       : a.budget[(size_t)g * kMaxLayers + tid];
        const int64_t T = B < 0 ? 0 : B;
        int b = -1;
        int64_t above = 0;  // S(b + 1)
        if ((int64_t)csfx[0] > T) {
            // the largest chunk whose suffix sum exceeds T ...
            int lo = 0, hi = kSelThreads - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if ((int64_t)csfx[mid] > T) lo = mid;
                else hi = mid - 1;
            }
            // ... then its largest bin b with S(b) > T
            uint64_t S = csfx[lo + 1];
            for (int i = kSelPer - 1; i >= 0; i--) {
                const uint64_t Sb = S + hbytes[kSelPer * lo + i];
                if ((int64_t)Sb > T) {
                    b = kSelPer * lo + i;
                    break;
                }
                S = Sb;
            }
            above = (int64_t)S;
        }
        lbin[tid] = b;
        lneed[tid] = b < 0 ? 0 : T - above;
    }
    __syncthreads();
    if (tid == 0) {  // one candidate list per distinct bin
        int n = 0;
        uint32_t o = 0;
        for (int l = 0; l < L; l++) {
            if (lbin[l] < 0) continue;
            int i = 0;
            while (i < n && list_bin[i] != lbin[l]) i++;
            if (i == n) {
                list_bin[n] = lbin[l];
                list_off[n] = o;
                o += hcount[lbin[l]];
                n++;
            }
            lli[l] = i;
        }
        list_off[n] = o;
        sh.nlist = n;
    }
    __syncthreads();
}

__global__ void __launch_bounds__(kSelThreads) k_select(SelectArgs a) {
    __shared__ SelBins sh;
    const int tid = threadIdx.x, lane = tid & 63, g = blockIdx.y;
    if (!a.init_on && a.halt && *a.halt) return;
    const int gb0 = a.grp_b0[g], gb1 = a.grp_b0[g + 1];
    if (a.init_on && blockIdx.x == 0 && g == 0 && tid == 0) {  // the rate loop's state (rate_step continues it)
        RateState r = a.init;
        r.it = 0;
        r.halt = 0;
        r.safety = 0;
        r.iters = 0;
        r.cs_bytes = 0;
        if (r.budget < 0) r.budget = 0;
        *a.rs = r;
        rate_budgets(r, a.layers, a.budget_w);
    }
    if (gb0 + (int)blockIdx.x * kSelThreads >= gb1) return;  // (the whole workgroup)
    select_bins(a, sh, g);
    const uint32_t *list_off = sh.list_off;
    const int *list_bin = sh.list_bin;
    const int nlist = sh.nlist;
    const uint32_t seg0 = a.grp_seg0[g];
    uint32_t *ctl = a.ctl + (size_t)g * (kMaxLayers + 1);
    // 2. candidates of those bins, thread per code-block of the group
    if (nlist > 0)
        for (int b = gb0 + blockIdx.x * kSelThreads + tid; b < gb1; b += gridDim.x * kSelThreads) {
            const int nh = a.nhull[b];
            const uint8_t *hp = a.hpass + (size_t)b * (kMaxPasses + 1);
            const uint64_t *hk = a.hkey + (size_t)b * (kMaxPasses + 1);
            const int32_t *R = a.rates + (size_t)b * kMaxPasses;
            for (int i0 = 1; i0 < nh; i0 += 8) {  // 8 keys' loads in flight together
                uint64_t k8[8];
#pragma unroll
                for (int j = 0; j < 8; j++) k8[j] = hk[min(i0 + j, nh - 1)];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int i = i0 + j;
                    const uint64_t key = k8[j];
                    int li = -1;
                    if (i < nh) {
                        const int bn = pcrd_bin(key);
                        for (int q = 0; q < nlist; q++) li = list_bin[q] == bn ? q : li;
                    }
                    // one fill atomic per wave and list (a list's lanes take
                    // consecutive slots): same-word atomics serialise in L2
                    uint64_t todo = __ballot(li >= 0);
                    while (todo) {
                        const int lead = __builtin_ctzll(todo);
                        const int lj = __shfl(li, lead, 64);
                        const uint64_t grp = __ballot(li == lj);
                        uint32_t base = 0;
                        if (lane == lead) base = atomicAdd(&ctl[1 + lj], (uint32_t)__popcll(grp));
                        base = (uint32_t)__shfl((int)base, lead, 64);
                        if (li == lj) {
                            const uint32_t at =
                                seg0 + list_off[lj] + base + (uint32_t)__popcll(grp & ((1ull << lane) - 1ull));
                            a.lkey[at] = key;
                            a.lsize[at] = (uint32_t)(R[hp[i] - 1] - (hp[i - 1] ? R[hp[i - 1] - 1] : 0));
                        }
                        todo &= ~grp;
                    }
                }
            }
        }
}

// 3. each layer in a workgroup of its own (grid = layers): the largest
// candidate key v with (bytes above the bin) + (candidate bytes with key >= v)
// > budget is the first key not taken, K' = v + 1.  Workgroup 0 also zeroes
// the list fill counters for the next k_select (the device rate loop runs
// several).  (Folded into k_select -- its group's last workgroup to finish
// resolving the layers, after a device-scope release/acquire count -- the
// pair took 104.5 us alone instead of 53 + 23 with the layers in turn, and
// 116.9 with a wave per layer, 4x longer candidate walks per wave; the C2
// bench did not move: profiles/r05/ab_select_fold.txt.)
__global__ void __launch_bounds__(kSelThreads) k_select_resolve(SelectArgs a) {
    __shared__ SelBins sh;
    // the narrowing state and the survivors
    __shared__ uint64_t rlo, rhi, rmax;
    __shared__ int64_t rneed;
    __shared__ uint32_t rcount;
    __shared__ uint64_t bkey[kSelBrute];
    __shared__ uint32_t bsize[kSelBrute];
    __shared__ uint64_t hist[kResBins];
    __shared__ uint32_t hcnt[kResBins];
    const int tid = threadIdx.x, lane = tid & 63, l = blockIdx.x, g = blockIdx.y;
    if (a.halt && *a.halt) return;  // (k_select has reset it on a first iteration)
    select_bins(a, sh, g);
    uint64_t *wsum = sh.wsum;
    const int *lbin = sh.lbin, *lli = sh.lli;
    const int64_t *lneed = sh.lneed;
    const uint32_t *list_off = sh.list_off;
    const int nlist = sh.nlist;
    const uint32_t seg0 = a.grp_seg0[g];
    uint64_t *Kg = a.K + (size_t)g * kMaxLayers, *Kcg = a.Kc + (size_t)g * kMaxLayers;
    if (l == 0 && tid <= nlist) a.ctl[(size_t)g * (kMaxLayers + 1) + tid] = 0u;  // (k_select has finished: stream order)
    if (a.dbg && l == 0 && g == 0 && tid == 0) {
        a.dbg[0] = nlist;
        for (int i = 0; i < nlist; i++) a.dbg[1 + i] = list_off[i + 1] - list_off[i];
    }
    // The key range is narrowed by
    // 1 024-way histograms (bytes and counts) over the candidates in range --
    // a bin is 2^47 keys wide, one round leaves a handful (a round starts
    // from the bin's own bounds and count: no pass for them) -- until at most
    // kSelBrute remain, whose totals are then summed directly.
    {
        if (lbin[l] < 0) {
            if (tid == 0) Kg[l] = Kcg[l] = 0ull;  // every segment fits
            return;
        }
        const int li = lli[l];
        const uint32_t i0 = seg0 + list_off[li], i1 = seg0 + list_off[li + 1];
        const int bn = lbin[l];
        if (tid == 0) {
            rcount = i1 - i0;
            rneed = lneed[l];
            if (bn > 0 && bn < kPcrdBins - 1) {
                rlo = (uint64_t)(bn + kPcrdBinBase) << 47;
                rhi = rlo + ((1ull << 47) - 1ull);
            } else {  // a clamped end bin: the candidates' own key range
                rlo = ~0ull;
                rhi = 0ull;
            }
        }
        __syncthreads();
        if (rlo > rhi) {
            uint64_t mn = ~0ull, mx = 0ull;
            for (uint32_t i = i0 + tid; i < i1; i += kSelThreads) {
                const uint64_t k = a.lkey[i];
                mn = min(mn, k);
                mx = max(mx, k);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                mn = min(mn, (uint64_t)__shfl_xor((long long)mn, o, 64));
                mx = max(mx, (uint64_t)__shfl_xor((long long)mx, o, 64));
            }
            if (lane == 0) {
                atomicMin((unsigned long long *)&rlo, (unsigned long long)mn);
                atomicMax((unsigned long long *)&rhi, (unsigned long long)mx);
            }
            __syncthreads();
        }
        for (int round = 0;; round++) {
            const uint64_t flo = rlo, fhi = rhi;
            const uint32_t cnt = rcount;
            const int64_t need = rneed;
            if (flo == fhi || cnt <= (uint32_t)kSelBrute) {
                // survivors: v = the largest key whose total exceeds need
                __syncthreads();
                if (tid == 0) {
                    rcount = 0;
                    rmax = flo;  // (one key value left: it is v)
                }
                __syncthreads();
                if (flo != fhi) {
                    if (tid == 0) rmax = 0ull;
                    for (uint32_t i = i0 + tid; i < i1; i += kSelThreads) {
                        const uint64_t k = a.lkey[i];
                        if (k >= flo && k <= fhi) {
                            const uint32_t at = atomicAdd(&rcount, 1u);
                            bkey[at] = k;  // (cnt <= kSelBrute candidates lie in range)
                            bsize[at] = a.lsize[i];
                        }
                    }
                    __syncthreads();
                    const uint32_t c = rcount;
                    if (tid < (int)c) {
                        const uint64_t k = bkey[tid];
                        int64_t g = 0;
                        for (uint32_t j = 0; j < c; j++) g += bkey[j] >= k ? (int64_t)bsize[j] : 0;
                        if (g > need) atomicMax((unsigned long long *)&rmax, (unsigned long long)k);
                    }
                }
                __syncthreads();
                if (tid == 0) {
                    Kg[l] = Kcg[l] = rmax + 1;
                    if (a.dbg && g == 0) {
                        a.dbg[33 + l] = round;
                        a.dbg[65 + l] = cnt;
                    }
                }
                break;
            }
            // bytes and counts per 1/4096 of the key range; the sub-range the
            // budget falls in
            const int shift = max(0, 64 - __builtin_clzll(fhi - flo) - kResLog2);
            for (int i = tid; i < kResBins; i += kSelThreads) {
                hist[i] = 0ull;
                hcnt[i] = 0u;
            }
            __syncthreads();
            for (uint32_t i = i0 + tid; i < i1; i += kSelThreads) {
                const uint64_t k = a.lkey[i];
                if (k >= flo && k <= fhi) {
                    const uint32_t sb = (uint32_t)((k - flo) >> shift);
                    atomicAdd((unsigned long long *)&hist[sb], (unsigned long long)a.lsize[i]);
                    atomicAdd(&hcnt[sb], 1u);
                }
            }
            __syncthreads();
            {
                uint64_t v[kResPer], sm = 0;
#pragma unroll
                for (int i = 0; i < kResPer; i++) sm += (v[i] = hist[kResPer * tid + i]);
                uint64_t tot;
                const uint64_t pre = wg_excl_scan64<kSelThreads>(sm, wsum, tot);
                uint64_t S = tot - pre;  // bytes of the sub-ranges >= kResPer tid
#pragma unroll
                for (int i = 0; i < kResPer; i++) {
                    // the largest sub-range s with S(s) > need: S(s) > need >= S(s + 1)
                    const uint64_t Sn = S - v[i];
                    if ((int64_t)S > need && (int64_t)Sn <= need) {
                        const uint64_t lo = flo + ((uint64_t)(kResPer * tid + i) << shift);
                        rlo = lo;
                        rhi = lo + ((1ull << shift) - 1ull) > fhi ? fhi : lo + ((1ull << shift) - 1ull);
                        rneed = need - (int64_t)Sn;
                        rcount = hcnt[kResPer * tid + i];
                    }
                    S = Sn;
                }
            }
            __syncthreads();
        }
    }
}

// Split path only (GpuEncoder::segments): every hull segment listed
// (key, bytes), for the host-side exact exchange.  Segment counts (hull
// points - 1) and their exclusive scan, one workgroup; rounds of 32
// consecutive blocks per thread, their 32 byte loads in flight together
constexpr int kSegThreads = 1024, kSegPer = 32;
__global__ void __launch_bounds__(kSegThreads) k_seg_offsets(int nblocks, const uint8_t *nhull, int32_t *nseg,
                                                             int32_t *segoff) {
    __shared__ uint32_t wsum[kSegThreads / 64 + 1];
    uint32_t base = 0;
    for (int r0 = 0; r0 < nblocks; r0 += kSegThreads * kSegPer) {
        const int b0 = r0 + (int)threadIdx.x * kSegPer;
        uint8_t n[kSegPer];
        uint32_t c = 0, tot;
        const bool whole = b0 + kSegPer <= nblocks;  // 16-byte loads / stores (b0 is 32-aligned)
        if (whole) {
            const uint4 v0 = *(const uint4 *)(nhull + b0), v1 = *(const uint4 *)(nhull + b0 + 16);
            const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
            for (int i = 0; i < kSegPer; i++) n[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
        } else {
#pragma unroll
            for (int i = 0; i < kSegPer; i++) n[i] = nhull[min(b0 + i, nblocks - 1)];
#pragma unroll
            for (int i = 0; i < kSegPer; i++)
                if (b0 + i >= nblocks) n[i] = 0;
        }
        int32_t k[kSegPer], off[kSegPer];
#pragma unroll
        for (int i = 0; i < kSegPer; i++) {
            k[i] = n[i] ? n[i] - 1 : 0;
            c += (uint32_t)k[i];
        }
        uint32_t o = base + wg_excl_scan<kSegThreads>(c, wsum, tot);
#pragma unroll
        for (int i = 0; i < kSegPer; i++) {
            off[i] = (int32_t)o;
            o += (uint32_t)k[i];
        }
        if (whole) {
#pragma unroll
            for (int i = 0; i < kSegPer; i += 4) {
                *(int4 *)(nseg + b0 + i) = make_int4(k[i], k[i + 1], k[i + 2], k[i + 3]);
                *(int4 *)(segoff + b0 + i) = make_int4(off[i], off[i + 1], off[i + 2], off[i + 3]);
            }
        } else {
#pragma unroll
            for (int i = 0; i < kSegPer; i++)
                if (b0 + i < nblocks) {
                    nseg[b0 + i] = k[i];
                    segoff[b0 + i] = off[i];
                }
        }
        base += tot;
    }
}

// segments of each block's hull at its offset; entries past the real count
// (up to the bound `nbound`) get key 0 and size 0
__global__ void __launch_bounds__(256) k_seg_emit(int nblocks, const uint8_t *nhull, const uint8_t *hpass,
                                                  const uint64_t *hkey, const int32_t *rates,
                                                  const int32_t *segoff, uint64_t *keys, int64_t *vals) {
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    int nh = nhull[b];
    const uint8_t *hp = hpass + (size_t)b * (kMaxPasses + 1);
    const uint64_t *hk = hkey + (size_t)b * (kMaxPasses + 1);
    const int32_t *R = rates + (size_t)b * kMaxPasses;
    int o = segoff[b];
    for (int i = 1; i < nh; i++) {
        keys[o + i - 1] = hk[i];
        vals[o + i - 1] = (int64_t)(R[hp[i] - 1] - (hp[i - 1] ? R[hp[i - 1] - 1] : 0));
    }
}

// last hull index whose key >= K (0 = nothing); hull keys strictly decrease
__device__ __forceinline__ int hull_pick(const uint64_t *hk, int nh, uint64_t K) {
    int lo = 1, hi = nh;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (hk[mid] >= K) lo = mid + 1;
        else hi = mid;
    }
    return lo - 1;
}

struct ApplyArgs {
    const int *halt;  // device rate loop: nothing to do once it has stopped
    int nblocks, layers, lossless;
    int ngroups;
    const int32_t *grp_b0;  // the block's rate-control group: its thresholds at K + group * kMaxLayers
    const uint8_t *nhull, *hpass, *npasses;
    const uint64_t *hkey, *K;
    const int32_t *rates;
    uint8_t *nl;      // [block][layers]
    int32_t *lrate;   // [block][layers]
};

__global__ void __launch_bounds__(256) k_apply(ApplyArgs a) {
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.nblocks || (a.halt && *a.halt)) return;
    const int L = a.layers;
    const uint8_t *hp = a.hpass + (size_t)b * (kMaxPasses + 1);
    const uint64_t *hk = a.hkey + (size_t)b * (kMaxPasses + 1);
    const int32_t *R = a.rates + (size_t)b * kMaxPasses;
    int nh = a.nhull[b];
    const uint64_t *K = a.K + (size_t)block_group(a.grp_b0, a.ngroups, b) * kMaxLayers;
    for (int l = 0; l < L; l++) {
        int n = (a.lossless && l == L - 1) ? (int)a.npasses[b] : (int)hp[hull_pick(hk, nh, K[l])];
        a.nl[(size_t)b * L + l] = (uint8_t)n;
        a.lrate[(size_t)b * L + l] = n ? R[n - 1] : 0;
    }
}

// --------------------------------------------------------------------------
// Device pipeline
// --------------------------------------------------------------------------
// Stage-cost experiments (tests/tools/stage_cost2.sh) build with
// -DJP2HIP_REPEAT_STAGE=<n> to launch one stage's kernels twice (they are
// idempotent): 1 DWT, 2 quantiser, 3 MQ, 4 hull, 5 tier-2 sizing wave kernel.
// Product builds never define it.
#ifndef JP2HIP_REPEAT_STAGE
#define JP2HIP_REPEAT_STAGE 0
#endif
#define REPEAT_IF(n) for (int rep_ = 0; rep_ < (JP2HIP_REPEAT_STAGE == (n) ? 2 : 1); rep_++)
// the largest rate-control group (its blocks set the grid's x extent)
static int grp_max_blocks(const Plan &plan) {
    int m = 0;
    for (int g = 0; g < plan.ngroups(); g++) m = std::max(m, plan.grp_b0[(size_t)g + 1] - plan.grp_b0[(size_t)g]);
    return std::max(m, 1);
}

std::vector<DevBuf *> GpuEncoder::bufs() {
    return {&coef, &blocks, &order, &bp, &sm, &P, &dref, &dsig, &t1out, &rates, &dists,
            &npasses, &lengths, &weight, &nhull, &hpass, &hkey, &budget, &nl, &lrate,
            &dstoff, &packed, &err, &tcw, &tch, &strips, &src, &llbuf0, &llbuf1, &ordkey, &segcnt, &segoff, &segkey,
            &segval, &thr, &items, &slotoff, &pcrd_hb, &pcrd_hc, &sel_ctl, &sel_key, &sel_size,
            &stream_buf, &counts, &dspp, &dbgbuf, &est, &hist, &kcut, &pmin, &mqspan, &stage, &soff, &lzwseg, &untiled,
            &inflnk, &t2prec, &t2tp, &t2tt, &t2lblock, &t2incl, &t2pklen, &t2pkoff, &t2tplen, &t2tphdr, &t2tpoff,
            &t2blkdst, &t2out, &t2sum, &hdist, &rstate, &t2ticket,
            &t1fill, &dbgsel, &grptab, &gtot};
}

// test-only model of a small device: every context's buffers together may
// not pass JP2HIP_TEST_DEVICE_BYTES (0 / unset: the device's own memory)
static std::atomic<long long> g_test_held{0};
static long long test_device_bytes() {
    static const long long v = [] {
        const char *s = getenv("JP2HIP_TEST_DEVICE_BYTES");
        return s ? atoll(s) : 0ll;
    }();
    return v;
}

hipError_t GpuEncoder::device_alloc(void **p, size_t n) {
    const long long cap = test_device_bytes();
    if (cap > 0) {
        if (g_test_held.fetch_add((long long)n) + (long long)n > cap) {
            g_test_held.fetch_sub((long long)n);
            return hipErrorOutOfMemory;
        }
        const hipError_t e = hipMalloc(p, n);
        if (e != hipSuccess) g_test_held.fetch_sub((long long)n);
        return e;
    }
    return hipMalloc(p, n);
}

void GpuEncoder::device_free(DevBuf &b) {
    if (b.ptr) {
        (void)hipFree(b.ptr);
        if (test_device_bytes() > 0) g_test_held.fetch_sub((long long)b.bytes);
    }
    held -= b.bytes;
    b.ptr = nullptr;
    b.bytes = 0;
}

bool GpuEncoder::trim(size_t soft) {
    if (held <= soft) return false;
    for (DevBuf *b : bufs()) device_free(*b);
    held = 0;
    // the device copies of the plan's tables went with the buffers
    front_gen = 0;
    t2_gen = 0;
    strips_dev = nullptr;
    strips_host.clear();
    dma_ok = false;  // (re-reads t2out's owner agent at the next copy)
    pool_hint = 0;   // (the outsized image's need)
    return true;
}

bool GpuEncoder::pool_grow(std::string &err) {
    unsigned long long used = 0;
    HIPCHECK(hipStreamSynchronize(stream));
    HIPCHECK(hipMemcpy(&used, (unsigned long long *)mqspan.ptr + 2, sizeof used, hipMemcpyDeviceToHost));
    pool_hint = std::max<uint64_t>(pool_hint, used + used / 8);
    pool_grows++;
    return true;
}

void GpuEncoder::quiesce() {
    if (stream) (void)hipStreamSynchronize(stream);
    (void)hipGetLastError();
}

GpuEncoder::~GpuEncoder() {
    for (DevBuf *b : bufs()) device_free(*b);
    if (sync_ev) (void)hipEventDestroy(sync_ev);
    if (stg_ev) (void)hipEventDestroy(stg_ev);
    for (const PinnedChunk &c : stg) (void)hipHostFree(c.p);
    if (stream) (void)hipStreamDestroy(stream);
    for (int i = 0; i < kNumEvents; i++)
        if (ev[i]) (void)hipEventDestroy(ev[i]);
    if (h_packed) (void)hipHostFree(h_packed);
    if (h_sum) (void)hipHostFree(h_sum);
    if (h_tot) (void)hipHostFree(h_tot);
    if (h_rs) (void)hipHostFree(h_rs);
    if (dma_dep.handle) (void)hsa_signal_destroy(dma_dep);
    if (dma_done.handle) (void)hsa_signal_destroy(dma_done);
    if (hsa_up) (void)hsa_shut_down();
}

bool GpuEncoder::init(int dev, std::string &err) {
    device = dev;
    if (const char *f = getenv("JP2HIP_TEST_POOL_FRAC")) pool_frac_test = atof(f);
    HIPCHECK(hipSetDevice(dev));
    HIPCHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    for (int i = 0; i < kNumEvents; i++) HIPCHECK(hipEventCreate(&ev[i]));
    HIPCHECK(hipEventCreateWithFlags(&sync_ev, hipEventBlockingSync | hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&stg_ev, hipEventDisableTiming));
    HIPCHECK(hipHostMalloc((void **)&h_tot, 8 * sizeof(int64_t), hipHostMallocDefault));
    return true;
}

bool GpuEncoder::check_residency(std::string &err) {
    hipDevice_t sd = -1;
    HIPCHECK(hipStreamGetDevice(stream, &sd));
    if ((int)sd != device) {
        err = "context on device " + std::to_string(device) + ": its stream is on device " + std::to_string((int)sd);
        return false;
    }
    const DevBuf *bufs[] = {&src, &coef, &bp, &t1out, &stream_buf, &t2out, &blocks};
    for (const DevBuf *b : bufs) {
        if (!b->ptr) continue;
        hipPointerAttribute_t at;
        HIPCHECK(hipPointerGetAttributes(&at, b->ptr));
        if (at.device != device) {
            err = "context on device " + std::to_string(device) + ": a buffer lives on device " +
                  std::to_string(at.device);
            return false;
        }
    }
    return true;
}

bool GpuEncoder::h2d(void *dst, const void *src, size_t bytes, std::string &err) {
    if (!bytes) return true;
    if (hipEventQuery(stg_ev) == hipSuccess) {  // every staged copy has landed: reuse from the start
        if (stg.size() > 1) {
            size_t tot = 0;
            for (const PinnedChunk &c : stg) {
                tot += c.cap;
                HIPCHECK(hipHostFree(c.p));
            }
            stg.clear();
            PinnedChunk c{nullptr, tot};
            HIPCHECK(hipHostMalloc((void **)&c.p, tot, hipHostMallocDefault));
            stg.push_back(c);
        }
        stg_used = 0;
    }
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (stg.empty() || stg_used + need > stg.back().cap) {  // a new chunk; the older ones stay until the copies land
        PinnedChunk c{nullptr, std::max<size_t>(need, stg.empty() ? (size_t)1 << 20 : 2 * stg.back().cap)};
        HIPCHECK(hipHostMalloc((void **)&c.p, c.cap, hipHostMallocDefault));
        stg.push_back(c);
        stg_used = 0;
    }
    uint8_t *h = stg.back().p + stg_used;
    stg_used += need;
    std::memcpy(h, src, bytes);
    HIPCHECK(hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipEventRecord(stg_ev, stream));
    return true;
}

// Host waits for this context's stream by sleeping on an event rather than
// spinning: with many images in flight the spinning callers would take the
// cores the tier-2 threads need.
#ifndef JP2HIP_WAIT_POLL_US
#define JP2HIP_WAIT_POLL_US 0  // A/B builds: poll the event every N us instead of sleeping on it
#endif
bool GpuEncoder::host_wait(std::string &err) {
    waits++;
    HIPCHECK(hipEventRecord(sync_ev, stream));
#if JP2HIP_WAIT_POLL_US > 0
    for (;;) {
        const hipError_t q = hipEventQuery(sync_ev);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) HIPCHECK(q);
        std::this_thread::sleep_for(std::chrono::microseconds(JP2HIP_WAIT_POLL_US));
    }
#else
    HIPCHECK(hipEventSynchronize(sync_ev));
#endif
    return true;
}

bool GpuEncoder::upload_source(const void *host, size_t len, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    if (!ensure<uint8_t>(src, len, err)) return false;
    // stream-ordered: the encode that follows (same stream) waits for it, and
    // the caller's buffer outlives the synchronous encode call
    HIPCHECK(hipMemcpyAsync(src.ptr, host, len, hipMemcpyHostToDevice, stream));
    return true;
}

bool GpuEncoder::dump(const char *dir, const char *name, const DevBuf &b, size_t bytes,
                      std::string &err) {
    std::vector<uint8_t> h(bytes);
    if (!host_wait(err)) return false;
    if (bytes) HIPCHECK(hipMemcpy(h.data(), b.ptr, bytes, hipMemcpyDeviceToHost));
    std::string path = std::string(dir) + "/" + name;
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) { err = "cannot write dump " + path; return false; }
    fwrite(h.data(), 1, bytes, f);
    fclose(f);
    return true;
}

bool GpuEncoder::unpack_strips(const void *d_src, const jp2hip_layout &lay, jp2hip_layout &out,
                               std::vector<uint64_t> &out_offs, const void **d_out, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    const int ns = lay.nstrips;  // strips, or tiles
    const bool tiled = lay.tile_width > 0;
    const int spp_row = lay.planar == 2 ? 1 : lay.components;
    const int px_bytes = spp_row * (lay.bits / 8);
    const int unit_w = tiled ? lay.tile_width : lay.width, unit_h = tiled ? lay.tile_height : lay.rows_per_strip;
    const int planes = lay.planar == 2 ? lay.components : 1;
    const int across = tiled ? (lay.width + lay.tile_width - 1) / lay.tile_width : 1;
    const int per_plane = tiled ? across * ((lay.height + lay.tile_height - 1) / lay.tile_height)
                                : (lay.height + lay.rows_per_strip - 1) / lay.rows_per_strip;
    const uint64_t row_bytes = (uint64_t)unit_w * px_bytes;
    const uint64_t stride = ((uint64_t)unit_h * row_bytes + 255) & ~255ull;
    const bool decode = lay.compression > 1;
    if (!ensure<uint64_t>(soff, (size_t)ns * 2, err) || !ensure<int>(this->err, 4, err)) return false;
    if (decode && !ensure<uint8_t>(stage, stride * ns, err)) return false;
    if (!h2d(soff.ptr, lay.strip_offsets, sizeof(uint64_t) * ns, err) ||
        !h2d((uint64_t *)soff.ptr + ns, lay.strip_bytes, sizeof(uint64_t) * ns, err))
        return false;
    HIPCHECK(hipMemsetAsync(this->err.ptr, 0, sizeof(int), stream));
    if (decode) {
        UnpackArgs ua;
        ua.src = (const uint8_t *)d_src;
        ua.off = (const uint64_t *)soff.ptr;
        ua.cnt = (const uint64_t *)soff.ptr + ns;
        ua.nstrips = ns;
        ua.per_plane = per_plane;
        ua.rps = lay.rows_per_strip;
        ua.h = lay.height;
        ua.row_bytes = row_bytes;
        ua.stride = stride;
        ua.unit_bytes = tiled ? (uint64_t)unit_h * row_bytes : 0;
        ua.dst = (uint8_t *)stage.ptr;
        ua.only = nullptr;
        ua.lnk = nullptr;
        ua.err = (int *)this->err.ptr;
        if (lay.compression == 5) {  // segment-parallel (lzw.hip)
            std::vector<uint64_t> slice;
            const uint64_t segs = lzw_slices(lay.strip_bytes, ns, slice);
            if (!ensure<uint8_t>(lzwseg, lzw_scratch_bytes(ns, segs), err) ||
                !h2d(lzwseg.ptr, slice.data(), sizeof(uint64_t) * ns, err))
                return false;
            if (!launch_lzw(ua, segs, lzwseg.ptr, stream)) {
                err = std::string("LZW launch failed: ") + hipGetErrorString(hipGetLastError());
                return false;
            }
        }
        else if (lay.compression == 8 || lay.compression == 32946) {
            // decode to links (a strip per wave), then resolve the links
            // (every strip's bytes in parallel; k_inflate_links)
            if (!ensure<uint32_t>(inflnk, stride * ns, err)) return false;
            ua.lnk = (uint32_t *)inflnk.ptr;
            hipLaunchKernelGGL(k_inflate, dim3(ns), dim3(kInfLanes), 0, stream, ua);
            const dim3 g((unsigned)((unit_h * row_bytes + kLinkChunk - 1) / kLinkChunk), (unsigned)ns);
            for (int r = 0; r <= kLinkDoublings; r++)
                hipLaunchKernelGGL(k_inflate_links, g, dim3(256), 0, stream, ua, r == kLinkDoublings ? 1 : 0);
        }
        else hipLaunchKernelGGL(k_unpackbits, dim3(ns), dim3(64), 0, stream, ua);
        HIPCHECK(hipGetLastError());
        if (lay.predictor == 2) {  // per decoded row of a strip / of a tile
            const int nrows = ns * unit_h;
            hipLaunchKernelGGL(k_unpredict, dim3((nrows + 255) / 256), dim3(256), 0, stream, (uint8_t *)stage.ptr,
                               nrows, unit_h, unit_h, tiled ? unit_h : lay.height, tiled ? 1 : per_plane, stride,
                               unit_w, spp_row, lay.bits, lay.big_endian);
            HIPCHECK(hipGetLastError());
        }
    } else if (lay.predictor == 2) {
        err = "tiff: Predictor 2 on uncompressed data is not supported";
        return false;
    }
    const void *res = decode ? stage.ptr : d_src;
    out = lay;
    out_offs.resize(tiled ? planes : ns);
    if (tiled) {  // tiles -> one row-major strip per plane
        const uint64_t plane_bytes = (uint64_t)lay.width * lay.height * px_bytes;
        if (!ensure<uint8_t>(untiled, plane_bytes * planes, err)) return false;
        hipLaunchKernelGGL(k_untile, dim3((lay.width + 255) / 256, lay.height, planes), dim3(256), 0, stream,
                           (const uint8_t *)res, decode ? nullptr : (const uint64_t *)soff.ptr, stride, lay.width,
                           lay.height, lay.tile_width, lay.tile_height, across, per_plane, px_bytes,
                           (uint8_t *)untiled.ptr);
        HIPCHECK(hipGetLastError());
        for (int p = 0; p < planes; p++) out_offs[p] = (uint64_t)p * plane_bytes;
        out.rows_per_strip = lay.height;
        out.nstrips = planes;
        out.tile_width = out.tile_height = 0;
        res = untiled.ptr;
    } else {
        for (int i = 0; i < ns; i++) out_offs[i] = (uint64_t)i * stride;
    }
    HIPCHECK(hipMemcpyAsync(h_tot + 4, this->err.ptr, sizeof(int), hipMemcpyDeviceToHost, stream));
    if (!host_wait(err)) return false;
    const int herr = *(const int *)(h_tot + 4);
    if (herr & 4) {
        err = "tiff: old-style (pre-TIFF 6.0, LSB-first) LZW strips are not supported";
        return false;
    }
    if (herr) {
        err = "tiff: corrupt compressed strip";
        return false;
    }
    out.strip_offsets = out_offs.data();
    out.compression = 1;
    out.predictor = 1;
    out.strip_bytes = nullptr;
    *d_out = res;
    return true;
}

bool GpuEncoder::run_front(const void *d_src, const jp2hip_layout &lay, const Plan &plan,
                           bool profile, StageTimes &st, std::string &err, int64_t skip_target,
                           const HistReduce *reduce, bool pool_worst) {
    HIPCHECK(hipSetDevice(device));
    const int nb = (int)plan.blocks.size();
    size_t plane = (size_t)plan.plane_w * plan.plane_h;
    if (!ensure<int32_t>(coef, plane * plan.ntc, err)) return false;
    if (!ensure<BlockDesc>(blocks, nb, err)) return false;
    if (!ensure<int32_t>(order, nb, err)) return false;
    if (!ensure<uint64_t>(bp, plan.bp_words, err)) return false;
    if (!ensure<int32_t>(sm, plan.sm_words, err)) return false;
    if (!ensure<uint8_t>(P, nb, err)) return false;
    if (!ensure<int64_t>(dref, (size_t)nb * 32, err)) return false;
    if (!ensure<int64_t>(dsig, (size_t)nb * 32, err)) return false;
    if (!ensure<uint32_t>(est, (size_t)nb * 32, err)) return false;
    if (!ensure<uint8_t>(pmin, nb, err)) return false;
    if (!ensure<unsigned long long>(hist, kSlopeBins, err)) return false;
    if (!ensure<int>(kcut, 1, err)) return false;
    if (!ensure<uint8_t>(t1out, plan.out_bytes + 64, err)) return false;  // + k_t2_copy's dword over-read
    if (!ensure<int32_t>(rates, (size_t)nb * kMaxPasses, err)) return false;
    if (!ensure<int64_t>(dists, (size_t)nb * kMaxPasses, err)) return false;
    if (!ensure<uint8_t>(npasses, nb, err)) return false;
    if (!ensure<int32_t>(lengths, nb, err)) return false;
    if (!ensure<double>(weight, nb, err)) return false;
    if (!ensure<uint8_t>(nhull, nb, err)) return false;
    if (!ensure<uint8_t>(hpass, (size_t)nb * (kMaxPasses + 1), err)) return false;
    if (!ensure<uint64_t>(hkey, (size_t)nb * (kMaxPasses + 1), err)) return false;
    if (!ensure<int64_t>(hdist, (size_t)nb * (kMaxPasses + 1) * 2, err)) return false;  // HullPt
    const int G = plan.ngroups();
    if (!ensure<int64_t>(budget, (size_t)G * kMaxLayers, err)) return false;
    if (!ensure<uint8_t>(nl, (size_t)nb * plan.rc.layers, err)) return false;
    if (!ensure<int32_t>(lrate, (size_t)nb * plan.rc.layers, err)) return false;
    if (!ensure<int>(this->err, 4, err)) return false;
    if (!ensure<int32_t>(tcw, plan.ntc, err)) return false;
    if (!ensure<int32_t>(tch, plan.ntc, err)) return false;
    if (!ensure<uint64_t>(strips, lay.nstrips, err)) return false;

    // tier-1 decision streams: one pool, carved on the device once the coded
    // planes are known (emit_t1_items: c planes x plane_stream_cap per
    // block).  Sized at a fraction of the every-plane bound -- or at what an
    // encode of this context last needed, when that is more -- and grown
    // after an encode that did not fit (the host re-encodes: pool_grow).
    // The tile-split path asks for the whole bound (its ranks cannot repeat
    // an exchange).
    uint64_t stream_bound = 0;
    for (int i = 0; i < nb; i++)
        stream_bound += (uint64_t)plan.blocks[i].Mb * t1_plane_stream_cap(plan.blocks[i].w, plan.blocks[i].h);
    const double pool_frac = pool_worst             ? 1.0
                             : pool_frac_test >= 0.0 ? pool_frac_test
                             : (plan.rc.reversible ? kPoolFracLossless : kPoolFracLossy);
    const uint64_t pool_want = std::min<uint64_t>(
        stream_bound, std::max<uint64_t>(pool_hint, (uint64_t)((double)stream_bound * pool_frac)));
    if (!ensure<uint64_t>(slotoff, nb, err) || !ensure<uint8_t>(stream_buf, std::max<uint64_t>(pool_want, 1), err))
        return false;
    // the strip offsets: uploaded only when they differ from the last upload
    // (repeat encodes of one layout skip the copy)
    if (strips.ptr != strips_dev || strips_host.size() != (size_t)lay.nstrips ||
        std::memcmp(strips_host.data(), lay.strip_offsets, sizeof(uint64_t) * lay.nstrips) != 0) {
        if (!h2d(strips.ptr, lay.strip_offsets, sizeof(uint64_t) * lay.nstrips, err)) return false;
        strips_host.assign(lay.strip_offsets, lay.strip_offsets + lay.nstrips);
        strips_dev = strips.ptr;
    }
    // the plan's tables stay resident while the context encodes the same
    // geometry (plan.gen; buffers only grow, so they are still in place)
    if (!plan.gen || plan.gen != front_gen) {
        front_gen = 0;
        if (!h2d(blocks.ptr, plan.blocks.data(), sizeof(BlockDesc) * nb, err) ||
            !h2d(weight.ptr, plan.weight.data(), sizeof(double) * nb, err) ||
            !h2d(tcw.ptr, plan.tc_w.data(), sizeof(int32_t) * plan.ntc, err) ||
            !h2d(tch.ptr, plan.tc_h.data(), sizeof(int32_t) * plan.ntc, err))
            return false;
        // rate-control groups: block ranges and each group's first
        // candidate slot (the bound sum(3 Mb - 2) over the groups before)
        std::vector<int32_t> gtab(2 * ((size_t)G + 1));
        int64_t sb = 0;
        for (int g = 0; g <= G; g++) {
            gtab[(size_t)g] = plan.grp_b0[(size_t)g];
            gtab[(size_t)G + 1 + g] = (int32_t)sb;
            if (g < G)
                for (int i = plan.grp_b0[(size_t)g]; i < plan.grp_b0[(size_t)g + 1]; i++)
                    sb += std::max(0, 3 * (int)plan.blocks[i].Mb - 2);
        }
        if (!ensure<int32_t>(grptab, gtab.size(), err) || !h2d(grptab.ptr, gtab.data(), sizeof(int32_t) * gtab.size(), err))
            return false;
        front_gen = plan.gen;
    }
    // (the error word is zeroed by k_quant, which every encode with blocks runs)
    if (!nb) {
        HIPCHECK(hipMemsetAsync(this->err.ptr, 0, sizeof(int), stream));
        if (!ensure<T2Summary>(t2sum, 1, err)) return false;
        HIPCHECK(hipMemsetAsync(t2sum.ptr, 0, sizeof(T2Summary), stream));  // (k_hull's totals: none)
    }

    // the first stage's arguments are prepared before its events: on an idle
    // stream the GPU waits from the event to the first launch, so host work
    // placed there was timed as DWT (≈80 us of a 310 us C2 stage alone,
    // against 232 us of DWT kernels in the rocprofv3 trace of the same run,
    // profiles/r06/dwt_stage_events.txt)
    // every stage's device buffer written to files: a debug build only
    // (make JP2HIP_DEBUG=1), for the tools in tests/tools
#ifdef JP2HIP_DEBUG_DUMPS
    const char *dd = getenv("JP2HIP_DUMP_DIR");
#else
    const char *dd = nullptr;
#endif
    // the final coefficients are written as quantisation indices
    const QuantTab qt = quant_tab(plan.rc, plan.bits);
    IngestArgs ing;
    DwtLaunch dl;
    if (plan.rc.levels == 0) {
        // S1+S2 only: no decomposition
        ing.src = (const uint8_t *)d_src;
        ing.strip_off = (const uint64_t *)strips.ptr;
        ing.rps = lay.rows_per_strip;
        ing.w = plan.w; ing.h = plan.band_h; ing.nc = plan.nc; ing.bits = plan.bits;
        ing.row0 = plan.row0;
        ing.planar = lay.planar; ing.big_endian = lay.big_endian;
        ing.mct = plan.rc.mct; ing.reversible = plan.rc.reversible;
        ing.ntx = plan.ntx; ing.tile_w = plan.rc.tile_w; ing.tile_h = plan.rc.tile_h;
        ing.plane_w = plan.plane_w; ing.plane_h = plan.plane_h;
        ing.spp_strips = (plan.h + lay.rows_per_strip - 1) / lay.rows_per_strip;
        ing.coef = coef.ptr;
        ing.inv = qt.inv[0][0]; ing.lim = qt.lim[0][0]; ing.q16 = qt.q16;
    } else {
        // S1+S2+S3 fused: ingest inside DWT level 1 (dwt.hip)
        const size_t llw = (size_t)((plan.plane_w + 1) / 2) * ((plan.plane_h + 1) / 2) * plan.ntc;
        if (!ensure<int32_t>(llbuf0, llw, err) || !ensure<int32_t>(llbuf1, llw, err)) return false;
        dl.tif = d_src;
        dl.strip_off = (const uint64_t *)strips.ptr;
        dl.rps = lay.rows_per_strip;
        dl.img_w = plan.w; dl.nc = plan.nc; dl.bits = plan.bits;
        dl.planar = lay.planar; dl.big_endian = lay.big_endian; dl.mct = plan.rc.mct;
        dl.spp_strips = (plan.h + lay.rows_per_strip - 1) / lay.rows_per_strip;
        dl.ntx = plan.ntx; dl.tile_w = plan.rc.tile_w; dl.tile_h = plan.rc.tile_h; dl.row0 = plan.row0;
        dl.last_tile_w = plan.w - (plan.ntx - 1) * plan.rc.tile_w;
        dl.plane_w = plan.plane_w; dl.plane_h = plan.plane_h; dl.ntc = plan.ntc;
        dl.levels = plan.rc.levels; dl.reversible = plan.rc.reversible;
        dl.tc_w = (const int32_t *)tcw.ptr; dl.tc_h = (const int32_t *)tch.ptr;
        dl.coef = coef.ptr; dl.scratch0 = llbuf0.ptr; dl.scratch1 = llbuf1.ptr;
        dl.qt = qt;
    }
    HIPCHECK(hipEventRecord(ev[0], stream));
    HIPCHECK(hipEventRecord(ev[1], stream));
    if (plan.rc.levels == 0) {
        dim3 gi((plan.w + 63) / 64, (plan.band_h + 3) / 4);
        hipLaunchKernelGGL(k_ingest, gi, dim3(256), 0, stream, ing);
        HIPCHECK(hipGetLastError());
    } else {
        bool dwt_ok = true;
        REPEAT_IF(1) dwt_ok = dwt_ok && launch_dwt(dl, stream);
        if (!dwt_ok) {
            err = std::string("DWT launch failed: ") + hipGetErrorString(hipGetLastError());
            return false;
        }
    }
    HIPCHECK(hipEventRecord(ev[2], stream));
    if (dd && !dump(dd, "dwt.bin", coef, plane * plan.ntc * (qt.q16 ? 2 : 4), err)) return false;
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
    qa.est = (uint32_t *)est.ptr;
    qa.nblocks = nb;
    qa.keep_sm = dd != nullptr;
    // tier-1 work lists and lane order, slope prediction, PCRD: their
    // counters are zeroed by k_quant's first workgroup (no memset launches)
    int kmax = 0;
    for (int i = 0; i < nb; i++) kmax = std::max(kmax, (int)plan.blocks[i].Mb);
    const size_t nflags = (size_t)nb * kmax;
    if (!ensure<unsigned long long>(pcrd_hb, (size_t)G * kPcrdBins, err) ||
        !ensure<uint32_t>(pcrd_hc, (size_t)G * kPcrdBins, err) ||
        !ensure<uint32_t>(sel_ctl, (size_t)G * (kMaxLayers + 1), err) ||
        !ensure<unsigned long long>(gtot, G, err) || !ensure<uint32_t>(t1fill, 64 + kOrderBuckets, err) ||
        !ensure<int32_t>(items, std::max<size_t>(nflags, 1), err) ||
        !ensure<int32_t>(order, (size_t)kOrderBuckets * std::max(nb, 1), err) ||
        !ensure<uint4>(counts, (size_t)nb * 32, err) || !ensure<int64_t>(dspp, (size_t)nb * 32, err) ||
        !ensure<unsigned long long>(ordkey, std::max(nb, 1), err) || !ensure<unsigned long long>(mqspan, 3, err))
        return false;
    uint32_t *dfill = (uint32_t *)t1fill.ptr, *bfill = dfill + 64;
    std::memset(qa.zero, 0, sizeof qa.zero);
    std::memset(qa.nzero, 0, sizeof qa.nzero);
    qa.zero[0] = (uint32_t *)pcrd_hb.ptr;
    qa.nzero[0] = 2 * kPcrdBins * G;
    qa.zero[1] = (uint32_t *)pcrd_hc.ptr;
    qa.nzero[1] = kPcrdBins * G;
    qa.zero[2] = (uint32_t *)sel_ctl.ptr;
    qa.nzero[2] = (kMaxLayers + 1) * G;
    qa.zero[3] = dfill;
    qa.nzero[3] = 64 + kOrderBuckets;
    qa.zero[4] = (uint32_t *)mqspan.ptr;  // k_t1_mq's span[2], then the stream pool's fill
    qa.nzero[4] = 6;
    // (span 5: the error word; span 6: the slope histogram; span 7: tier-1
    // totals; span 8: the rate-control groups' tier-1 bytes)
    qa.zero[8] = (uint32_t *)gtot.ptr;
    qa.nzero[8] = 2 * G;
    qa.zero[5] = (uint32_t *)this->err.ptr;
    qa.nzero[5] = 1;
    // the tier-1 totals k_hull sums (t1_bytes .. skipped: contiguous)
    if (!ensure<T2Summary>(t2sum, 1, err)) return false;
    qa.zero[7] = (uint32_t *)&((T2Summary *)t2sum.ptr)->t1_bytes;
    qa.nzero[7] = (uint32_t)((offsetof(T2Summary, skipped) + sizeof(int32_t) - offsetof(T2Summary, t1_bytes)) / 4);
    if (skip_target > 0) {
        if (!ensure<unsigned long long>(hist, kSlopeBins, err)) return false;
        qa.zero[6] = (uint32_t *)hist.ptr;
        qa.nzero[6] = 2 * kSlopeBins;
    }
    qa.max_mb = std::max(1, kmax);
    const size_t qlds = (size_t)qa.max_mb * 64 * sizeof(uint64_t);
    if (nb) {
        const dim3 gq((nb + kQuantWaves - 1) / kQuantWaves), bq(64 * kQuantWaves);
        REPEAT_IF(2) {
            const size_t ql = qlds * kQuantWaves;
            if (plan.rc.reversible) {
                if (qt.q16) hipLaunchKernelGGL((k_quant<true, true>), gq, bq, ql, stream, qa);
                else hipLaunchKernelGGL((k_quant<true, false>), gq, bq, ql, stream, qa);
            } else {
                if (qt.q16) hipLaunchKernelGGL((k_quant<false, true>), gq, bq, ql, stream, qa);
                else hipLaunchKernelGGL((k_quant<false, false>), gq, bq, ql, stream, qa);
            }
        }
    }
    HIPCHECK(hipGetLastError());
    // S4b: slope prediction -> lowest coded plane per block, and the tier-1
    // work lists: list k = the blocks with more than k coded planes
    T1ItemArgs ia;
    ia.nb = nb;
    ia.kmax = kmax;
    ia.P = (const uint8_t *)P.ptr;
    ia.pmin = (uint8_t *)pmin.ptr;
    ia.dfill = dfill;
    ia.dlist = (int32_t *)items.ptr;
    ia.acc = (unsigned long long *)ordkey.ptr;
    ia.npasses = (uint8_t *)npasses.ptr;
    ia.lengths = (int32_t *)lengths.ptr;
    ia.blocks = (const BlockDesc *)blocks.ptr;
    ia.pool_used = (unsigned long long *)mqspan.ptr + 2;
    ia.pool_cap = stream_buf.bytes;
    ia.slot_off = (uint64_t *)slotoff.ptr;
    ia.err = (int *)this->err.ptr;
    if (skip_target > 0 && nb) {
        PredictArgs pa;
        pa.nblocks = nb;
        pa.P = (const uint8_t *)P.ptr;
        pa.dref = (const int64_t *)dref.ptr;
        pa.dsig = (const int64_t *)dsig.ptr;
        pa.est = (const uint32_t *)est.ptr;
        pa.weight = (const double *)weight.ptr;
        pa.hist = (unsigned long long *)hist.ptr;
        pa.kcut = (int *)kcut.ptr;
        pa.pmin = (uint8_t *)pmin.ptr;
        hipLaunchKernelGGL(k_plane_hist, dim3((nb + kHistBlocks - 1) / kHistBlocks), dim3(256), 0, stream, pa);
        HIPCHECK(hipGetLastError());
        if (reduce) {
            h_hist.resize(kSlopeBins);
            if (!host_wait(err)) return false;  // (a pageable copy waits for the stream holding a shared lock)
            HIPCHECK(hipMemcpyAsync(h_hist.data(), hist.ptr, sizeof(int64_t) * kSlopeBins, hipMemcpyDeviceToHost,
                                    stream));
            if (!host_wait(err)) return false;
            if (!(*reduce)(h_hist)) {
                err = "split: slope-prediction exchange failed";
                return false;
            }
            if (!h2d(hist.ptr, h_hist.data(), sizeof(int64_t) * kSlopeBins, err)) return false;
        }
        hipLaunchKernelGGL(k_plane_pmin, dim3((nb + 255) / 256), dim3(256), 0, stream, pa, ia, skip_target * 128);
        HIPCHECK(hipGetLastError());
    } else {
        launch_t1_items(ia, stream);
        HIPCHECK(hipGetLastError());
    }
    HIPCHECK(hipEventRecord(ev[3], stream));
    // S5: tier-1.  k_t1_cm3 takes the items depth by depth; each block's last
    // plane files it in its MQ lane-order bucket (decision count), which
    // k_t1_mq reads.  Buffers and the grid are sized by the plan's bound
    // (every plane of every block coded).
    HIPCHECK(hipEventRecord(ev[10], stream));
    T1CmArgs ca;
    ca.dfill = dfill;
    ca.dlist = (const int32_t *)items.ptr;
    ca.nb = nb;
    ca.kmax = kmax;
    ca.max_items = (int)nflags;
    ca.blocks = (const BlockDesc *)blocks.ptr;
    ca.bp = (const uint64_t *)bp.ptr;
    ca.sm = (const int32_t *)sm.ptr;
    ca.P = (const uint8_t *)P.ptr;
    ca.stream = (uint8_t *)stream_buf.ptr;
    ca.slot_off = (const uint64_t *)slotoff.ptr;
    ca.counts = (uint4 *)counts.ptr;
    ca.dspp = (int64_t *)dspp.ptr;
    ca.acc = (unsigned long long *)ordkey.ptr;
    ca.bfill = bfill;
    ca.bslots = (int32_t *)order.ptr;
    ca.lossless = plan.rc.reversible;
    launch_t1_cm(ca, stream);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(ev[11], stream));
    T1MqArgs ma;
    ma.blocks = (const BlockDesc *)blocks.ptr;
    ma.bfill = bfill;
    ma.bslots = (const int32_t *)order.ptr;
    ma.nblocks = nb;
    ma.P = (const uint8_t *)P.ptr;
    ma.pmin = (const uint8_t *)pmin.ptr;
    ma.stream = (const uint8_t *)stream_buf.ptr;
    ma.slot_off = (const uint64_t *)slotoff.ptr;
    ma.counts = (const uint4 *)counts.ptr;
    ma.dspp = (const int64_t *)dspp.ptr;
    ma.dref = (const int64_t *)dref.ptr;
    ma.dsig = (const int64_t *)dsig.ptr;
    ma.out = (uint8_t *)t1out.ptr;
    ma.rates = (int32_t *)rates.ptr;
    ma.dists = (int64_t *)dists.ptr;
    ma.npasses = (uint8_t *)npasses.ptr;
    ma.lengths = (int32_t *)lengths.ptr;
    ma.err = (int *)this->err.ptr;
    ma.dbg = nullptr;
    ma.span = (unsigned long long *)mqspan.ptr;
    if (dd) {
        if (!ensure<int64_t>(dbgbuf, (size_t)nb * 6, err)) return false;
        ma.dbg = (int64_t *)dbgbuf.ptr;
    }
    REPEAT_IF(3) launch_t1_mq(ma, stream);

    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(ev[4], stream));
    // S6a hulls + their slope-bin histogram (k_select resolves thresholds)
    HullArgs ha;
    ha.nblocks = nb;
    ha.npasses = (const uint8_t *)npasses.ptr;
    ha.rates = (const int32_t *)rates.ptr;
    ha.dists = (const int64_t *)dists.ptr;
    ha.weight = (const double *)weight.ptr;
    ha.nhull = (uint8_t *)nhull.ptr;
    ha.hpass = (uint8_t *)hpass.ptr;
    ha.hkey = (uint64_t *)hkey.ptr;
    ha.hdist = (int64_t *)hdist.ptr;
    ha.hbytes = (unsigned long long *)pcrd_hb.ptr;
    ha.hcount = (uint32_t *)pcrd_hc.ptr;
    ha.lengths = (const int32_t *)lengths.ptr;
    ha.acc = (const unsigned long long *)ordkey.ptr;
    ha.pmin = (const uint8_t *)pmin.ptr;
    ha.sum = (T2Summary *)t2sum.ptr;
    ha.grp_b0 = (const int32_t *)grptab.ptr;
    ha.gtot = (unsigned long long *)gtot.ptr;
    REPEAT_IF(4) if (nb) hipLaunchKernelGGL(k_hull, dim3((grp_max_blocks(plan) + kHullThreads - 1) / kHullThreads, G),
                                            dim3(kHullThreads), 0, stream, ha);
    HIPCHECK(hipGetLastError());
    // candidate lists: room for every hull segment (the bound sum(3 Mb - 2))
    int64_t nseg_bound = 0;
    for (int i = 0; i < nb; i++) nseg_bound += std::max(0, 3 * (int)plan.blocks[i].Mb - 2);
    nseg = (int)nseg_bound;
    if (!ensure<uint64_t>(sel_key, std::max(nseg, 1), err) || !ensure<uint32_t>(sel_size, std::max(nseg, 1), err) ||
        !ensure<uint64_t>(thr, 2 * (size_t)G * kMaxLayers, err))
        return false;
    HIPCHECK(hipEventRecord(ev[5], stream));
    profiled = profile;
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
        if (!dump(dd, "est.bin", est, (size_t)nb * 32 * 4, err)) return false;
        if (!dump(dd, "pmin.bin", pmin, nb, err)) return false;
        if (!dump(dd, "bp.bin", bp, plan.bp_words * 8, err)) return false;
        if (!dump(dd, "mqdbg.bin", dbgbuf, (size_t)nb * 6 * 8, err)) return false;
    }
    // no host wait: tier-1 totals and the overflow flag reach the host with
    // the first tier-2 summary (t2_size), stage times via collect_profile()
    return true;
}

// Stage times from the events of the last encode (all complete once the
// encode's final host wait returned).
bool GpuEncoder::collect_profile(StageTimes &st, std::string &err) {
    if (!profiled || !h_tot) return true;
    float t;
    HIPCHECK(hipEventElapsedTime(&t, ev[0], ev[1])); st.ingest = t;
    HIPCHECK(hipEventElapsedTime(&t, ev[1], ev[2])); st.dwt = t;
    HIPCHECK(hipEventElapsedTime(&t, ev[2], ev[3])); st.quant = t;
    HIPCHECK(hipEventElapsedTime(&t, ev[10], ev[11])); st.t1_cm = t;
    // k_t1_mq from HIP events on the context's stream around its launch, as
    // rocprofv3 times a dispatch (from when the queue reaches it: under load
    // that includes waiting for CUs)
    HIPCHECK(hipEventElapsedTime(&t, ev[11], ev[4])); st.t1_mq = t;
    HIPCHECK(hipEventElapsedTime(&t, ev[4], ev[5])); st.pcrd += t;
    return true;
}

// k_select per rate-control group: lossless budgets from each group's tier-1
// bytes, else from `budget` (the device rate loop's) -- thresholds of group g
// -> thr[g * kMaxLayers ..), Kc -> thr[(G + g) * kMaxLayers ..)
void GpuEncoder::select_launch(const Plan &plan, const int *halt, const RateState *init, RateState *rs) {
    const int nb = (int)plan.blocks.size(), G = plan.ngroups();
    if (!nb) return;
    SelectArgs sa;
    std::memset(&sa, 0, sizeof sa);
    sa.halt = halt;
    sa.nblocks = nb;
    sa.layers = plan.rc.layers;
    sa.nhull = (const uint8_t *)nhull.ptr;
    sa.hpass = (const uint8_t *)hpass.ptr;
    sa.hkey = (const uint64_t *)hkey.ptr;
    sa.rates = (const int32_t *)rates.ptr;
    sa.hbytes = (const unsigned long long *)pcrd_hb.ptr;
    sa.hcount = (const uint32_t *)pcrd_hc.ptr;
    sa.budget = (const int64_t *)budget.ptr;
    sa.lkey = (uint64_t *)sel_key.ptr;
    sa.lsize = (uint32_t *)sel_size.ptr;
    sa.ctl = (uint32_t *)sel_ctl.ptr;
    sa.K = (uint64_t *)thr.ptr;
    sa.Kc = (uint64_t *)thr.ptr + (size_t)G * kMaxLayers;
    sa.grp_b0 = (const int32_t *)grptab.ptr;
    sa.grp_seg0 = (const uint32_t *)grptab.ptr + G + 1;
    sa.lossless = plan.rc.rate_bpp <= 0.0;
    sa.gtot = (const unsigned long long *)gtot.ptr;
    for (int l = 0; l < plan.rc.layers; l++) sa.frac[l] = lossless_layer_frac(l, plan.rc.layers);
    sa.init_on = init != nullptr;
    if (init) sa.init = *init;
    sa.rs = rs;
    sa.budget_w = (int64_t *)budget.ptr;
    sa.dbg = nullptr;
#ifdef JP2HIP_DEBUG_DUMPS
    if (getenv("JP2HIP_DUMP_DIR")) {
        std::string e;
        if (ensure<int64_t>(dbgsel, 128, e)) sa.dbg = (int64_t *)dbgsel.ptr;
    }
#endif
    hipLaunchKernelGGL(k_select, dim3((grp_max_blocks(plan) + kSelThreads - 1) / kSelThreads, G), dim3(kSelThreads), 0,
                       stream, sa);
    hipLaunchKernelGGL(k_select_resolve, dim3(plan.rc.layers, G), dim3(kSelThreads), 0, stream, sa);
}

// lossless "-rate -": each -flush_period stripe (rate-control group) keeps
// per layer the passes that fit lossless_layer_frac of its own tier-1 bytes
// (k_hull summed them per group); the last layer takes every pass
bool GpuEncoder::select_lossless(const Plan &plan, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    HIPCHECK(hipEventRecord(ev[6], stream));
    select_launch(plan, nullptr);
    HIPCHECK(hipGetLastError());
    return apply_thresholds(plan, nullptr, err);
}

bool GpuEncoder::select_keys(const Plan &plan, const std::vector<uint64_t> &K, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    if (plan.ngroups() != 1) {
        err = "select_keys: one rate-control group expected";
        return false;
    }
    if (!h2d(thr.ptr, K.data(), sizeof(uint64_t) * plan.rc.layers, err)) return false;
    HIPCHECK(hipEventRecord(ev[6], stream));
    return apply_thresholds(plan, nullptr, err);
}

// per-block layer tables for the thresholds in `thr` (ev[6] already recorded)
bool GpuEncoder::apply_thresholds(const Plan &plan, const int *halt, std::string &err) {
    const int nb = (int)plan.blocks.size();
    const int L = plan.rc.layers;
    ApplyArgs aa;
    aa.halt = halt;
    aa.nblocks = nb;
    aa.layers = L;
    aa.lossless = plan.rc.rate_bpp <= 0.0;
    aa.nhull = (const uint8_t *)nhull.ptr;
    aa.hpass = (const uint8_t *)hpass.ptr;
    aa.npasses = (const uint8_t *)npasses.ptr;
    aa.hkey = (const uint64_t *)hkey.ptr;
    aa.K = (const uint64_t *)thr.ptr;
    aa.rates = (const int32_t *)rates.ptr;
    aa.nl = (uint8_t *)nl.ptr;
    aa.lrate = (int32_t *)lrate.ptr;
    aa.ngroups = plan.ngroups();
    aa.grp_b0 = (const int32_t *)grptab.ptr;
    // (k_t2_wave assigns the layers itself in its sizing pass)
    if (nb && !t2_wave) hipLaunchKernelGGL(k_apply, dim3((nb + 255) / 256), dim3(256), 0, stream, aa);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(ev[7], stream));
    return true;
}

// Device rate loop (RateState, jp2hip_internal.h): the first k_select of a
// restart writes the initial state; the step itself is rate_step in
// device_common.h, run by the sizing totals (t2_total_body: the last
// workgroup of k_t2_wave<false>, or k_t2_total)
bool GpuEncoder::rate_loop(const Plan &plan, const RateState &init, bool restart, int batch, bool profile,
                           StageTimes &st, RateState &rs, T2Summary &sum, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    if (!ensure<RateState>(rstate, 1, err)) return false;
    if (!h_rs) {  // host-mapped: k_rate_step writes the state and summary here
        HIPCHECK(hipHostMalloc((void **)&h_rs, sizeof(RateState) + sizeof(T2Summary), hipHostMallocMapped));
        HIPCHECK(hipHostGetDevicePointer((void **)&d_rs_out, h_rs, 0));
    }
    RateState *o_rs = d_rs_out;
    T2Summary *o_sum = (T2Summary *)(d_rs_out + 1);
    RateState *d = (RateState *)rstate.ptr;
    const int *halt = &d->halt;
    HIPCHECK(hipEventRecord(ev[6], stream));
    (void)o_sum;
    for (int i = 0; i < batch; i++) {
        // (the first k_select of a restart also initialises the loop's state)
        select_launch(plan, halt, (restart && i == 0) ? &init : nullptr, d);
        if (!apply_thresholds(plan, halt, err)) return false;
        t2_size_launch(plan, true, halt, d, o_rs);
    }
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(ev[9], stream));
    if (!host_wait(err)) return false;
#ifdef JP2HIP_DEBUG_DUMPS
    if (const char *dd = getenv("JP2HIP_DUMP_DIR"))
        if (dbgsel.ptr && !dump(dd, "seldbg.bin", dbgsel, 128 * 8, err)) return false;
#endif
    std::atomic_thread_fence(std::memory_order_acquire);
    std::memcpy(&sum, h_rs + 1, sizeof sum);
    std::memcpy(&rs, h_rs, sizeof rs);
    if (profile) {
        float t;
        HIPCHECK(hipEventElapsedTime(&t, ev[6], ev[9]));
        st.t2 += t;
    }
    return true;
}

bool GpuEncoder::segments(const Plan &plan, std::vector<uint64_t> &keys, std::vector<int64_t> &cum,
                          std::string &err) {
    HIPCHECK(hipSetDevice(device));
    // every hull segment (key, bytes), listed on the device, sorted here by
    // key, descending (the tile-split exchange's input; the single-image path
    // never needs the whole order: k_select)
    const int nb = (int)plan.blocks.size();
    keys.clear();
    cum.clear();
    if (!nb) return true;
    if (!ensure<int32_t>(segcnt, nb, err) || !ensure<int32_t>(segoff, nb, err) ||
        !ensure<uint64_t>(segkey, std::max(nseg, 1), err) || !ensure<int64_t>(segval, std::max(nseg, 1), err))
        return false;
    hipLaunchKernelGGL(k_seg_offsets, dim3(1), dim3(kSegThreads), 0, stream, nb, (const uint8_t *)nhull.ptr,
                       (int32_t *)segcnt.ptr, (int32_t *)segoff.ptr);
    hipLaunchKernelGGL(k_seg_emit, dim3((nb + 255) / 256), dim3(256), 0, stream, nb, (const uint8_t *)nhull.ptr,
                       (const uint8_t *)hpass.ptr, (const uint64_t *)hkey.ptr, (const int32_t *)rates.ptr,
                       (const int32_t *)segoff.ptr, (uint64_t *)segkey.ptr, (int64_t *)segval.ptr);
    HIPCHECK(hipGetLastError());
    int32_t *tail = (int32_t *)(h_tot + 5);  // pinned
    tail[0] = tail[1] = 0;
    HIPCHECK(hipMemcpyAsync(&tail[0], (int32_t *)segoff.ptr + nb - 1, 4, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipMemcpyAsync(&tail[1], (int32_t *)segcnt.ptr + nb - 1, 4, hipMemcpyDeviceToHost, stream));
    if (!host_wait(err)) return false;
    const int n = tail[0] + tail[1];
    std::vector<uint64_t> k((size_t)n);
    std::vector<int64_t> v((size_t)n);
    if (n > 0) {
        HIPCHECK(hipMemcpyAsync(k.data(), segkey.ptr, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipMemcpyAsync(v.data(), segval.ptr, sizeof(int64_t) * n, hipMemcpyDeviceToHost, stream));
    }
    if (!host_wait(err)) return false;
    std::vector<int> idx((size_t)n);
    for (int i = 0; i < n; i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](int x, int y) { return k[x] > k[y]; });
    keys.resize((size_t)n);
    cum.resize((size_t)n);
    int64_t acc = 0;
    for (int i = 0; i < n; i++) {
        keys[i] = k[idx[i]];
        acc += v[idx[i]];
        cum[i] = acc;
    }
    return true;
}

}  // namespace jp2hip
