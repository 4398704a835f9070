// lzw.hip -- TIFF LZW strips (compression 5) decoded segment-parallel.
//
// A strip is one MSB-first code stream, and decoding it code by code is a
// serial chain (k_unlzw in kernels.hip, ~0.35 us per code on one lane).  The
// format has more parallelism than that:
//
//  * Between two Clear codes (a *segment*) the dictionary grows by one entry
//    per code, so the width of the k-th code of a segment is a fixed
//    function of k (9 bits for k < 254, 10 to 765, 11 to 1789, then 12) and
//    its bit offset a closed-form sum.  64 lanes read 64 consecutive codes at
//    once and a ballot finds the next Clear / EOI: one wave per strip lists
//    its segments (k_lzw_scan), ~60 code reads per wave instruction.
//  * Inside a segment, code k >= 258 names entry E = code, created while
//    decoding code j = E - 257 as string(code j-1) + first byte of string(code
//    j), i.e. string(k) = string(p) + F[p+1] with p = E - 258 < k.  So every
//    code has a parent index, its length is (depth in that forest) + 1 and its
//    first byte F is its root's literal: pointer jumping over the segment's
//    codes in LDS gives both for all codes together (k_lzw_len, k_lzw_emit).
//  * A segment's output size is the sum of its code lengths, a strip's
//    segment offsets are a scan (k_lzw_offsets), and every code's bytes are
//    then written independently: byte L-1 of string(k) is F[p+1], byte L-2 is
//    F[p'+1] for p' = parent(p), ..., byte 0 is F[k] -- lane per code.
//
// Results, truncation at the strip size and error codes are those of the
// serial decoder (and of libtiff): decoding stops once the strip is full; an
// invalid code before that, or a stream that ends early, is error 2; the old
// (LSB-first) LZW flavour is error 4.  Strips with more segments than their
// slice holds, or a segment longer than kLzwSegMax codes (encoders that do
// not clear a full dictionary), are decoded by k_unlzw instead.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "gpu_encoder.h"

namespace jp2hip {

__global__ void k_unlzw(UnpackArgs a);  // kernels.hip (serial fallback)

constexpr int kLzwSegMax = 4096;        // codes of a segment handled in LDS (libtiff: <= 3837)
constexpr int kLzwScanWin = 16384;      // k_lzw_scan input window (bytes)
constexpr int kLzwSegIn = (kLzwSegMax * 12) / 8 + 96;  // a segment's input bytes + alignment slack
constexpr uint32_t kLzwBad = 0xFFFFFFFFu;

// width of the k-th code after a Clear, and the bits of codes 0..k-1
__host__ __device__ inline int lzw_width(uint32_t k) { return k < 254 ? 9 : k < 766 ? 10 : k < 1790 ? 11 : 12; }
__host__ __device__ inline uint64_t lzw_bits(uint32_t k) {
    if (k <= 254) return 9ull * k;
    if (k <= 766) return 2286ull + 10ull * (k - 254);
    if (k <= 1790) return 7406ull + 11ull * (k - 766);
    return 18670ull + 12ull * (k - 1790);
}

// segment slice of a strip: room for n / 512 + 64 segments (libtiff clears
// every ~5.7 KB of input)
__host__ __device__ inline uint64_t lzw_slice_cap(uint64_t n) { return n / 512 + 64; }

struct LzwArgs {
    UnpackArgs u;
    const uint64_t *slice;  // first segment slot of each strip
    uint64_t *seg_bit;      // segment: bit offset of its first code
    uint32_t *seg_n;        // codes in the segment
    uint32_t *seg_len;      // output bytes (codes before the first invalid one)
    uint32_t *seg_bad;      // first invalid code (kLzwBad: none)
    uint64_t *seg_out;      // output offset in the strip (k_lzw_offsets)
    uint32_t *nseg;         // per strip
    int *serial;            // per strip: decode with k_unlzw
};

// Input bytes [base, base + len) of stream `in` (n bytes) into LDS, from
// the 16-byte aligned address at or below in + base: byte base + i lands at
// dst[head + i] (head returned), bytes outside the stream read as 0.  A
// 16-byte aligned chunk holding a stream byte lies in that byte's page, so no
// load leaves the mapped buffer.
__device__ __forceinline__ int lzw_stage(uint8_t *dst, const uint8_t *in, uint64_t n, uint64_t base, int len,
                                         int lane) {
    const uintptr_t a0 = (uintptr_t)in + base;
    const uintptr_t al = a0 & ~(uintptr_t)15;
    const int head = (int)(a0 - al);
    const uintptr_t lo = (uintptr_t)in, end = (uintptr_t)in + n;
    for (int c = lane; c * 16 < head + len; c += 64) {
        const uintptr_t at = al + 16 * (uintptr_t)c;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (at < end && at + 16 > lo) {
            v = *(const uint4 *)at;
            if (at < lo || at + 16 > end) {  // a chunk at either end of the stream
                uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    const uintptr_t x = at + j;
                    if (x < lo || x >= end) w[j >> 2] &= ~(0xFFu << (8 * (j & 3)));
                }
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
        *(uint4 *)(dst + 16 * c) = v;
    }
    return head;
}

// code at stream bit b (width w) from LDS bytes staged from byte `base`
__device__ __forceinline__ uint32_t lzw_read(const uint8_t *buf, int head, uint64_t base, uint64_t b, int w) {
    const uint32_t o = (uint32_t)((b >> 3) - base) + (uint32_t)head;
    const uint32_t v = ((uint32_t)buf[o] << 16) | ((uint32_t)buf[o + 1] << 8) | buf[o + 2];
    return (v >> (24 - (int)(b & 7) - w)) & ((1u << w) - 1u);
}

// ---- segments of each strip: one wave per strip ----
__global__ void __launch_bounds__(64) k_lzw_scan(LzwArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t win[kLzwScanWin + 16];
    const int s = blockIdx.x, lane = threadIdx.x;
    if (s >= a.u.nstrips) return;
    const uint8_t *in = a.u.src + a.u.off[s];
    const uint64_t n = a.u.cnt[s], nbits = 8 * n;
    const uint64_t slot0 = a.slice[s], cap = lzw_slice_cap(n);
    if (n >= 2 && in[0] == 0 && (in[1] & 1)) {  // pre-TIFF 6.0 (LSB-first) LZW, as libtiff detects it
        if (lane == 0) {
            atomicOr(a.u.err, 4);
            a.nseg[s] = 0;
            a.serial[s] = 0;
        }
        return;
    }
    uint64_t wbase = 0;
    int head = 0;
    bool loaded = false;
    uint64_t bit = 0;  // first bit of the current segment
    uint32_t k = 0, ns = 0;
    int serial = 0;
    for (;;) {
        const uint64_t lo = (bit + lzw_bits(k)) >> 3;  // lane 0's first byte (the chunk spans < 100 bytes)
        if (!loaded || lo < wbase || lo + 128 > wbase + kLzwScanWin) {
            wbase = lo;
            head = lzw_stage(win, in, n, wbase, kLzwScanWin, lane);
            loaded = true;
        }
        const uint32_t kk = k + lane;
        const int w = lzw_width(kk);
        const uint64_t b = bit + lzw_bits(kk);
        const bool valid = b + (uint64_t)w <= nbits;
        const uint32_t code = valid ? lzw_read(win, head, wbase, b, w) : 0u;
        const uint64_t stop = __ballot(!valid || code == 256u || code == 257u);
        if (!stop) {
            k += 64;
            continue;
        }
        const int f = __builtin_ctzll(stop);
        const uint32_t kend = k + (uint32_t)f;  // codes of this segment
        const uint32_t ce = (uint32_t)__shfl((int)code, f, 64);
        const bool ve = __shfl((int)valid, f, 64) != 0;
        if (kend > 0) {
            if (ns >= cap || kend > (uint32_t)kLzwSegMax) {
                serial = 1;
                break;
            }
            if (lane == 0) {
                a.seg_bit[slot0 + ns] = bit;
                a.seg_n[slot0 + ns] = kend;
            }
            ns++;
        }
        if (!ve || ce == 257u) break;  // input exhausted / end of information
        bit += lzw_bits(kend) + (uint64_t)lzw_width(kend);  // past the Clear
        k = 0;
    }
    if (lane == 0) {
        a.nseg[s] = ns;
        a.serial[s] = serial;
    }
}

// One segment in LDS: codes, then pointer jumping over the parent links
// (bits 0-12 ancestor, 13-25 distance to it, bit 31 = the ancestor is a
// literal root).  Returns the first invalid code (kLzwBad: none); fills F
// (first byte) and L (length) of every code before it.
struct LzwSegLds {
    __attribute__((aligned(16))) uint8_t in[kLzwSegIn];
    uint16_t code[kLzwSegMax];
    uint32_t link[kLzwSegMax];
    uint8_t first[kLzwSegMax];
};
__device__ uint32_t lzw_segment(LzwSegLds &S, const uint8_t *in, uint64_t n, uint64_t bit0, uint32_t nc, int lane) {
    const uint64_t base = bit0 >> 3;
    const int len = (int)(((bit0 + lzw_bits(nc)) >> 3) - base) + 3;
    const int head = lzw_stage(S.in, in, n, base, len, lane);
    uint32_t bad = kLzwBad;
    for (uint32_t k0 = 0; k0 < nc; k0 += 64) {
        const uint32_t k = k0 + lane;
        uint32_t c = 0;
        bool inv = false;
        if (k < nc) {
            c = lzw_read(S.in, head, base, bit0 + lzw_bits(k), lzw_width(k));
            inv = c > 257u + k;  // an entry not yet defined (257 + k = the one being defined)
            S.code[k] = (uint16_t)c;
            S.link[k] = (c < 256u || inv) ? (0x80000000u | k) : ((c - 258u) | (1u << 13));
        }
        const uint64_t m = __ballot(inv);
        if (m && bad == kLzwBad) bad = k0 + (uint32_t)__builtin_ctzll(m);
    }
    const uint32_t ne = bad == kLzwBad ? nc : bad;  // codes decoded
    for (;;) {  // pointer jumping (in place: each link stays "distance to its ancestor")
        bool open = false;
        for (uint32_t k0 = 0; k0 < ne; k0 += 64) {
            const uint32_t k = k0 + lane;
            if (k >= ne) continue;
            const uint32_t e = S.link[k];
            if (e & 0x80000000u) continue;
            const uint32_t f = S.link[e & 0x1FFFu];
            S.link[k] = (f & 0x80000000u) | (f & 0x1FFFu) | ((((e >> 13) & 0x1FFFu) + ((f >> 13) & 0x1FFFu)) << 13);
            open |= !(f & 0x80000000u);
        }
        if (!__any(open)) break;
    }
    for (uint32_t k0 = 0; k0 < ne; k0 += 64) {
        const uint32_t k = k0 + lane;
        if (k < ne) S.first[k] = (uint8_t)S.code[S.link[k] & 0x1FFFu];
    }
    return bad;
}
__device__ __forceinline__ uint32_t lzw_len(const LzwSegLds &S, uint32_t k) { return ((S.link[k] >> 13) & 0x1FFFu) + 1u; }

// ---- segment output sizes: one wave per segment ----
__global__ void __launch_bounds__(64) k_lzw_len(LzwArgs a) {
    extern __shared__ uint8_t lds[];
    LzwSegLds &S = *(LzwSegLds *)lds;
    const int s = blockIdx.x, lane = threadIdx.x;
    if (s >= a.u.nstrips || a.serial[s]) return;
    const uint8_t *in = a.u.src + a.u.off[s];
    const uint64_t n = a.u.cnt[s];
    const uint32_t ns = a.nseg[s];
    for (uint32_t i = blockIdx.y; i < ns; i += gridDim.y) {
        const uint64_t slot = a.slice[s] + i;
        const uint32_t nc = a.seg_n[slot];
        const uint32_t bad = lzw_segment(S, in, n, a.seg_bit[slot], nc, lane);
        const uint32_t ne = bad == kLzwBad ? nc : bad;
        uint32_t t = 0;
        for (uint32_t k = lane; k < ne; k += 64) t += lzw_len(S, k);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) t += (uint32_t)__shfl_xor((int)t, o, 64);
        if (lane == 0) {
            a.seg_len[slot] = t;
            a.seg_bad[slot] = bad;
        }
    }
}

// ---- segment offsets and the strip's errors: thread per strip ----
__global__ void __launch_bounds__(64) k_lzw_offsets(LzwArgs a) {
    const int s = blockIdx.x * 64 + threadIdx.x;
    if (s >= a.u.nstrips || a.serial[s]) return;
    const uint64_t cap = strip_out_bytes(a.u, s);
    const uint64_t slot0 = a.slice[s];
    const uint32_t ns = a.nseg[s];
    uint64_t acc = 0;
    bool ended = false;  // an invalid code ends the decode
    for (uint32_t i = 0; i < ns; i++) {
        a.seg_out[slot0 + i] = ended ? cap : acc;  // segments after an invalid code write nothing
        if (ended) continue;
        acc += a.seg_len[slot0 + i];
        if (a.seg_bad[slot0 + i] != kLzwBad) ended = true;
    }
    // the serial decoder stops once the strip is full: an invalid code or the
    // end of the codes before that is an error
    if (acc < cap) atomicOr(a.u.err, 2);
}

// ---- every code's bytes: one wave per segment, lane per code ----
__global__ void __launch_bounds__(64) k_lzw_emit(LzwArgs a) {
    extern __shared__ uint8_t lds[];
    LzwSegLds &S = *(LzwSegLds *)lds;
    const int s = blockIdx.x, lane = threadIdx.x;
    if (s >= a.u.nstrips || a.serial[s]) return;
    const uint8_t *in = a.u.src + a.u.off[s];
    const uint64_t n = a.u.cnt[s], cap = strip_out_bytes(a.u, s);
    uint8_t *out = a.u.dst + (uint64_t)s * a.u.stride;
    const uint32_t ns = a.nseg[s];
    for (uint32_t i = blockIdx.y; i < ns; i += gridDim.y) {
        const uint64_t slot = a.slice[s] + i;
        const uint64_t o0 = a.seg_out[slot];
        if (o0 >= cap) continue;
        const uint32_t nc = a.seg_n[slot];
        const uint32_t bad = lzw_segment(S, in, n, a.seg_bit[slot], nc, lane);
        const uint32_t ne = bad == kLzwBad ? nc : bad;
        uint64_t run = o0;  // output offset of code k0
        for (uint32_t k0 = 0; k0 < ne && run < cap; k0 += 64) {
            const uint32_t k = k0 + lane;
            const uint32_t L = k < ne ? lzw_len(S, k) : 0u;
            // exclusive prefix of L over the lanes (DPP row shifts, then rows)
            int v = (int)L;
            v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
            v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
            v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
            v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
            v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
            v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
            const uint64_t pos = run + (uint32_t)v - L;
            if (L && pos < cap) {
                out[pos] = S.first[k];
                // bytes L-1 .. 1: F of (parent + 1) up the chain
                uint32_t c = S.code[k];
                for (uint32_t j = L - 1; j >= 1; j--) {
                    const uint32_t p = c - 258u;
                    if (pos + j < cap) out[pos + j] = S.first[p + 1];
                    c = S.code[p];
                }
            }
            run += (uint32_t)__builtin_amdgcn_readlane(v, 63);
        }
    }
}

uint64_t lzw_slices(const uint64_t *strip_bytes, int nstrips, std::vector<uint64_t> &slice) {
    uint64_t segs = 0;
    slice.resize(nstrips);
    for (int s = 0; s < nstrips; s++) {
        slice[s] = segs;
        segs += lzw_slice_cap(strip_bytes[s]);
    }
    return segs;
}
size_t lzw_scratch_bytes(int nstrips, uint64_t segs) {
    // slice[ns] + per segment (bit 8, out 8, n 4, len 4, bad 4) + per strip (nseg 4, serial 4)
    return (size_t)nstrips * 8 + (size_t)segs * 28 + (size_t)nstrips * 8 + 256;
}

bool launch_lzw(const UnpackArgs &u, uint64_t segs, void *scratch, hipStream_t st) {
    const int ns = u.nstrips;
    uint8_t *p = (uint8_t *)scratch;
    LzwArgs a;
    a.u = u;
    a.slice = (const uint64_t *)p;  // uploaded by the caller (lzw_slices)
    p += (size_t)ns * 8;
    a.seg_bit = (uint64_t *)p;
    p += segs * 8;
    a.seg_out = (uint64_t *)p;
    p += segs * 8;
    a.seg_n = (uint32_t *)p;
    p += segs * 4;
    a.seg_len = (uint32_t *)p;
    p += segs * 4;
    a.seg_bad = (uint32_t *)p;
    p += segs * 4;
    a.nseg = (uint32_t *)p;
    p += (size_t)ns * 4;
    a.serial = (int *)p;
    static const bool attr =
        hipFuncSetAttribute((const void *)k_lzw_len, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(LzwSegLds)) == hipSuccess &&
        hipFuncSetAttribute((const void *)k_lzw_emit, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(LzwSegLds)) == hipSuccess;
    if (!attr) return false;
    hipLaunchKernelGGL(k_lzw_scan, dim3(ns), dim3(64), 0, st, a);
    const dim3 gs(ns, 16);
    hipLaunchKernelGGL(k_lzw_len, gs, dim3(64), sizeof(LzwSegLds), st, a);
    hipLaunchKernelGGL(k_lzw_offsets, dim3((ns + 63) / 64), dim3(64), 0, st, a);
    hipLaunchKernelGGL(k_lzw_emit, gs, dim3(64), sizeof(LzwSegLds), st, a);
    // strips the segment tables could not hold: the serial decoder
    UnpackArgs f = u;
    f.only = a.serial;
    hipLaunchKernelGGL(k_unlzw, dim3(ns), dim3(1), 0, st, f);
    return hipGetLastError() == hipSuccess;
}

}  // namespace jp2hip
