// t1.hip -- EBCOT tier-1 (ISO/IEC 15444-1 Annex D) and the MQ coder (Annex C)
// for gfx950, split in two kernels so the serial part is as short as possible:
//
//   k_t1_cm3 context modelling, one wave per code-block (its coded planes
//            top-down), lane = column.  Significance lives in 64-bit column
//            masks (bit r = row r), so the neighbourhood and context rules
//            run bit-sliced for the whole column at once.  The state at the
//            start of plane p is known from the bit-planes (S[p+1] = OR of
//            planes above p), so a plane needs no state from the passes
//            coded before it:
//              - SPP membership is the least fixed point of the causal
//                neighbourhood rule (iterated on the whole masks);
//              - MRP neighbours all see the post-SPP state S[p+1] | N;
//              - CUP neighbours see S[p] (already visited) or S[p+1] | N
//                (not yet visited): closed form, no sample-serial state.
//            Output: the (context, decision) byte stream of the plane's
//            passes plus per-pass counts and the SPP distortion decrease.
//   k_t1_mq  one lane per code-block: runs the MQ coder over the block's
//            streams in pass order, records the truncation length after every
//            pass, terminates the codeword (Annex C.2.9 FLUSH).
//
// The decision order, contexts, truncation lengths and distortion values are
// those of the oracle's sample-at-a-time coder (oracle/jp2_oracle.c,
// oracle_t1_encode); the parity tests compare them byte for byte.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "device_common.h"
#include "gpu_encoder.h"

namespace jp2hip {

enum { CX_RL = 17, CX_UNI = 18, CX_PAD = 19 };
// Every pass stream is padded to a 16-byte boundary with decisions of the
// neutral context CX_PAD, whose MQ state (Qe = 0, MPS = 0) leaves the coder
// unchanged: the MQ kernel codes whole 16-decision chunks with no per-decision
// validity test.
constexpr uint8_t kPadDecision = CX_PAD << 1;


// plane_stream_cap: device_common.h (emit_t1_items places the slots)

constexpr int kCmWaves = 2;  // code-blocks (waves) per workgroup

// MQ lane order: blocks by decreasing decision count, so the lanes of an MQ
// wave carry similar work.  The order only groups blocks (it changes no
// output): bucket = 16 * floor(log2(n + 1)) + the next 4 bits of n + 1 (6.25 %
// wide; 8 / 3 bits before round 4: lanes idle 4.2 -> 2.6 % of the wave-steps,
// simulated on the oracle's per-block counts of C2), largest first; inside a
// bucket the order is whatever the atomics give.  k_t1_cm3 files a block at
// its end (bslots[bucket][i]);
// k_t1_mq maps its lanes through the bucket fills' prefix.
__device__ __forceinline__ int order_bucket(uint32_t n) {
    const uint32_t v = n + 1u;
    const int e = 31 - __clz(v);                                      // 0..31
    constexpr int kLog = kOrderSub == 16 ? 4 : 3;                     // bits of the sub-bucket
    const int f = e >= kLog ? (int)((v >> (e - kLog)) & (kOrderSub - 1u)) : (int)((v << (kLog - e)) & (kOrderSub - 1u));
    return kOrderBuckets - 1 - min(kOrderBuckets - 1, kOrderSub * e + f);  // descending
}


// --------------------------------------------------------------------------
// Context modelling on column masks.  One wavefront per code-block, one
// bit-plane at a time, in the transposed layout: lane
// c holds column c of every mask as a 64-bit word (bit r = row r; k_quant
// writes them), so a vertical neighbour is a bit shift inside the lane and a
// horizontal one is the next lane.  The neighbourhood and context rules then
// run once per (block, plane) for all 64 rows at a time, bit-sliced (a
// context number as four masks), instead of once per sample; per stripe a
// lane only picks its four rows' bits and writes its decision bytes.
//
// Causal states: a neighbour already visited in the scan
// (stripe by stripe, column by column, top to bottom) is seen in the state
// Vb, one not yet visited in Va -- SPP: Vb = S[p+1] | N, Va = S[p+1];
// CUP: Vb = S[p], Va = S[p+1] | N.  For row r, column c: (r-1, c), (r, c-1),
// (r-1, c-1) are visited; (r+1, c), (r, c+1), (r+1, c+1) are not; (r-1, c+1)
// is visited only when r starts a stripe, (r+1, c-1) only when it does not
// end one.
// --------------------------------------------------------------------------
constexpr uint64_t kStripeTop = 0x1111111111111111ull;  // rows with r % 4 == 0
constexpr uint64_t kStripeBot = 0x8888888888888888ull;  // rows with r % 4 == 3

// (DPP whole-wave shifts: lane 0 / 63 get 0, no ds_bpermute round trip)
__device__ __forceinline__ uint64_t col_left(uint64_t x, int) { return wave_shr1(x); }   // column c-1's word
__device__ __forceinline__ uint64_t col_right(uint64_t x, int) { return wave_shl1(x); }  // column c+1's word

// The 8 neighbour masks of every row of the lane's column under (Vb, Va).
struct Nbr8 {
    uint64_t UL, U, UR, L, R, DL, D, DR;
};
__device__ __forceinline__ Nbr8 nbr8(uint64_t Vb, uint64_t Va, uint64_t LVb, uint64_t RVb, uint64_t LVa,
                                     uint64_t RVa) {
    Nbr8 n;
    n.UL = LVb << 1;
    n.U = Vb << 1;
    n.UR = ((RVb << 1) & kStripeTop) | ((RVa << 1) & ~kStripeTop);
    n.L = LVb;
    n.R = RVa;
    n.DL = ((LVa >> 1) & kStripeBot) | ((LVb >> 1) & ~kStripeBot);
    n.D = Va >> 1;
    n.DR = RVa >> 1;
    return n;
}

// A 3-input bitwise function on both 32-bit halves (one v_bitop3_b32 each):
// TT is the function's value on a = 0xF0, b = 0xCC, c = 0xAA (bit a b c of
// the table = f(a, b, c)), e.g. (a & b) | c -> 0xEA.
template <uint32_t TT>
__device__ __forceinline__ uint64_t b3(uint64_t a, uint64_t b, uint64_t c) {
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, TT);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), TT);
    return ((uint64_t)hi << 32) | lo;
}

// Zero-coding context (Table D.1, zc_ctx) of every row, as 4 bit masks.
// The table's cases reduced to a few 3-input functions of the neighbour
// counts (diagonals as a thermometer dge1 / dge2 / dge3, horizontal and
// vertical pairs); checked equal to the case-by-case form on all 256
// neighbourhoods of each band.
struct Ctx4 {
    uint64_t b0, b1, b2, b3;
};
__device__ __forceinline__ Ctx4 zc_masks(int band, const Nbr8 &n) {
    const uint64_t u = n.UL | n.UR, d = n.DL | n.DR, dge1 = u | d;
    const uint64_t s2a = n.DL & n.DR;
    const uint64_t dge2 = b3<0xEA>(u, d, b3<0xEA>(n.UL, n.UR, s2a));  // (u & d) | (UL & UR) | (DL & DR)
    Ctx4 z;
    if (band == 3) {
        const uint64_t dge3 = b3<0xEA>(s2a, u, (n.UL & n.UR) & d);  // three or four diagonals
        const uint64_t a = n.L | n.R, c = n.U | n.D, hvge1 = a | c;
        const uint64_t hvge2 = b3<0xEA>(a, c, b3<0xEA>(n.L, n.R, n.U & n.D));
        const uint64_t d2 = b3<0x30>(dge2, dge3, dge3), d1 = b3<0x30>(dge1, dge2, dge2);  // exactly 2 / 1
        const uint64_t hv1 = b3<0x30>(hvge1, hvge2, hvge2);                              // exactly 1
        z.b3 = dge3;
        z.b2 = b3<0xEA>(d1, hvge1, d2);                                  // d2 | (d1 & hvge1)
        z.b1 = b3<0xAE>(dge1, hvge2, b3<0xBA>(d1, hvge1, d2));           // .. | (d1 & ~hvge1) | (d0 & hvge2)
        z.b0 = b3<0xEA>(d2, hvge1, b3<0x72>(d1, dge1, hv1));             // (d2 & hvge1) | (d1 & ~hv1) | (d0 & hv1)
    } else {
        // A: the pair that counts most (horizontal; vertical for HL), B: the other
        const uint64_t A1 = band == 1 ? n.U : n.L, A2 = band == 1 ? n.D : n.R;
        const uint64_t B1 = band == 1 ? n.L : n.U, B2 = band == 1 ? n.R : n.D;
        const uint64_t e = b3<0x30>(dge1, dge2, dge2);  // exactly one diagonal
        const uint64_t x = A1 ^ A2;                     // exactly one of A
        z.b3 = A1 & A2;
        z.b2 = b3<0x3E>(A1, A2, B1 & B2);               // x | (no A & both B)
        z.b1 = b3<0xEA>(x, B1 | B2 | dge1, b3<0x02>(A1, A2, b3<0x3E>(B1, B2, dge2)));
        z.b0 = b3<0xEA>(x, b3<0xFD>(B1, B2, dge1), b3<0x02>(A1, A2, b3<0x3E>(B1, B2, e)));
    }
    return z;
}

// Sign-coding context (Tables D.2/D.3, sc_lut) of every row: context 9..13
// (bit 3 always set) in b0..b2 and the XOR bit.  A pair of neighbours
// contributes p (their signs sum > 0) or n (< 0); the outputs are functions
// of (hp, hn, vp, vn), checked equal to the table on all 256 cases.
struct Sc4 {
    uint64_t b0, b1, b2, xr;
};
__device__ __forceinline__ void sc_pair(uint64_t As, uint64_t An, uint64_t Bs, uint64_t Bn, uint64_t &p, uint64_t &n) {
    const uint64_t nA = As & An, nB = Bs & Bn;
    const uint64_t pA = b3<0x30>(As, An, An), pB = b3<0x30>(Bs, Bn, Bn);
    p = b3<0xBA>(pB, nA, b3<0x10>(As, An, nB));  // (pA & ~nB) | (pB & ~nA)
    n = b3<0xBA>(nB, pA, b3<0x30>(nA, pB, pB));  // (nA & ~pB) | (nB & ~pA)
}
__device__ __forceinline__ Sc4 sc_masks(uint64_t Ls, uint64_t Ln, uint64_t Rs, uint64_t Rn, uint64_t Us, uint64_t Un,
                                        uint64_t Ds, uint64_t Dn) {
    uint64_t hp, hn, vp, vn;
    sc_pair(Ls, Ln, Rs, Rn, hp, hn);
    sc_pair(Us, Un, Ds, Dn, vp, vn);
    const uint64_t hnz = hp | hn, vnz = vp | vn;
    const uint64_t opp = b3<0xEA>(hn, vp, hp & vn);  // opposite signs
    Sc4 c;
    c.b0 = ~(hnz ^ vnz);               // ctx 9, 11, 13: both zero or both not
    c.b1 = b3<0xAE>(hnz, vnz, opp);     // ctx 10, 11
    c.b2 = b3<0x30>(hnz, opp, opp);     // ctx 12, 13
    c.xr = b3<0xF2>(hn, hnz, vn);       // hn | (h zero & vn)
    return c;
}


// --------------------------------------------------------------------------
// k_t1_cm3: the stripe step, branch-free, and LDS-staged output.
//
// Per stripe a lane (column) builds its four rows' decision bytes at once,
// one byte per row in a dword: the zero-coding byte (ctx << 1 | bit) and the
// sign byte ((8 | ctx) << 1 | sign ^ xor) from the context masks' nibbles,
// spread to byte lanes by one multiply (nibble * 0x204081 & 0x01010101).  The
// member samples' bytes are compacted in scan order by two v_perm_b32 whose
// selectors come from a 256-entry table indexed by (members | members with a
// 1 bit << 4) -- no per-sample branch.  Two stripes at a time, the wave's
// lanes place their <= 12 bytes per stripe at an exclusive prefix of the
// counts (one DPP wave scan of both stripes' counts packed in a dword) in a
// 4 KB LDS ring per wave, OR-ing whole dwords (the ring is zero where nothing
// has been written, and a lane's bytes are zero-padded, so neighbours'
// partial dwords merge); every full KiB leaves the ring in one 16-byte store
// per lane.
// Blocks are taken in a grid-stride loop (the grid is sized to the chip, not
// to the plan's block count).
// --------------------------------------------------------------------------
constexpr int kRingBytes = 4096;  // a stripe pair adds <= 1536 bytes; drains every KiB
constexpr int kRingGuard = 4;     // dwords past the ring: a lane's <= 4 dwords never wrap
constexpr int kRingWords = kRingBytes / 4 + kRingGuard;
constexpr int kCm3Blocks = 4096;  // workgroups (2 waves each) at most

__device__ __forceinline__ uint32_t spread4(uint32_t nib) { return (nib * 0x00204081u) & 0x01010101u; }
// spread4(nib) << k, as one 24-bit multiply (k <= 4: nib << k < 2^24)
__device__ __forceinline__ uint32_t spread4s(uint32_t nib, int k) {
    return __umul24(nib << k, 0x00204081u) & (0x01010101u << k);
}
__device__ __forceinline__ uint32_t nibw(uint32_t w, int sh) { return __builtin_amdgcn_ubfe(w, (uint32_t)sh, 4u); }

// Ring writer state (wave-uniform): `pos` = next byte of the plane's slot,
// `fl` = bytes already stored to HBM (a multiple of 16).
struct Ring {
    uint32_t *r;  // this wave's ring (kRingWords)
    uint8_t *out;
    int pos, fl;
};

// OR this lane's n bytes (o0, o1, o2 little-endian; NW = the dwords they can
// span at any alignment: 2 for <= 4 bytes, 3 for <= 8, 4 for <= 12) into the
// ring at byte `at`: one base address, constant offsets (dwords past the
// ring's end land in its guard, which ring_drain folds back to its start),
// each dword a funnel shift of (o_k : o_k-1) by one v_perm.
template <int NW>
__device__ __forceinline__ void ring_or(const Ring &g, uint32_t at, uint32_t o0, uint32_t o1, uint32_t o2,
                                        uint32_t n) {
    const uint32_t t = at & 3u;
    const uint32_t sel = 0x07060504u - __builtin_amdgcn_perm(0u, t, 0u);  // byte j: 4 + j - t
    uint32_t *q = g.r + ((at >> 2) & (uint32_t)(kRingBytes / 4 - 1));
    if (n) {
        atomicOr(q, o0 << (8u * t));
        atomicOr(q + 1, __builtin_amdgcn_perm(o1, o0, sel));
        if (NW >= 3) atomicOr(q + 2, __builtin_amdgcn_perm(o2, o1, sel));
        if (NW >= 4) atomicOr(q + 3, __builtin_amdgcn_perm(0u, o2, sel));
    }
}

// Two consecutive stripes' bytes (A then B, each in column order) at pos:
// ONE wave scan of both counts packed in a dword (<= 768 each), so a stripe
// pair costs one DPP scan; advances pos.
template <int NW>
__device__ __forceinline__ void ring_put2(Ring &g, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t na, uint32_t b0,
                                          uint32_t b1, uint32_t b2, uint32_t nb) {
    // inclusive scan over the wave: DPP row shifts 1, 2, 4, 8, then lane 15
    // into 16..31 / 47 into 48..63 and lane 31 into 32..63
    const uint32_t n = na | (nb << 16);
    int v = (int)n;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane(v, 63);
    const uint32_t ex = (uint32_t)v - n;  // exclusive prefixes, packed
    const uint32_t ta = tot & 0xFFFFu;
    ring_or<NW>(g, (uint32_t)g.pos + (ex & 0xFFFFu), a0, a1, a2, na);
    ring_or<NW>(g, (uint32_t)g.pos + ta + (ex >> 16), b0, b1, b2, nb);
    g.pos += (int)(ta + (tot >> 16));
}

// Store ring bytes [fl, upto) (upto a multiple of 16) and zero them; the
// guard's dwords (bytes that ran past the ring's end) are first OR-ed into
// the ring's first dwords.  (Safe: pending bytes stay below 2560, well inside
// the ring, so the ring's first dwords of the previous lap were stored and
// zeroed before any lane reached its end again.)
__device__ __forceinline__ void ring_drain(Ring &g, int upto, int lane) {
    if (lane < kRingGuard) {
        const uint32_t gv = g.r[kRingBytes / 4 + lane];
        if (gv) {
            g.r[lane] |= gv;
            g.r[kRingBytes / 4 + lane] = 0u;
        }
    }
    __builtin_amdgcn_wave_barrier();
    for (int o = g.fl + 16 * lane; o < upto; o += 1024) {
        uint4 *src = (uint4 *)((uint8_t *)g.r + (o & (kRingBytes - 1)));
        const uint4 v = *src;
        *src = make_uint4(0u, 0u, 0u, 0u);
        *(uint4 *)(g.out + o) = v;
    }
    g.fl = __builtin_amdgcn_readfirstlane(upto);
}

// After a stripe pair: whole KiBs leave the ring (a pair adds <= 1536 bytes,
// so at most 2560 of the ring's 4096 are pending).
__device__ __forceinline__ void ring_step(Ring &g, int lane) {
    // (wave-uniform: a scalar branch)
    if (__builtin_amdgcn_readfirstlane(g.pos - g.fl) >= 1024) ring_drain(g, g.fl + 1024, lane);
}

// Pass end: neutral decisions to the next 16-byte boundary, every byte out.
__device__ __forceinline__ void ring_pass_end(Ring &g, int lane) {
    const int end = (g.pos + 15) & ~15;
    if (lane < end - g.pos) ((uint8_t *)g.r)[(g.pos + lane) & (kRingBytes - 1)] = kPadDecision;
    ring_drain(g, end, lane);
    g.pos = end;
}

// 32-bit halves of the masks a stripe step reads
struct Half {
    uint32_t mem, bb, z0, z1, z2, z3, c0, c1, c2, xs, x;
};
__device__ __forceinline__ Half half_of(int hf, uint64_t mem, uint64_t bb, const Ctx4 &z, const Sc4 &sc, uint64_t xs,
                                        uint64_t x) {
    const int sh = hf * 32;
    return Half{(uint32_t)(mem >> sh),  (uint32_t)(bb >> sh),    (uint32_t)(z.b0 >> sh), (uint32_t)(z.b1 >> sh),
                (uint32_t)(z.b2 >> sh), (uint32_t)(z.b3 >> sh),  (uint32_t)(sc.b0 >> sh), (uint32_t)(sc.b1 >> sh),
                (uint32_t)(sc.b2 >> sh), (uint32_t)(xs >> sh), (uint32_t)(x >> sh)};
}
// the four rows' zero-coding bytes and sign bytes of a stripe
// (bit k of each byte: a 24-bit multiply by 0x204081 << k for k <= 2, whose
// constant still fits 24 bits -- no shift of the nibble -- else spread4s)
__device__ __forceinline__ uint32_t spread_or(uint32_t w, int sh, int k, uint32_t acc) {
    const uint32_t nib = nibw(w, sh);
    if (k <= 2) return (__umul24(nib, 0x00204081u << k) & (0x01010101u << k)) | acc;
    return spread4s(nib, k) | acc;  // (nib << k) * 0x204081: no 32-bit multiply
}
__device__ __forceinline__ void zc_sg_bytes(const Half &m, int sh, uint32_t &zc, uint32_t &sg) {
    zc = spread_or(m.bb, sh, 0, 0u);
    zc = spread_or(m.z0, sh, 1, zc);
    zc = spread_or(m.z1, sh, 2, zc);
    zc = spread_or(m.z2, sh, 3, zc);
    zc = spread_or(m.z3, sh, 4, zc);
    sg = spread_or(m.xs, sh, 0, 0x10101010u);
    sg = spread_or(m.c0, sh, 1, sg);
    sg = spread_or(m.c1, sh, 2, sg);
    sg = spread_or(m.c2, sh, 3, sg);
}

// One stripe's decision bytes of each pass (sh = its nibble in the half):
// members in scan order, each its zero-coding byte then (CUP/SPP, when its
// bit is 1) its sign byte; n bytes.
__device__ __forceinline__ void spp_stripe(const Half &m, int sh, const uint2 *lut, uint32_t &o0, uint32_t &o1,
                                           uint32_t &n) {
    const uint32_t mem = nibw(m.mem, sh);
    uint32_t zc, sg;
    zc_sg_bytes(m, sh, zc, sg);
    const uint32_t K = mem | ((mem & nibw(m.bb, sh)) << 4);
    const uint2 sel = lut[K];
    o0 = __builtin_amdgcn_perm(sg, zc, sel.x);
    o1 = __builtin_amdgcn_perm(sg, zc, sel.y);
    n = (uint32_t)__popc(K);
}
// ctx 14 (first refinement), 15 (... with a significant neighbour), 16
// (later refinements): bytes 0x1C, 0x1E, 0x20 -- 0x20 - 4 f per byte (f =
// first refinement, 0 / 1), no borrow across bytes; the neighbour flag (a
// subset of f) in bit 1, the refinement bit in bit 0
__device__ __forceinline__ void mrp_stripe(uint32_t wm, uint32_t wb, uint32_t wf, uint32_t wa, int sh,
                                           const uint2 *lut, uint32_t &o0, uint32_t &n) {
    const uint32_t mem = nibw(wm, sh);
    const uint32_t f = spread4(nibw(wf, sh));
    const uint32_t mr = (0x20202020u - (f << 2)) | spread_or(wa, sh, 1, spread4(nibw(wb, sh)));
    o0 = __builtin_amdgcn_perm(0u, mr, lut[mem].x);
    n = (uint32_t)__popc(mem);
}
__device__ __forceinline__ void cup_stripe(const Half &m, int sh, const uint2 *lut, uint32_t &o0, uint32_t &o1,
                                           uint32_t &o2, uint32_t &n) {
    const uint32_t mem = nibw(m.mem, sh);
    uint32_t zc, sg;
    zc_sg_bytes(m, sh, zc, sg);
    const uint32_t bb = nibw(m.bb, sh);
    // four members, none with a significant neighbour (mem == 0xF implies
    // the stripe's four rows lie inside the block)
    const bool rl = mem == 0xFu && nibw(m.x, sh) == 0u;
    const uint32_t r = __builtin_ctz(bb | 16u);
    const uint32_t mr = rl ? (0xEu << r) & 0xFu : mem;  // samples coded normally
    const uint32_t K = mr | ((mr & bb) << 4);
    const uint2 sel = lut[K];
    o0 = __builtin_amdgcn_perm(sg, zc, sel.x);
    o1 = __builtin_amdgcn_perm(sg, zc, sel.y);
    o2 = 0u;
    n = (uint32_t)__popc(K);
    if (rl) {  // run-length prefix: RL 0 alone, or RL 1, two UNI bits, row r's sign
        if (bb == 0u) {
            o0 = (uint32_t)(CX_RL << 1);
            n = 1;
        } else {
            o2 = o1;
            o1 = o0;
            o0 = (uint32_t)((CX_RL << 1) | 1) | ((uint32_t)((CX_UNI << 1) | (r >> 1)) << 8) |
                 ((uint32_t)((CX_UNI << 1) | (r & 1u)) << 16) | (((sg >> (8 * r)) & 0xFFu) << 24);
            n += 4;
        }
    }
}

// One bit-plane p (depth k = P-1-p) of block b: the three passes' decision
// bytes through the wave's ring into the plane's stream slot, the pass counts
// and the SPP distortion decrease stored; returns the plane's decisions.
// B, S0 = S[p], S1 = S[p+1], S2 = S[p+2] and SG are the lane's column masks
// (0 past the block width, S1 / S2 0 above the top plane).
__device__ __forceinline__ uint32_t cm_plane(const T1CmArgs &a, Ring &g, const uint2 *lut, int lane, int b, int k,
                                             int p, int P, int w, int h, int band, const uint64_t *CT, uint64_t B,
                                             uint64_t S0, uint64_t S1, uint64_t S2, uint64_t SG, uint64_t LSG,
                                             uint64_t RSG) {
    const bool lossless = a.lossless != 0;
    const bool vl = lane < w;
    const uint64_t VR = vl ? (h >= 64 ? ~0ull : ((1ull << h) - 1ull)) : 0ull;
    const int nstripes = (h + 3) >> 2;
    g.out = a.stream + a.slot_off[b] + (size_t)k * plane_stream_cap(w, h);
    g.pos = 0;
    g.fl = 0;
    int n_spp = 0, n_mrp = 0;
    const bool spp = p < P - 1;
    const uint64_t LS1 = col_left(S1, lane), RS1 = col_right(S1, lane);
    uint64_t N = 0, memS = 0;
    if (spp) {
        // ---- significance propagation: least fixed point of the causal rule ----
        for (;;) {
            const uint64_t Vb = S1 | N, LVb = col_left(Vb, lane), RVb = col_right(Vb, lane);
            const Nbr8 nb = nbr8(Vb, S1, LVb, RVb, LS1, RS1);
            const uint64_t cand = ~S1 & VR & (nb.UL | nb.U | nb.UR | nb.L | nb.R | nb.DL | nb.D | nb.DR);
            const uint64_t Nn = cand & B;
            if (!__any(Nn != N)) {
                memS = cand;
                break;
            }
            N = Nn;
        }
        {
            const uint64_t Vb = S1 | N, LVb = col_left(Vb, lane), RVb = col_right(Vb, lane);
            const Nbr8 nb = nbr8(Vb, S1, LVb, RVb, LS1, RS1);
            const Ctx4 z = zc_masks(band, nb);
            const Sc4 sc = sc_masks(nb.L, LSG, nb.R, RSG, nb.U, SG << 1, nb.D, SG >> 1);
            for (int hf = 0; hf * 8 < nstripes; hf++) {
                const Half m = half_of(hf, memS, B, z, sc, SG ^ sc.xr, 0);
                // stripe pairs (A, B = A + 1; B past the block: no members)
                for (int s4 = 0; s4 < 8 && hf * 8 + s4 < nstripes; s4 += 2) {
                    const int sh = s4 * 4;
                    const bool hb = hf * 8 + s4 + 1 < nstripes;
                    if (!__any(nibw(m.mem, sh) | (hb ? nibw(m.mem, sh + 4) : 0u))) continue;
                    uint32_t a0, a1, ca, b0 = 0, b1 = 0, cb = 0;
                    spp_stripe(m, sh, lut, a0, a1, ca);
                    if (hb) spp_stripe(m, sh + 4, lut, b0, b1, cb);
                    ring_put2<3>(g, a0, a1, 0u, ca, b0, b1, 0u, cb);
                    ring_step(g, lane);
                }
            }
        }
        n_spp = g.pos;
        ring_pass_end(g, lane);
        const int mrp0 = g.pos;
        // ---- magnitude refinement: neighbours in the post-SPP state ----
        {
            const uint64_t Pst = S1 | N, LP = col_left(Pst, lane), RP = col_right(Pst, lane);
            const uint64_t anyn = (Pst << 1) | (Pst >> 1) | LP | RP | (LP << 1) | (RP << 1) | (LP >> 1) | (RP >> 1);
            const uint64_t memM = S1 & VR, fr = S1 & ~S2, fa = fr & anyn;
            for (int hf = 0; hf * 8 < nstripes; hf++) {
                const int hs = hf * 32;
                const uint32_t wm = (uint32_t)(memM >> hs), wb = (uint32_t)(B >> hs), wf = (uint32_t)(fr >> hs),
                               wa = (uint32_t)(fa >> hs);
                for (int s4 = 0; s4 < 8 && hf * 8 + s4 < nstripes; s4 += 2) {
                    const int sh = s4 * 4;
                    const bool hb = hf * 8 + s4 + 1 < nstripes;
                    if (!__any(nibw(wm, sh) | (hb ? nibw(wm, sh + 4) : 0u))) continue;
                    uint32_t a0, ca, b0 = 0, cb = 0;
                    mrp_stripe(wm, wb, wf, wa, sh, lut, a0, ca);
                    if (hb) mrp_stripe(wm, wb, wf, wa, sh + 4, lut, b0, cb);
                    ring_put2<2>(g, a0, 0u, 0u, ca, b0, 0u, 0u, cb);
                    ring_step(g, lane);
                }
            }
        }
        n_mrp = g.pos - mrp0;
        ring_pass_end(g, lane);
    }
    const int cup0 = g.pos;
    // ---- cleanup: visited neighbours in S[p], the others post-SPP ----
    {
        const uint64_t Pst = S1 | N, LP = col_left(Pst, lane), RP = col_right(Pst, lane);
        const uint64_t LS0 = col_left(S0, lane), RS0 = col_right(S0, lane);
        const Nbr8 nb = nbr8(S0, Pst, LS0, RS0, LP, RP);
        const Ctx4 z = zc_masks(band, nb);
        const Sc4 sc = sc_masks(nb.L, LSG, nb.R, RSG, nb.U, SG << 1, nb.D, SG >> 1);
        const uint64_t memC = ~S1 & ~memS & VR;
        // run-length mode blocked by a significant neighbour: left column
        // (visited) in S[p], right column post-SPP, the row above a stripe
        // in S[p], the row below it post-SPP
        const uint64_t side = LS0 | RP, above = S0 | LS0 | RS0, below = Pst | LP | RP;
        const uint64_t blk = side | ((above << 1) & kStripeTop) | ((below >> 1) & kStripeBot);
        for (int hf = 0; hf * 8 < nstripes; hf++) {
            const Half m = half_of(hf, memC, B, z, sc, SG ^ sc.xr, blk);
            for (int s4 = 0; s4 < 8 && hf * 8 + s4 < nstripes; s4 += 2) {
                const int sh = s4 * 4;
                const bool hb = hf * 8 + s4 + 1 < nstripes;
                if (!__any(nibw(m.mem, sh) | (hb ? nibw(m.mem, sh + 4) : 0u))) continue;
                uint32_t a0, a1, a2, ca, b0 = 0, b1 = 0, b2 = 0, cb = 0;
                cup_stripe(m, sh, lut, a0, a1, a2, ca);
                if (hb) cup_stripe(m, sh + 4, lut, b0, b1, b2, cb);
                ring_put2<4>(g, a0, a1, a2, ca, b0, b1, b2, cb);
                ring_step(g, lane);
            }
        }
    }
    const int n_cup = g.pos - cup0;
    ring_pass_end(g, lane);
    // SPP distortion decrease: the newly significant samples N have top bit
    // p, each gains 2^p (12 v + 6d - 9 2^p) (d = 1 lossy, 0 lossless; 4 at
    // lossless p = 0), and sum_N v = 2^p |N| + sum_{q<p} 2^q |N & B[q]|
    // from the column masks of the lower planes (dist_gain, exact)
    // (a plane whose SPP makes nothing significant skips the sums: 0)
    int64_t dspp = 0;
    if (spp && __any(N != 0ull)) {
        const uint32_t nl = (uint32_t)__popcll(N);
        int64_t sv = (int64_t)nl << p;
        // (N is 0 on lanes past the block width: no lane test, so the
        // unrolled loads issue together)
#pragma unroll 4
        for (int q = 0; q < p; q++) sv += (int64_t)__popcll(N & CT[(size_t)q * 64 + lane]) << q;
        const int64_t nN = (int64_t)wave_sum_u32(nl);  // <= 4096
        sv = wave_sum64(sv);
        dspp = (lossless && p == 0) ? 4 * nN
                                    : ((12 * sv + (6 * (lossless ? 0 : 1) - 9 * ((int64_t)1 << p)) * nN) << p);
    }
    if (lane == 0) {
        uint4 cnt;
        cnt.x = (uint32_t)n_spp;
        cnt.y = (uint32_t)n_mrp;
        cnt.z = (uint32_t)n_cup;
        cnt.w = 0;
        a.counts[(size_t)b * 32 + k] = cnt;
        a.dspp[(size_t)b * 32 + k] = dspp;
    }
    return (uint32_t)(n_spp + n_mrp + n_cup);
}

// Compaction selectors of the stripe step: entry K = members (bits 0-3) |
// members with a 1 bit (bits 4-7); output byte order q = 0..3: zc byte q
// (selector q), then its sign byte (selector 4 + q); unused bytes select 0x00
// (0x0C).  (Byte n of the 64-bit pair set by shifts: no private array.)
__device__ __forceinline__ uint2 cm_selectors(int K) {
    uint64_t sel = 0x0C0C0C0C0C0C0C0Cull;
    int n = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int bit = (q & 1) ? 4 + (q >> 1) : (q >> 1);  // zc q/2, then its sign
        if ((K >> bit) & 1) {
            sel = (sel & ~(0xFFull << (8 * n))) | ((uint64_t)((q & 1) ? 4 + (q >> 1) : (q >> 1)) << (8 * n));
            n++;
        }
    }
    return make_uint2((uint32_t)sel, (uint32_t)(sel >> 32));
}

// A block's descriptor fields k_t1_cm3 uses (wave-uniform), and its first
// masks (the sign column and B of the top plane).
struct CmBlk {
    int b, P, c, w, h, Mb, band;
    uint64_t bp_off, slot;
};
__device__ __forceinline__ CmBlk cm_blk_load(const T1CmArgs &a, int b) {
    const BlockDesc d = a.blocks[b];
    CmBlk k;
    k.b = b;
    k.P = a.P[b];
    k.c = (int)(a.acc[b] >> 40);  // coded planes (emit_t1_items)
    k.w = d.w;
    k.h = d.h;
    k.Mb = d.Mb;
    k.band = d.band;
    k.bp_off = d.bp_off;
    k.slot = a.slot_off[b];
    return k;
}
struct CmMasks {
    uint64_t SG, B;
};
__device__ __forceinline__ CmMasks cm_masks_load(const T1CmArgs &a, const CmBlk &k, int lane) {
    const uint64_t *CT = a.bp + k.bp_off;
    CmMasks m;
    m.SG = CT[(size_t)k.Mb * 64 + lane];
    m.B = CT[(size_t)(k.P - 1) * 64 + lane];
    return m;
}

// k_t1_cm3, one wave per code-block: the block's coded planes top-down, in
// order, so a plane's S[p+1] and S[p+2] are the masks the wave already holds
// and the next plane's two masks load while this one is coded (one dependent
// descriptor chain per block instead of per plane); the block's decision
// total is known at its end, where it is filed in its MQ lane-order bucket.
// Blocks are taken from the depth-0 work list (every block with a coded
// plane) in a grid-stride loop.
#ifdef JP2HIP_CM_WAVES_PER_EU
__global__ void __launch_bounds__(64 * kCmWaves) __attribute__((amdgpu_waves_per_eu(JP2HIP_CM_WAVES_PER_EU))) k_t1_cm3(T1CmArgs a) {
#else
__global__ void __launch_bounds__(64 * kCmWaves) k_t1_cm3(T1CmArgs a) {
#endif
    __shared__ uint2 lut[256];
    __shared__ uint32_t rings[kCmWaves][kRingWords];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int K = threadIdx.x; K < 256; K += 64 * kCmWaves) lut[K] = cm_selectors(K);
    for (int i = threadIdx.x; i < kCmWaves * kRingWords; i += 64 * kCmWaves) (&rings[0][0])[i] = 0u;
    __syncthreads();
    const int nblk = a.kmax > 0 ? (int)a.dfill[0] : 0;
    Ring g;
    g.r = rings[wv];
    const int stride = gridDim.x * kCmWaves;
    int bi = blockIdx.x * kCmWaves + wv;
    if (bi >= nblk) return;  // (no barrier follows)
    // Blocks are pipelined one ahead: during block i the wave loads block
    // i+1's descriptor (while block i's first plane is coded) and then its
    // first masks (at block i's end), and the work-list index of block i+2,
    // so a block starts with nothing to wait for -- the four dependent loads
    // (work list -> descriptor -> masks) of a block no longer sit between
    // two blocks.
    CmBlk cur = cm_blk_load(a, a.dlist[bi]);
    CmMasks mk = cm_masks_load(a, cur, lane);
    int idx_next = bi + stride < nblk ? a.dlist[bi + stride] : -1;
    for (;;) {
        const int b = cur.b, P = cur.P, c = cur.c, w = cur.w, h = cur.h, band = cur.band;
        const bool vl = lane < w;
        const uint64_t *CT = a.bp + cur.bp_off;
        uint64_t Bl = mk.B;
        const uint64_t SG = vl ? mk.SG : 0ull;
        const uint64_t LSG = col_left(SG, lane), RSG = col_right(SG, lane);
        uint64_t S1 = 0, S2 = 0;
        uint32_t tot = 0;
        const uint32_t cap = plane_stream_cap(w, h);
        uint8_t *out = a.stream + cur.slot;
        CmBlk nxt;
        int idx_after = -1;
        for (int k = 0; k < c; k++) {
            const int p = P - 1 - k;
            // S[p] = S[p+1] | B[p] (planes above the top one are empty)
            const uint64_t B = vl ? Bl : 0ull, S0 = S1 | B;
            if (k + 1 < c) Bl = CT[(size_t)(p - 1) * 64 + lane];  // the next plane's mask, in flight during this one
            if (k == 0 && idx_next >= 0) {  // the next block's descriptor, and the index after it
                nxt = cm_blk_load(a, idx_next);
                if (bi + 2 * stride < nblk) idx_after = a.dlist[bi + 2 * stride];
            }
            g.out = out + (size_t)k * cap;
            g.pos = 0;
            g.fl = 0;
            tot += cm_plane(a, g, lut, lane, b, k, p, P, w, h, band, CT, B, S0, S1, S2, SG, LSG, RSG);
#ifdef JP2HIP_BURN_VALU  // resource experiments only: N dependent VALU per plane
            {
                uint32_t x = (uint32_t)B ^ (uint32_t)lane;
                for (int i = 0; i < JP2HIP_BURN_VALU; i++) x = (x ^ (uint32_t)i) + (x << 3);
                if (x == 0x9E3779B9u) a.counts[(size_t)b * 32 + k].w = x;
            }
#endif
#ifdef JP2HIP_BURN_SLEEP  // ... or a wave that idles N x 64 cycles per plane
            __builtin_amdgcn_s_sleep(JP2HIP_BURN_SLEEP);
#endif
            S2 = S1;
            S1 = S0;
        }
        const bool more = idx_next >= 0;
        if (more) mk = cm_masks_load(a, nxt, lane);  // the next block's first masks
        if (lane == 0) {
            a.acc[b] = tot;  // decisions (k_hull's tier-1 totals); no planes left
            const int bk = order_bucket(tot);
            a.bslots[(size_t)bk * a.nb + atomicAdd(&a.bfill[bk], 1u)] = b;
        }
        if (!more) break;
        bi += stride;
        cur = nxt;
        idx_next = idx_after;
    }
}

// --------------------------------------------------------------------------
// MQ coder
// --------------------------------------------------------------------------
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

// The coder's byte ring: 64 bytes per lane, lane L's at LDS byte 64 L, byte
// position bp (offset by 4 L, which spreads the lanes over the banks) at
// slot bp & 63 -- one bit-field insert per address.  (Measured before:
// rings at a 68-byte stride, and interleaved by lane -- dword k of lane L at
// dword 64 k + L, no conflicts but more address arithmetic: k_t1_mq alone
// 2894 -> 2905 us, C2 bench 24.9 -> 24.3 GP/s, gpurun_out/r4a/ab_ring.)
__device__ __forceinline__ uint32_t ring_at(int bp, uint32_t lb) {  // lb = 64 L
    uint32_t r;  // (bp & 63) | lb as one bit-field insert (the compiler adds after an AND)
    asm("v_bfi_b32 %0, 63, %1, %2" : "=v"(r) : "v"(bp), "v"(lb));
    return r;
}

__device__ __forceinline__ void ring_byteout(Mq &m, uint8_t *ring, uint32_t lb) {
    uint32_t B = m.B;
    if (B != 0xFF && m.C >= 0x8000000u) {
        B++;
        m.C &= 0x7FFFFFFu;
    }
    ring[ring_at(m.bp, lb)] = (uint8_t)B;  // bp = -1 -> the ring's last slot, see mq_code
    m.bp++;
    const bool ff = B == 0xFF;
    m.B = ff ? (m.C >> 20) : (m.C >> 19);
    m.C &= ff ? 0xFFFFFu : 0x7FFFFu;
    m.CT = ff ? 7 : 8;
}

// --------------------------------------------------------------------------
// k_t1_mq: two waves per 64 code-blocks, a software pipeline over the MQ
// coder's two dependency chains (Annex C.2):
//   wave 0 (modeller) walks the blocks' decision streams with the context
//     states and the interval register A: per decision it knows whether C
//     gains Qe and how many bits the renormalisation shifts -- the code
//     register's whole input -- and leaves (add << 16 | shifts) in an LDS slot;
//   wave 1 (coder) runs C, CT and the byte-outs over those words.
// Chunks of 16 decisions per lane, double-buffered, one workgroup barrier per
// chunk: the modeller writes chunk i + 1 while the coder codes chunk i, so a
// decision costs the longer of the two chains, not their sum.
//
// Context state = the 32-bit word of its (table index i, MPS symbol) pair,
// entry e = 2 i + MPS: Qe << 16 | 8 e | MPS.  Entry e's 8 bytes in the LDS
// table are the words of its NMPS and NLPS entries (the NLPS one with a
// SWITCH state's MPS flip applied), so the state word is also the address of
// both candidate next states: they are read (one 8-byte LDS read) as soon as
// the state is known, while the decision's arithmetic runs, and a select
// picks one.  The interval register A is kept scaled by 2^16 (the Qe field
// needs no shift, and the renormalisation count is its leading zeros).
//
// The CODEMPS/CODELPS procedures fold into one select -- the interval keeps
// A - Qe exactly when "MPS" xor "conditional exchange" -- and the context
// moves to NMPS / NLPS exactly when renormalisation happens.  Pass padding
// (CX_PAD, state 0) makes a step with Qe = 0 and d = MPS: no interval change,
// no shift, no byte -- so every step is coded, and lanes whose block is done
// code padding.
// --------------------------------------------------------------------------
constexpr int kMqChunk = 16;
// Census experiments (debug builds, tests/tools/mq_census.py; output not
// valid): 2 = the modeller alone (no coder wave, no chunk barrier); 3 = as 2
// and the next-state table read replaced by register values (what the LDS
// round trip costs the modeller)
#ifndef JP2HIP_MQ_EXP
#define JP2HIP_MQ_EXP 0
#endif
constexpr uint32_t kPadWord = 0x01010101u * kPadDecision;
// The modeller's interval register and the state words' Qe field are scaled
// by 2^16.  (Measured and dropped: scaled by 2^15, so that "A - Qe < Qe" and
// "A < 0x8000" are sign bits of 32-bit differences and every select is a
// bit-field select on VGPR masks, no compare -> VCC -> v_cndmask hop: 255
// instead of 251 cycles per decision, MQ +3 %, C2 bench -3 %:
// profiles/r05/ab_mq_masks.txt.)
constexpr int kQeShift = 16;
#ifndef JP2HIP_MQ_SCHED
#define JP2HIP_MQ_SCHED 1
#endif
#ifndef JP2HIP_MQ_PASS_PREFETCH
#define JP2HIP_MQ_PASS_PREFETCH 1
#endif


// the state word of entry e (Qe << kQeShift | 8 e | MPS)
__device__ __forceinline__ uint32_t mq_word(int e) {
    return ((uint32_t)c_qe[e >> 1] << kQeShift) | ((uint32_t)e << 3) | (uint32_t)(e & 1);
}

// modeller: one decision; returns the context's next state and stores the
// coder's input word (C's addend << 16 | renormalisation shifts) to *code.
// A = the interval register << 16.
__device__ __forceinline__ uint32_t mq_model(uint32_t &A, const uint32_t t, const uint8_t *tab, const uint32_t d,
                                             uint32_t *code) {
#if JP2HIP_MQ_EXP == 3
    const uint2 nx = make_uint2(t ^ 0x10008u, t ^ 0x20010u);
#else
    const uint2 nx = *(const uint2 *)(tab + (t & 0x3F8u));  // NMPS / NLPS words, read first
#endif
    const uint32_t qe = t & 0xFFFF0000u;  // Qe << 16
    const bool isM = d == (t & 1u);
    const uint32_t A1 = A - qe;
    const bool keep = isM != (A1 < qe);
    const uint32_t An = keep ? A1 : qe;  // never 0: Qe >= 1, and A1 = A >= 2^31 for Qe = 0
    const bool ren = !isM || A1 < 0x80000000u;
    const uint32_t n = (uint32_t)__builtin_clz(An);  // renormalisation shifts
    A = An << n;
    const uint32_t cw = (keep ? qe : 0u) | n;
#if JP2HIP_MQ_SCHED
    // the interval register's chain (and what the caller computed before the
    // call) is issued in full before the wait for the table read: it runs
    // under the read's latency instead of after it (the wave issues in
    // order, and the first use of nx waits for LDS).  Census 250 -> 237
    // cycles per decision, k_t1_mq alone 2.48 -> 2.36 ms on C2
    // (profiles/r05/mq/ab_sched.txt; the code word stored ahead of the wait
    // as well: 239; the next table read issued ahead of the next decision's
    // stream bookkeeping: 245)
    __builtin_amdgcn_sched_barrier(0);
#endif
    *code = cw;
    return ren ? (isM ? nx.x : nx.y) : t;
}

// coder: C += add, then n shifts with their byte-outs.  The (at most one,
// common) byte-out is applied by select and its byte written to the lane's
// 64-byte LDS ring on every step -- so the only branch is the rare second
// byte-out of one renormalisation.
// TWO = false: no decision of the chunk shifts 8 or more (a second byte-out
// in one renormalisation needs n >= CT + 7 >= 8), so its test is left out.
template <bool TWO>
__device__ __forceinline__ void mq_code(Mq &m, const uint32_t code, uint8_t *ring, uint32_t lb) {
    const uint32_t add = code >> kQeShift;
    const int n = (int)(code & 0x1Fu);
    const uint32_t C0 = m.C + add;
    const int CT = m.CT;
    const bool bo = n >= CT;  // a byte-out inside this renormalisation
    const int s1 = min(n, CT);
    const uint32_t C1 = C0 << s1;
    const bool carry = (m.B != 0xFFu) && (C1 >= 0x8000000u);
    const uint32_t Bc = m.B + (carry ? 1u : 0u);
    const uint32_t C2 = carry ? (C1 & 0x7FFFFFFu) : C1;
    const bool ff = Bc == 0xFFu;
    const uint32_t sh = ff ? 20u : 19u;
    // the byte goes to slot bp whether or not it is emitted: without a
    // byte-out the slot is the next byte's, written again when it is emitted
    // and never flushed before (ring_flush copies whole groups below bp).
    // Byte -1 (the MQ coder's initial pending byte, never output) lands in
    // the ring's last slot, which the byte of that slot overwrites before
    // its group is flushed
    ring[ring_at(m.bp, lb)] = (uint8_t)Bc;
    uint32_t Cx = bo ? (C2 & ((1u << sh) - 1u)) : C1;
    int CTx = bo ? 27 - (int)sh : CT - n;
    int rem = n - s1;
    m.B = bo ? (C2 >> sh) : m.B;
    m.bp += bo ? 1 : 0;
    if (TWO && bo && rem >= CTx) {  // rare: a second byte-out in this renormalisation
        m.C = Cx << CTx;
        rem -= CTx;
        ring_byteout(m, ring, lb);
        Cx = m.C;
        CTx = m.CT;
    }
    m.C = Cx << rem;
    m.CT = CTx - rem;
}

// Copy the lane's completed 16-byte groups to the code-block output (byte
// positions run `off` = 4 L ahead of the output's, so a group's dwords may
// wrap round the lane's ring).
__device__ __forceinline__ void ring_flush(const Mq &m, const uint8_t *ring, uint32_t lb, int off, int &fl) {
    while (m.bp - fl >= 16) {
        uint4 v;
        v.x = *(const uint32_t *)(ring + ring_at(fl, lb));
        v.y = *(const uint32_t *)(ring + ring_at(fl + 4, lb));
        v.z = *(const uint32_t *)(ring + ring_at(fl + 8, lb));
        v.w = *(const uint32_t *)(ring + ring_at(fl + 12, lb));
        if (fl - off + 16 <= m.cap) *(uint4 *)(m.out + (fl - off)) = v;
        fl += 16;
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

// LDS of one k_t1_mq workgroup
struct MqShared {
    uint2 mqt[94];                         // per entry: its NMPS and NLPS state words
    uint32_t cxs[20 * 64];                 // 19 contexts + CX_PAD, lane-interleaved (modeller)
    uint32_t rings[64 * 16];               // coder: a 64-byte byte ring per lane
    // (the bucket bases are done with before the first chunk: one LDS slot,
    // 19.1 KB a workgroup, 8 per CU instead of 7)
    union {
        uint32_t bbase[kOrderBuckets + 1];  // lane order: bucket bases
        uint32_t code[2][kMqChunk][64];     // modeller -> coder, double-buffered
    };
    int32_t segs[2][64];                   // passes closed before the chunk (per lane)
    uint32_t finA[64];                     // the interval register at the end (mq_flush)
    int32_t blk[64];                       // the lane's block, -1 none
    int32_t more[2];                       // chunk present
#ifdef JP2HIP_MQ_LDS_PAD  // residency experiments only: bytes of unused LDS per workgroup
    uint8_t pad_[JP2HIP_MQ_LDS_PAD];
#endif
};

// Modeller (wave 0).  One lane per block walks the block's passes -- segments
// of the decision streams, each 16-byte aligned (k_t1_cm3) -- with ONE
// data-driven loop of 16-decision chunks; the segment switch and the per-pass
// distortion record are data, not control flow.  Segment s of a block with P
// coded planes: s = 0 is the top plane's cleanup pass; s >= 1 is pass
// (s+2)%3 (0 SPP, 1 MRP, 2 CUP) of plane k = (s+2)/3, planes counted from the
// top.  Blocks are ordered by decision count (the buckets k_t1_cm3 files
// them in), so the lanes of a wave finish together.
__device__ __forceinline__ void mq_modeller(const T1MqArgs &a, MqShared &sh) {
    const int lane = threadIdx.x & 63;
    const int b = sh.blk[lane];
    uint32_t *cx = sh.cxs + lane;
    const uint8_t *mqt = (const uint8_t *)sh.mqt;
    const uint32_t w0 = mq_word(0);
#pragma unroll
    for (int q = 0; q < 19; q++) cx[q * 64] = w0;  // entry 2 i + MPS; all start with MPS 0
    cx[CX_PAD * 64] = 0u;  // Qe 0, MPS 0: the padding decisions' no-op state
    cx[0] = mq_word(2 * 4);
    cx[CX_RL * 64] = mq_word(2 * 3);
    cx[CX_UNI * 64] = mq_word(2 * 46);
    uint32_t A = 0x8000u << kQeShift;
    int nseg = 0, s = 0, k = 0, pass = 2, left = 0, Pt = 0;
    uint32_t cap = 0;
    const uint8_t *sbase = nullptr;
    const uint4 *cntp = nullptr, *ptr = nullptr;
    const int64_t *dspp = nullptr, *dref = nullptr, *dsig = nullptr;
    int64_t *D = nullptr;
    const uint4 pad4 = make_uint4(kPadWord, kPadWord, kPadWord, kPadWord);
    // the decision stream is read two chunks ahead: cur = this chunk, nx1 =
    // the next (loaded iff the pass has more than 16 decisions left), and a
    // chunk issues the load of the one after nx1 -- a 16-byte load's latency
    // is about one chunk's 16 decisions
    uint4 cnt = make_uint4(0u, 0u, 0u, 0u), cur = pad4, nx1 = pad4;
    int64_t ndec = 0;
#if JP2HIP_MQ_PASS_PREFETCH
    // The pass after the current one, loaded as soon as the current one
    // starts (its plane's counts when it opens a plane, its first two
    // chunks): a pass switch then takes registers instead of a dependent
    // counts -> stream load while the whole wave waits -- in a wave of 64
    // blocks some lane switches passes in most chunks
    int pf_pass = 0, pf_k = 0, pf_valid = 0;
    uint4 pf_cnt = cnt, pf_cur = pad4, pf_nx1 = pad4;
    const uint4 *pf_ptr = nullptr;
    auto prefetch = [&]() {
        pf_valid = 0;
        if (s + 1 >= nseg) return;
        const int np = pass == 2 ? 0 : pass + 1, nk = pass == 2 ? k + 1 : k;
        // (compiled as a flat load from a selected address -- `cnt` gets a
        // 16-byte scratch slot -- which leaves the next chunks' stream loads
        // in flight at the chunk start; a global load of plane nk's counts,
        // selected or not, made that wait vmcnt(0): census 221 -> 243-255
        // cycles per decision, profiles/r05/mq/ab_pass_counts.txt)
        const uint4 nc = np == 0 ? cntp[nk] : cnt;
        const int o_mrp = ((int)cnt.x + 15) & ~15;
        const int o_cup = (o_mrp + (int)cnt.y + 15) & ~15;
        pf_ptr = (const uint4 *)(sbase + (size_t)nk * cap + (np == 0 ? 0 : (np == 1 ? o_mrp : o_cup)));
        pf_cur = pf_ptr[0];
        pf_nx1 = pf_ptr[1];  // (inside the slot: a pass is padded, a plane's slot has 128 bytes to spare)
        pf_pass = np;
        pf_k = nk;
        pf_cnt = nc;
        pf_valid = 1;
    };
#endif
    if (b >= 0) {
        const BlockDesc d = a.blocks[b];
        Pt = a.P[b];
        const int P = Pt - a.pmin[b];  // coded planes Pt-1 .. pmin (slope prediction)
        nseg = 3 * P - 2;
        D = a.dists + (size_t)b * kMaxPasses;
        cap = plane_stream_cap(d.w, d.h);
        sbase = a.stream + a.slot_off[b];
        cntp = a.counts + (size_t)b * 32;
        dspp = a.dspp + (size_t)b * 32;
        dref = a.dref + (size_t)b * 32;
        dsig = a.dsig + (size_t)b * 32;
        cnt = cntp[0];
        ptr = (const uint4 *)sbase;  // top plane: cleanup at offset 0
        left = (int)cnt.z;
        ndec = left;
        cur = ptr[0];
        if (left > 16) nx1 = ptr[1];
#if JP2HIP_MQ_PASS_PREFETCH
        prefetch();
#endif
    }
    uint64_t cyc_wait = 0;  // debug census: shader cycles spent at the chunk barrier
    const uint64_t cyc0 = __builtin_readcyclecounter();
    for (int it = 0;; it++) {
        // close finished passes (empty passes close at once)
        while (left <= 0 && s < nseg) {
#if JP2HIP_MQ_PASS_PREFETCH
            // (the pass's distortion record is written after the block)
            if (++s >= nseg) break;
            pass = pf_pass;
            k = pf_k;
            cnt = pf_cnt;
            ptr = pf_ptr;
            cur = pf_cur;
            nx1 = pf_nx1;  // (whatever it holds when the pass has <= 16 decisions: never coded)
            left = pass == 0 ? (int)cnt.x : (pass == 1 ? (int)cnt.y : (int)cnt.z);
            ndec += left;
            prefetch();
#else
            const int p = Pt - 1 - k;
            D[s] = pass == 0 ? dspp[k] : (pass == 1 ? dref[p] : dsig[p] - dspp[k]);
            if (++s >= nseg) break;
            pass = pass == 2 ? 0 : pass + 1;
            if (pass == 0) {
                k++;
                cnt = cntp[k];
            }
            const int o_mrp = ((int)cnt.x + 15) & ~15;
            const int o_cup = (o_mrp + (int)cnt.y + 15) & ~15;
            ptr = (const uint4 *)(sbase + (size_t)k * cap + (pass == 0 ? 0 : (pass == 1 ? o_mrp : o_cup)));
            left = pass == 0 ? (int)cnt.x : (pass == 1 ? (int)cnt.y : (int)cnt.z);
            ndec += left;
            cur = ptr[0];
            nx1 = left > 16 ? ptr[1] : pad4;
#endif
        }
        const bool active = s < nseg;
        const int buf = it & 1;
        sh.segs[buf][lane] = s;
        if (!__any(active)) {
            sh.finA[lane] = A >> kQeShift;
            if (lane == 0) sh.more[buf] = 0;
#if JP2HIP_MQ_EXP < 2
            __syncthreads();
#endif
            break;
        }
        if (lane == 0) sh.more[buf] = 1;
        // one chunk of 16 decisions (a pass's last chunk is padded; a lane
        // whose block is done codes padding); the loads of the next two
        // chunks are in flight behind it, and each context state is read one
        // decision ahead
        uint4 nx2 = pad4;
        if (active && left > 32) nx2 = ptr[2];
        if (!active) cur = pad4;
        const uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
        uint32_t t = cx[__builtin_amdgcn_ubfe(w[0], 1, 5) * 64];
        uint32_t *out = &sh.code[buf][0][lane];
#pragma unroll
        for (int j = 0; j < kMqChunk; j++) {
            // decision byte = (context << 1) | d; context in bits 1..5
            const uint32_t cur_cx = __builtin_amdgcn_ubfe(w[j >> 2], (j & 3) * 8 + 1, 5);
            const uint32_t dd = __builtin_amdgcn_ubfe(w[j >> 2], (j & 3) * 8, 1);
            uint32_t nxt_cx = 0, nt = 0;
            if (j < kMqChunk - 1) {
                nxt_cx = __builtin_amdgcn_ubfe(w[(j + 1) >> 2], ((j + 1) & 3) * 8 + 1, 5);
                nt = cx[nxt_cx * 64];
            }
            const bool same = nxt_cx == cur_cx;  // (before the call: ahead of the table wait)
            const uint32_t tn = mq_model(A, t, mqt, dd, &out[j * 64]);
            cx[cur_cx * 64] = tn;
            t = same ? tn : nt;
        }
        if (active) {
            left -= min(16, left);
            ptr++;
            cur = nx1;
            nx1 = nx2;
        }
        const uint64_t c1 = a.dbg ? __builtin_readcyclecounter() : 0;
#if JP2HIP_MQ_EXP >= 2
        __builtin_amdgcn_wave_barrier();
#else
        __syncthreads();  // chunk `it` ready; the coder is done with chunk it - 1
#endif
        if (a.dbg) cyc_wait += __builtin_readcyclecounter() - c1;
    }
#if JP2HIP_MQ_PASS_PREFETCH
    // the passes' distortion records (segment s: s = 0 the top plane's
    // cleanup, else pass (s+2)%3 of plane (s+2)/3 from the top)
    for (int q = 0; q < nseg; q++) {
        const int kq = q == 0 ? 0 : (q + 2) / 3, pq = q == 0 ? 2 : (q + 2) % 3, p = Pt - 1 - kq;
        D[q] = pq == 0 ? dspp[kq] : (pq == 1 ? dref[p] : dsig[p] - dspp[kq]);
    }
#endif
#if JP2HIP_MQ_EXP >= 2
    if (b >= 0) {  // no coder ran: the block codes as empty downstream
        a.npasses[b] = 0;
        a.lengths[b] = 0;
    }
#endif
    if (a.dbg && b >= 0) {  // debug census: decisions, modeller cycles, of which at the barrier
        a.dbg[(size_t)b * 6 + 0] = ndec;
        a.dbg[(size_t)b * 6 + 1] = (int64_t)(__builtin_readcyclecounter() - cyc0);
        a.dbg[(size_t)b * 6 + 2] = (int64_t)cyc_wait;
    }
}

// Coder (wave 1): C, CT, B and the output bytes of the same 64 blocks.
__device__ __forceinline__ void mq_coder(const T1MqArgs &a, MqShared &sh) {
    const int lane = threadIdx.x & 63;
    const int b = sh.blk[lane];
    uint8_t *ring = (uint8_t *)sh.rings;
    const uint32_t lb = (uint32_t)lane << 6;  // the lane's ring
    const int off = 4 * lane;                 // byte positions run off ahead (ring_at)
    int fl = off;                             // bytes already copied from the ring
    Mq m;
    m.C = 0; m.A = 0x8000; m.B = 0; m.CT = 12; m.bp = off - 1;
    m.cap = 0;
    m.out = nullptr;
    int32_t *R = nullptr;
    if (b >= 0) {
        const BlockDesc d = a.blocks[b];
        m.cap = (int)d.out_cap;
        m.out = a.out + d.out_off;
        R = a.rates + (size_t)b * kMaxPasses;
    }
    int sdone = 0;
    uint64_t cyc_wait = 0;  // debug census (as the modeller's)
    const uint64_t cyc0 = __builtin_readcyclecounter();
    for (int it = 0;; it++) {
        const uint64_t c1 = a.dbg ? __builtin_readcyclecounter() : 0;
        __syncthreads();  // chunk `it` written by the modeller
        if (a.dbg) cyc_wait += __builtin_readcyclecounter() - c1;
        const int buf = it & 1;
        // passes that ended before this chunk end at the current length
        const int s_now = sh.segs[buf][lane];
        for (; sdone < s_now; sdone++) R[sdone] = m.bp - off + 3;
        if (!sh.more[buf]) break;
        // the chunk's 16 words read up front (one wait, not one per decision)
        const uint32_t *in = &sh.code[buf][0][lane];
        uint32_t cw[kMqChunk];
#pragma unroll
        for (int j = 0; j < kMqChunk; j++) cw[j] = in[j * 64];
        // a chunk whose shifts are all < 8 (about 9 in 10 on C2) takes the
        // coder without the second-byte-out branch (bit 3 of the shift field)
        const uint32_t any8 = (cw[0] | cw[1] | cw[2] | cw[3] | cw[4] | cw[5] | cw[6] | cw[7] | cw[8] | cw[9] |
                               cw[10] | cw[11] | cw[12] | cw[13] | cw[14] | cw[15]) & 8u;
        if (__any(any8 != 0u)) {
#pragma unroll
            for (int j = 0; j < kMqChunk; j++) mq_code<true>(m, cw[j], ring, lb);
        } else {
#pragma unroll
            for (int j = 0; j < kMqChunk; j++) mq_code<false>(m, cw[j], ring, lb);
        }
        ring_flush(m, ring, lb, off, fl);
    }
    if (b < 0) return;
    const int nseg = sdone;
    m.A = sh.finA[lane];
    for (int i = fl; i < m.bp; i++)  // bytes still in the ring
        if (i - off < m.cap) m.out[i - off] = ring[ring_at(i, lb)];
    m.bp -= off;
    const int len = mq_flush(m);
    if (len > m.cap) atomicOr(a.err, 1);
    R[nseg - 1] = len;
    for (int i = 0; i < nseg; i++) {
        int r = min(R[i], len);
        if (r > 1 && r <= m.cap && m.out[r - 1] == 0xFF) r--;
        R[i] = r;
    }
    a.npasses[b] = (uint8_t)nseg;
    a.lengths[b] = len;
    if (a.dbg) {  // coder cycles, of which at the barrier; lane-order position
        a.dbg[(size_t)b * 6 + 3] = (int64_t)(__builtin_readcyclecounter() - cyc0);
        a.dbg[(size_t)b * 6 + 4] = (int64_t)cyc_wait;
        a.dbg[(size_t)b * 6 + 5] = blockIdx.x * 64 + lane;
    }
}

// The launch's execution span is recorded in 100 MHz wall-clock ticks
// (span[0] = ~earliest wave start, span[1] = latest lane end; vector atomics
// on words k_quant zeroed).
__global__ void __launch_bounds__(128) k_t1_mq(T1MqArgs a) {
    __shared__ MqShared sh;
    const int tid = threadIdx.x, lane = tid & 63;
#ifdef JP2HIP_MQ_PRIO
    // issue priority over the other kernels' waves on the SIMD: the MQ
    // chains are latency-bound and hold their LDS until they end
    __builtin_amdgcn_s_setprio(JP2HIP_MQ_PRIO);
#endif
    const uint64_t w0 = wall_clock64();
    if (tid == 0) atomicMax(&a.span[0], ~(unsigned long long)w0);
    for (int e = tid; e < 94; e += 128) {
        const int i = e >> 1, mps = e & 1;
        const int sw = i == 0 || i == 6 || i == 14;
        sh.mqt[e] = make_uint2(mq_word(2 * c_nmps[i] + mps), mq_word(2 * c_nlps[i] + (mps ^ sw)));
    }
    if (tid < 64) {  // exclusive scan of the bucket fills, kOrderBuckets / 64 per lane
        uint32_t v[kOrderBuckets / 64], t = 0;
#pragma unroll
        for (int i = 0; i < kOrderBuckets / 64; i++) t += (v[i] = a.bfill[kOrderBuckets / 64 * lane + i]);
        uint32_t o = wave_incl_scan(t) - t;
#pragma unroll
        for (int i = 0; i < kOrderBuckets / 64; i++) {
            sh.bbase[kOrderBuckets / 64 * lane + i] = o;
            o += v[i];
        }
        if (lane == 63) sh.bbase[kOrderBuckets] = o;
    }
    __syncthreads();
    if (tid < 64) {
        // lane-order position gi -> its bucket -> the block (blocks with no
        // coded plane are in no bucket: emit_t1_items recorded them)
        const int gi = blockIdx.x * 64 + lane;
        int b = -1;
        if (gi < (int)sh.bbase[kOrderBuckets]) {
            int bk = 0;
            for (int step = kOrderBuckets / 2; step > 0; step >>= 1)
                if (sh.bbase[bk + step] <= (uint32_t)gi) bk += step;
            b = a.bslots[(size_t)bk * a.nblocks + (gi - (int)sh.bbase[bk])];
        }
        sh.blk[lane] = b;
    }
    __syncthreads();
    if (tid < 64) mq_modeller(a, sh);
#if JP2HIP_MQ_EXP < 2
    else mq_coder(a, sh);
#endif
    if (tid == 64) atomicMax(&a.span[1], (unsigned long long)wall_clock64());
}

void launch_t1_cm(const T1CmArgs &a, hipStream_t st) {
    if (!a.max_items) return;
    const dim3 g((a.nb + kCmWaves - 1) / kCmWaves);  // a wave per block at most
    hipLaunchKernelGGL(k_t1_cm3, dim3(std::min<int>((int)g.x, kCm3Blocks)), dim3(64 * kCmWaves), 0, st, a);
}
void launch_t1_mq(const T1MqArgs &a, hipStream_t st) {
    if (a.nblocks) hipLaunchKernelGGL(k_t1_mq, dim3((a.nblocks + 63) / 64), dim3(128), 0, st, a);
}
// no slope prediction: every plane coded (pmin = 0), the work lists filled
__global__ void __launch_bounds__(256) k_t1_items(T1ItemArgs a) {
    __shared__ ItemScratch sc;
    const int b = blockIdx.x * 256 + threadIdx.x;
    const bool in = b < a.nb;
    const int P = in ? a.P[b] : 0;
    if (in) a.pmin[b] = 0;
    emit_t1_items<256>(a, b, in, P, 0, sc);
}
void launch_t1_items(const T1ItemArgs &a, hipStream_t st) {
    if (a.nb > 0) hipLaunchKernelGGL(k_t1_items, dim3((a.nb + 255) / 256), dim3(256), 0, st, a);
}
uint32_t t1_plane_stream_cap(int w, int h) { return plane_stream_cap(w, h); }

}  // namespace jp2hip
