// t2_device.hip -- tier-2 on the GPU (ISO/IEC 15444-1 Annex B.9-B.10, A.4, A.7.3):
// packet headers, tile-part sizes and the code-stream itself, written in HBM.
//
// Structure produced for the Bucketeer recipe (KakaduConverter.java:38-44):
// RPCL packets, SOP before and EPH after every packet header, one tile-part
// per resolution (ORGtparts=R) with a PLT marker (ORGgen_plt=yes), tile-parts
// in -flush_period stripe order (t2_tables, test.jpx).  The byte layout is
// the oracle's (oracle/jp2_oracle.c encode_packet / write_codestream).
//
// Parallel structure.  A precinct's L packets share state (tag trees, each
// block's Lblock and inclusion layer); precincts are independent (C2: 2 880
// per image, C5: 51 153).  A wave codes a precinct, a lane per code-block,
// with the tag trees in closed form (k_t2_wave); precincts of more than 64
// blocks take the serial coder, a lane per precinct (k_t2_code + k_apply).
// Sizing and emission run the same coder (template EMIT):
//   k_t2_wave<false>  layer assignment, header bytes + packet lengths  (every rate pass)
//   k_t2_total        tile-part sizes, stream offsets, sums for the host (every rate pass)
//   k_t2_tp_emit      SOT + PLT + SOD, packet offsets                  (final pass)
//   k_t2_wave<true>   SOP + header + EPH, body offsets                 (final pass)
//   k_t2_copy         code-block bytes into the bodies                 (final pass)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "device_common.h"
#include "gpu_encoder.h"
#include "host_wait.h"

namespace jp2hip {

#define HIPCHECK(x)                                                                    \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            err = std::string(#x) + ": " + hipGetErrorString(e_);                      \
            return false;                                                              \
        }                                                                              \
    } while (0)

struct T2Args {
    const PrecDesc *prec;
    int nprec;
    const TpDesc *tps;
    int ntp;
    const BlockDesc *blocks;
    const uint8_t *P;       // coded planes per block
    uint8_t *nl;            // [block][L] cumulative passes (written by k_t2_wave<false> / k_apply)
    int32_t *lrate;         // [block][L] cumulative bytes
    // layer assignment inputs (k_t2_wave<false>): hulls, thresholds
    const uint8_t *nhull, *hpass, *npasses;
    const uint64_t *hkey, *K;  // K: kMaxLayers per rate-control group
    const int32_t *grp_b0;     // the groups' block ranges (Plan::grp_b0)
    int ngroups;
    const int32_t *rates;
    int lossless;
    int L, sop, eph, plt;
    uint32_t *tt;           // tag-tree nodes: value | low << 8 | known << 16
    int8_t *lblock, *incl;  // per block coding state
    uint32_t *pk_len;       // [nprec * L] SOP + header + EPH + body
    uint32_t *tp_len;       // [ntp] Psot
    uint32_t *tp_hdr;       // [ntp] SOT + PLT + SOD
    uint64_t *tp_off;       // [ntp] offset of the tile-part in the part
    uint64_t *pk_off;       // [nprec * L] offset of the packet (its SOP) in `out`
    uint64_t *blkdst;       // [block][L] offset of the block's layer-l bytes in `out`
    uint8_t *out;           // the part: tile-parts from byte `base`
    uint64_t base;
    const int *halt;        // sizing kernels do nothing while *halt (device rate loop); may be null
};

// Packet-header bit writer (B.10.1): MSB first, a byte after 0xFF carries 7
// bits; a header never ends in 0xFF (t2.cpp Bits, oracle bw_*).
template <bool EMIT>
struct DevBits {
    uint8_t *p;
    uint32_t nbytes;
    uint64_t acc;
    int n, cap;
    __device__ __forceinline__ void init(uint8_t *dst) { p = dst; nbytes = 0; acc = 0; n = 0; cap = 8; }
    __device__ __forceinline__ void put(uint32_t val, int nb) {
        acc = (acc << nb) | val;
        n += nb;
        while (n >= cap) {
            n -= cap;
            const uint32_t byte = (uint32_t)(acc >> n) & ((1u << cap) - 1u);
            if (EMIT) p[nbytes] = (uint8_t)byte;
            nbytes++;
            cap = (byte == 0xFF) ? 7 : 8;
        }
    }
    __device__ __forceinline__ void bit(int b) { put((uint32_t)(b & 1), 1); }
    __device__ __forceinline__ void flush() {
        if (n) {
            const uint32_t byte = (uint32_t)(acc << (cap - n)) & ((1u << cap) - 1u);
            if (EMIT) p[nbytes] = (uint8_t)byte;
            nbytes++;
        } else if (cap == 7) {
            if (EMIT) p[nbytes] = 0;
            nbytes++;
        }
        cap = 8;
        n = 0;
        acc = 0;
    }
};

// Tag trees (B.10.2).  A tree over a w x h leaf grid is stored level by
// level (raster inside a level, level sizes ceil(w / 2^k) x ceil(h / 2^k)),
// each node one word: value | low << 8 | known << 16.  Geometry is recomputed
// from (w, h) on every walk, so a lane keeps no arrays (no scratch memory).
__device__ __forceinline__ int tree_size(int w, int h) {
    int n = 0;
    for (;;) {
        n += w * h;
        if (w == 1 && h == 1) return n;
        w = (w + 1) >> 1;
        h = (h + 1) >> 1;
    }
}

__device__ __forceinline__ void tree_set(uint32_t *nd, int w, int h, int leaf, int v) {
    int x = leaf % w, y = leaf / w, base = 0;
    for (;;) {
        uint32_t &e = nd[base + y * w + x];
        if ((int)(e & 0xFFu) <= v) return;
        e = (e & ~0xFFu) | (uint32_t)v;
        if (w == 1 && h == 1) return;
        base += w * h;
        w = (w + 1) >> 1;
        h = (h + 1) >> 1;
        x >>= 1;
        y >>= 1;
    }
}

// Codes leaf `leaf` against `threshold`, root first (t2.cpp / oracle tt_encode).
template <bool EMIT>
__device__ __forceinline__ void tree_encode(uint32_t *nd, int w, int h, int leaf, int threshold, DevBits<EMIT> &bw) {
    const int lx = leaf % w, ly = leaf / w;
    int nlev = 1;
    for (int cw = w, ch = h; cw != 1 || ch != 1; cw = (cw + 1) >> 1, ch = (ch + 1) >> 1) nlev++;
    int low = 0;
    for (int k = nlev - 1; k >= 0; k--) {
        int base = 0, cw = w, ch = h;
        for (int j = 0; j < k; j++) {
            base += cw * ch;
            cw = (cw + 1) >> 1;
            ch = (ch + 1) >> 1;
        }
        uint32_t &e = nd[base + (ly >> k) * cw + (lx >> k)];
        const int value = (int)(e & 0xFFu);
        int nlow = (int)((e >> 8) & 0xFFu);
        bool known = (e >> 16) & 1u;
        if (low > nlow) nlow = low;
        else low = nlow;
        // B.10.2 walk, as one field: a 0 per step of `low` up to
        // min(value, threshold), then a 1 if the value is reached below the
        // threshold and not yet known
        const int nz = max(0, min(value, threshold) - low);
        low += nz;
        const bool one = low < threshold && !known;
        if (one) known = true;
        const int nb = nz + (one ? 1 : 0);
        if (nb > 32) {
            bw.put(0u, nb - 32);
            bw.put(one ? 1u : 0u, 32);
        } else if (nb > 0) {
            bw.put(one ? 1u : 0u, nb);
        }
        e = (uint32_t)value | ((uint32_t)low << 8) | (known ? (1u << 16) : 0u);
    }
}

__device__ __forceinline__ int dev_floor_log2(int v) { return 31 - __clz(v); }

// One precinct's L packets (oracle encode_packet).  Tag-tree nodes live in
// the lane's LDS slot when they fit (the recipe's precincts: at most 2 x 2
// blocks per band, 30 nodes), else in the global scratch.
constexpr int kLdsNodes = 48;

template <bool EMIT>
__global__ void __launch_bounds__(64) k_t2_code(T2Args a) {
    __shared__ uint32_t lds_nodes[64 * kLdsNodes];
    const int pi = blockIdx.x * 64 + threadIdx.x;
    if (pi >= a.nprec || (!EMIT && a.halt && *a.halt)) return;
    const PrecDesc d = a.prec[pi];
    const int L = a.L;
    int nodes = 0;
#pragma unroll
    for (int bi = 0; bi < 3; bi++)
        if (bi < d.nb && d.ncw[bi] && d.nch[bi]) nodes += 2 * tree_size(d.ncw[bi], d.nch[bi]);
    uint32_t *tt = nodes <= kLdsNodes ? lds_nodes + threadIdx.x * kLdsNodes : a.tt + d.tt_off;
    for (int i = 0; i < nodes; i++) tt[i] = 0xFFu;  // value 255 = unset, low 0, not known
    // node offsets of the (inclusion, zero bit-plane) trees of each band
    int toff[3];
    {
        int o = 0;
#pragma unroll
        for (int bi = 0; bi < 3; bi++) {
            toff[bi] = o;
            if (bi < d.nb && d.ncw[bi] && d.nch[bi]) o += 2 * tree_size(d.ncw[bi], d.nch[bi]);
        }
    }
#pragma unroll
    for (int bi = 0; bi < 3; bi++) {
        const int w = bi < d.nb ? d.ncw[bi] : 0, h = bi < d.nb ? d.nch[bi] : 0;
        if (!w || !h) continue;
        uint32_t *ti = tt + toff[bi], *tz = ti + tree_size(w, h);
        for (int k = 0; k < w * h; k++) {
            const int b = d.first[bi] + k;
            a.lblock[b] = 3;
            a.incl[b] = -1;
            const uint8_t *nb = a.nl + (size_t)b * L;
            int first = L;
            for (int l = 0; l < L; l++)
                if (nb[l] > 0) { first = l; break; }
            tree_set(ti, w, h, k, first);
            tree_set(tz, w, h, k, a.blocks[b].Mb - a.P[b]);
        }
    }
    const uint32_t fixed = (a.sop ? 6u : 0u) + (a.eph ? 2u : 0u);
    for (int l = 0; l < L; l++) {
        const size_t pk = (size_t)pi * L + l;
        bool nonempty = false;
#pragma unroll
        for (int bi = 0; bi < 3; bi++) {
            const int nk = bi < d.nb ? d.ncw[bi] * d.nch[bi] : 0;
            for (int k = 0; k < nk && !nonempty; k++) {
                const uint8_t *nb = a.nl + (size_t)(d.first[bi] + k) * L;
                if (nb[l] > (l ? nb[l - 1] : 0)) nonempty = true;
            }
        }
        uint8_t *o = nullptr;
        if (EMIT) {
            o = a.out + a.pk_off[pk];
            if (a.sop) {
                const uint32_t ns = (uint32_t)(d.nsop0 + l) & 0xFFFFu;
                o[0] = 0xFF; o[1] = 0x91; o[2] = 0; o[3] = 4; o[4] = (uint8_t)(ns >> 8); o[5] = (uint8_t)ns;
                o += 6;
            }
        }
        DevBits<EMIT> w;
        w.init(o);
        w.bit(nonempty ? 1 : 0);
        uint32_t body = 0;
        if (nonempty) {
#pragma unroll
            for (int bi = 0; bi < 3; bi++) {
                const int cw = bi < d.nb ? d.ncw[bi] : 0, ch = bi < d.nb ? d.nch[bi] : 0;
                if (!cw || !ch) continue;
                uint32_t *ti = tt + toff[bi], *tz = ti + tree_size(cw, ch);
                for (int k = 0; k < cw * ch; k++) {
                    const int b = d.first[bi] + k;
                    const uint8_t *nb = a.nl + (size_t)b * L;
                    const int n = nb[l] - (l ? nb[l - 1] : 0);
                    const bool first_time = a.incl[b] < 0;
                    if (first_time) tree_encode(ti, cw, ch, k, l + 1, w);
                    else w.bit(n > 0 ? 1 : 0);
                    if (n <= 0) continue;
                    if (first_time) {
                        tree_encode(tz, cw, ch, k, 1 << 20, w);
                        a.incl[b] = (int8_t)l;
                    }
                    // number of passes, Table B.4
                    if (n == 1) w.bit(0);
                    else if (n == 2) w.put(2u, 2);
                    else if (n <= 5) w.put((3u << 2) | (uint32_t)(n - 3), 4);
                    else if (n <= 36) w.put((15u << 5) | (uint32_t)(n - 6), 9);
                    else w.put((511u << 7) | (uint32_t)(n - 37), 16);
                    const int32_t *lr = a.lrate + (size_t)b * L;
                    const int r0 = l ? lr[l - 1] : 0;
                    const int len = lr[l] - r0;
                    int lb = a.lblock[b];
                    int nbits = lb + dev_floor_log2(n);
                    while (len >= (1 << nbits)) { w.bit(1); lb++; nbits++; }
                    a.lblock[b] = (int8_t)lb;
                    w.bit(0);
                    w.put((uint32_t)len, nbits);
                    if (EMIT) a.blkdst[(size_t)b * L + l] = body;  // relative; the header length is added below
                    body += (uint32_t)len;
                }
            }
        }
        w.flush();
        if (EMIT) {
            o += w.nbytes;
            if (a.eph) { o[0] = 0xFF; o[1] = 0x92; o += 2; }
            // body pieces start here, in block order
            const uint64_t at = (uint64_t)(o - a.out);
            if (nonempty)
#pragma unroll
                for (int bi = 0; bi < 3; bi++) {
                    const int nk = bi < d.nb ? d.ncw[bi] * d.nch[bi] : 0;
                    for (int k = 0; k < nk; k++) {
                        const int b = d.first[bi] + k;
                        const uint8_t *nb = a.nl + (size_t)b * L;
                        if (nb[l] > (l ? nb[l - 1] : 0)) a.blkdst[(size_t)b * L + l] += at;
                    }
                }
        } else {
            a.pk_len[pk] = fixed + w.nbytes + body;
        }
    }
}

// --------------------------------------------------------------------------
// k_t2_wave: one wave per precinct, lane j = the precinct's j-th code-block
// (bands in order, raster order inside a band), for precincts of <= 64
// blocks (the recipe's: at most 2 x 2 per band).  Every header bit of a
// packet is worked out by the lanes in parallel -- the tag-tree bits
// included -- and laid out in LDS by a prefix sum of the lanes' bit counts;
// the 0xFF bit stuffing then runs a lane per packet.  No global memory is
// touched inside the layer loop.
//
// Tag trees in closed form (what tree_encode's walk amounts to; k_t2_code
// keeps the walk).  Inclusion tree, packet l (threshold l+1): a leaf is
// coded in every non-empty packet up to its inclusion layer, so a node is
// visited in every non-empty packet up to the last of its leaves'; entering
// packet l its state is low = min(v, tp), known = (v < tp), tp = 1 + the
// last non-empty packet before l (0: none), and its parent leaves it the
// lower bound min(pv, l+1) (pv <= v; the root's pv: 0).  Only the first
// visiting leaf (block order) writes the node's bits: nz = min(v, l+1) -
// max(min(v, tp), min(pv, l+1)) "0"s, then a "1" if tp <= v <= l.  The
// nodes a leaf writes are a suffix of its root-to-leaf path, whose "0"s add
// up to at most l+1.  Zero bit-plane tree (threshold unbounded), coded when
// a leaf is first included: a node writes (v - pv) "0"s and a "1" on its
// first visit ever, by the leaf of its subtree included first (earliest
// layer, then block order); those nodes are a suffix of that leaf's
// root-to-leaf path.
// The sizing pass (EMIT = false) also assigns each block its passes per layer
// from the thresholds K (what k_apply does for the serial kernel) and writes
// nl / lrate for the emission pass and k_t2_copy.
// --------------------------------------------------------------------------
constexpr int kT2Waves = 4;     // precincts per workgroup
constexpr int kTreeLev = 7;     // levels of a tag tree over <= 64 leaves
constexpr int kBitWords = 512;  // pending packet headers in LDS, per wave
constexpr int kWaveMaxMb = 48;  // a leaf's zero bit-plane path stays within 64 bits (host check)
// One wave's slice of k_t2_wave's dynamic LDS, sized by the layer count
// (t2_lane_bytes): L = 6 takes 4 KB a wave, 16 KB a workgroup -- sized for
// 32 layers it was 48 KB, and under load a workgroup waited for a CU to free
// that much.
struct T2LaneShared {
    int32_t *lr;    // [L][64] cumulative bytes per layer
    uint32_t *bits; // [kBitWords] header bits of the pending packets, MSB first, a zero word after each
    uint8_t *nl;    // [L][64] cumulative passes per layer
};
__host__ __device__ constexpr size_t t2_lane_bytes(int L) {
    return ((size_t)L * 64 * 5 + (size_t)kBitWords * 4 + 15) & ~(size_t)15;
}
__device__ __forceinline__ T2LaneShared t2_lane(uint8_t *dyn, int L, int wv) {
    uint8_t *p = dyn + (size_t)wv * t2_lane_bytes(L);
    T2LaneShared S;
    S.lr = (int32_t *)p;
    S.bits = (uint32_t *)(p + (size_t)L * 64 * 4);
    S.nl = p + (size_t)L * 64 * 4 + (size_t)kBitWords * 4;
    return S;
}

// the lanes of one wave see each other's LDS writes in program order (the
// LDS performs a wave's operations in issue order); this only keeps the
// compiler from moving or caching memory accesses across the point -- no
// s_waitcnt (a wavefront-scope fence waited for every global store in flight)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// OR the nb (0..64) low bits of v, MSB first, into the LDS bit string at bit p
__device__ __forceinline__ void lds_put_bits(uint32_t *buf, uint32_t p, uint64_t v, int nb) {
    if (nb <= 0) return;
    const uint64_t x = v << (64 - nb);
    const int sh = (int)(p & 31u);
    uint32_t *w = buf + (p >> 5);
    const uint64_t hi = x >> sh;
    const uint32_t w0 = (uint32_t)(hi >> 32), w1 = (uint32_t)hi, w2 = sh ? (uint32_t)((x << (64 - sh)) >> 32) : 0u;
    if (w0) atomicOr(w, w0);
    if (w1) atomicOr(w + 1, w1);
    if (w2) atomicOr(w + 2, w2);
}

// B.10.1 bit stuffing of the header bit string [p0, p0 + nbits) (DevBits):
// 8 bits a byte, 7 after an 0xFF, a 0 byte if it would end in 0xFF.  The
// string is followed by a zero word, so the two-word window never reads
// another packet's bits.  Returns the byte count (EMIT: bytes to o).
template <bool EMIT>
__device__ __forceinline__ uint32_t stuff_header(const uint32_t *buf, uint32_t p0, uint32_t nbits, uint8_t *o) {
    uint32_t q = 0, nbytes = 0, byte = 0;
    int cap = 8;
    while (q < nbits) {
        const uint32_t p = p0 + q;
        const uint64_t win = ((uint64_t)buf[p >> 5] << 32) | buf[(p >> 5) + 1];
        byte = (uint32_t)(win >> (64 - cap - (int)(p & 31u))) & ((1u << cap) - 1u);
        if (EMIT) o[nbytes] = (uint8_t)byte;
        nbytes++;
        q += (uint32_t)cap;
        cap = byte == 0xFFu ? 7 : 8;
    }
    if (byte == 0xFFu) {
        if (EMIT) o[nbytes] = 0;
        nbytes++;
    }
    return nbytes;
}

// precinct pi's L packets, by one wave (k_t2_wave)
template <bool EMIT>
__device__ __forceinline__ void t2_wave_precinct(const T2Args &a, const T2LaneShared &S, int pi) {
    const int lane = threadIdx.x & 63;
    const PrecDesc d = a.prec[pi];
    const int L = a.L;
    // lane -> (band, leaf, block)
    const int c0 = d.nb > 0 ? d.ncw[0] * d.nch[0] : 0, c1 = d.nb > 1 ? d.ncw[1] * d.nch[1] : 0,
              c2 = d.nb > 2 ? d.ncw[2] * d.nch[2] : 0;
    const int nbt = c0 + c1 + c2;
    const bool own = lane < nbt;
    const int bi = lane < c0 ? 0 : (lane < c0 + c1 ? 1 : 2);
    const int leaf = own ? lane - (bi == 0 ? 0 : (bi == 1 ? c0 : c0 + c1)) : 0;
    // (the band's fields by select: an indexed PrecDesc would live in scratch)
    const int bfirst = bi == 0 ? d.first[0] : (bi == 1 ? d.first[1] : d.first[2]);
    const int bcw = bi == 0 ? d.ncw[0] : (bi == 1 ? d.ncw[1] : d.ncw[2]);
    const int bch = bi == 0 ? d.nch[0] : (bi == 1 ? d.nch[1] : d.nch[2]);
    const int b = own ? bfirst + leaf : 0;
    int zero_planes = 0;
    if (own) {
        zero_planes = a.blocks[b].Mb - a.P[b];
        uint8_t *gnl = a.nl + (size_t)b * L;
        int32_t *glr = a.lrate + (size_t)b * L;
        if (!EMIT) {
            // passes per layer from the thresholds: the last hull point whose
            // slope key >= K (lossless: the last layer takes every pass).
            // Hull keys strictly decrease, so each layer's point is found by
            // walking from the previous layer's (thresholds fall with the
            // layer: forward); the first 8 keys are loaded together
            const int nh = a.nhull[b];
            const uint8_t *hp = a.hpass + (size_t)b * (kMaxPasses + 1);
            const uint64_t *hk = a.hkey + (size_t)b * (kMaxPasses + 1);
            const int32_t *R = a.rates + (size_t)b * kMaxPasses;
            const uint64_t *Kb = a.K + (size_t)block_group(a.grp_b0, a.ngroups, b) * kMaxLayers;
            uint64_t k8[8];
#pragma unroll
            for (int i = 0; i < 8; i++) k8[i] = hk[min(i, kMaxPasses)];
            // layers in groups of 8: the hull points of the group first (keys
            // in registers), then its 8 pass-table loads together, then the 8
            // rate loads together (two load round trips per group, not two
            // per layer)
            int at = 0;  // last hull point with key >= K (point 0: nothing)
            auto key = [&](int i) {  // (k8 by select: an indexed k8 would live in scratch)
                uint64_t r = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) r = i == t ? k8[t] : r;
                return i < 8 ? r : hk[i];
            };
            for (int l0 = 0; l0 < L; l0 += 8) {
                int atv[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int l = l0 + j;
                    if (l < L && !(a.lossless && l == L - 1)) {
                        const uint64_t K = Kb[l];
                        while (at + 1 < nh && key(at + 1) >= K) at++;
                        while (at > 0 && key(at) < K) at--;  // (a threshold above the previous one)
                    }
                    atv[j] = at;
                }
                int ncv[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int l = l0 + j;
                    ncv[j] = (a.lossless && l == L - 1) ? (int)a.npasses[b] : (int)hp[atv[j]];
                }
                int32_t rv[8];
#pragma unroll
                for (int j = 0; j < 8; j++) rv[j] = R[max(ncv[j], 1) - 1];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int l = l0 + j;
                    if (l >= L) break;
                    const int32_t r = ncv[j] ? rv[j] : 0;
                    S.nl[l * 64 + lane] = (uint8_t)ncv[j];
                    S.lr[l * 64 + lane] = r;
                    gnl[l] = (uint8_t)ncv[j];
                    glr[l] = r;
                }
            }
        } else {
            for (int l = 0; l < L; l++) {
                S.nl[l * 64 + lane] = gnl[l];
                S.lr[l * 64 + lane] = glr[l];
            }
        }
    }
    int firstl = L;  // inclusion layer (L: never)
    if (own)
        for (int l = 0; l < L; l++)
            if (S.nl[l * 64 + lane] > 0) {
                firstl = l;
                break;
            }
    // the leaf's tag-tree path: per level the lanes under the same node, the
    // node's inclusion and zero bit-plane values, and the node's first
    // zero-bit-plane visitor (inclusion layer << 6 | lane)
    const int cw0 = own ? bcw : 1, ch0 = own ? bch : 1;
    const int lx = leaf % cw0, ly = leaf / cw0;
    int nlev = 1;
    for (int w = cw0, h = ch0; w != 1 || h != 1; w = (w + 1) >> 1, h = (h + 1) >> 1) nlev++;
    const int key = (bi << 16) | (ly << 8) | lx;
    uint64_t imask[kTreeLev];
    int ival[kTreeLev], zval[kTreeLev], zbest[kTreeLev];
#pragma unroll
    for (int k = 0; k < kTreeLev; k++) {
        imask[k] = 0;
        ival[k] = L;
        zval[k] = 255;
        zbest[k] = 0x7FFFFFFF;
    }
    for (int j = 0; j < nbt; j++) {
        const int kj = __builtin_amdgcn_readlane(key, j);
        const int fj = __builtin_amdgcn_readlane(firstl, j), zj = __builtin_amdgcn_readlane(zero_planes, j);
        const int xj = kj & 0xFF, yj = (kj >> 8) & 0xFF;
        const bool band = (kj >> 16) == bi;
#pragma unroll
        for (int k = 0; k < kTreeLev; k++)
            if (band && (xj >> k) == (lx >> k) && (yj >> k) == (ly >> k)) {
                imask[k] |= 1ull << j;
                ival[k] = min(ival[k], fj);
                zval[k] = min(zval[k], zj);
                if (fj < L) zbest[k] = min(zbest[k], (fj << 6) | j);
            }
    }
    const int myz = (firstl << 6) | lane;
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t *buf = S.bits;
    for (int i = lane; i < kBitWords; i += 64) buf[i] = 0;
    wave_lds_sync();
    int lb = 3;  // the lane's block: Lblock
    const uint32_t fixed = (a.sop ? 6u : 0u) + (a.eph ? 2u : 0u);
    // pending packets [l0, l) occupy buf[0, used); lane i holds packet l0 + i's
    // first word, bit count and body bytes (all wave-uniform but the lane ones)
    uint32_t used = 0, pws = 0, pnb = 0, pbody = 0;
    int l0 = 0;
    int tp = 0;  // 1 + the last non-empty packet (wave-uniform)
    for (int l = 0; l <= L; l++) {
        int n = 0, len = 0;
        uint64_t I = 0, Z = 0, p1v = 0;  // inclusion bits, zero bit-plane bits, pass count codeword
        int nI = 0, nZ = 0, p1n = 0, p2n = 0;
        uint32_t nbits = 0, need = 0, off = 0, body = 0;
        if (l < L) {
            // this block's part of packet l
            if (own) {
                n = (int)S.nl[l * 64 + lane] - (l ? (int)S.nl[(l - 1) * 64 + lane] : 0);
                len = S.lr[l * 64 + lane] - (l ? S.lr[(l - 1) * 64 + lane] : 0);
            }
            if (n > 0) {
                uint32_t cv;
                int cn;
                if (n == 1) { cv = 0u; cn = 1; }
                else if (n == 2) { cv = 2u; cn = 2; }
                else if (n <= 5) { cv = (3u << 2) | (uint32_t)(n - 3); cn = 4; }
                else if (n <= 36) { cv = (15u << 5) | (uint32_t)(n - 6); cn = 9; }
                else { cv = (511u << 7) | (uint32_t)(n - 37); cn = 16; }
                const int nbits0 = lb + dev_floor_log2(n);
                const int bl = len > 0 ? 32 - __clz(len) : 0;  // bit length of len
                const int extra = bl > nbits0 ? bl - nbits0 : 0;
                lb += extra;
                p1v = ((uint64_t)cv << (extra + 1)) | (((1ull << extra) - 1ull) << 1);
                p1n = cn + extra + 1;
                p2n = lb + dev_floor_log2(n);
            }
            const bool nonempty = __ballot(n > 0) != 0ull;
            const bool visitor = own && firstl >= l;  // not yet included: codes the inclusion tree
            const uint64_t vis = __ballot(visitor);
            if (nonempty && own) {
                if (visitor) {
#pragma unroll
                    for (int k = kTreeLev - 1; k >= 0; k--) {
                        if (k >= nlev || (imask[k] & vis & below)) continue;
                        const int v = ival[k], pv = k + 1 < nlev ? ival[k + 1 < kTreeLev ? k + 1 : k] : 0;
                        const int nz = max(0, min(v, l + 1) - max(min(v, tp), min(pv, l + 1)));
                        const int one = (v >= tp && v <= l) ? 1 : 0;
                        I = (I << (nz + one)) | (uint64_t)one;
                        nI += nz + one;
                    }
                    if (n > 0)  // first inclusion: the zero bit-plane path
#pragma unroll
                        for (int k = kTreeLev - 1; k >= 0; k--) {
                            if (k >= nlev || zbest[k] != myz) continue;
                            const int z = zval[k] - (k + 1 < nlev ? zval[k + 1 < kTreeLev ? k + 1 : k] : 0);
                            Z = (Z << (z + 1)) | 1u;
                            nZ += z + 1;
                        }
                } else {
                    I = n > 0 ? 1u : 0u;
                    nI = 1;
                }
            }
            if (nonempty) tp = l + 1;
            const uint32_t T = (uint32_t)(nI + nZ + p1n + p2n);
            off = wave_incl_scan(T) - T;
            nbits = 1u + (uint32_t)__shfl((int)(off + T), 63, 64);
            const uint32_t lin = n > 0 ? (uint32_t)len : 0u;
            body = (uint32_t)__shfl((int)wave_incl_scan(lin), 63, 64);
            need = (nbits + 31u) / 32u + 1u;  // + the zero word
            if (!nonempty) nbits = 1;
        }
        if (l == L || used + need > (uint32_t)kBitWords) {
            // stuff the pending packets, a lane each
            wave_lds_sync();
            uint32_t hdr = 0;
            if (lane < l - l0) {
                const size_t pk = (size_t)pi * L + l0 + lane;
                uint8_t *o = nullptr;
                if (EMIT) {
                    o = a.out + a.pk_off[pk];
                    if (a.sop) {
                        const uint32_t ns = (uint32_t)(d.nsop0 + l0 + lane) & 0xFFFFu;
                        o[0] = 0xFF; o[1] = 0x91; o[2] = 0; o[3] = 4; o[4] = (uint8_t)(ns >> 8); o[5] = (uint8_t)ns;
                        o += 6;
                    }
                }
                const uint32_t nbytes = stuff_header<EMIT>(buf, pws * 32u, pnb, o);
                if (EMIT) {
                    if (a.eph) { o[nbytes] = 0xFF; o[nbytes + 1] = 0x92; }
                    hdr = fixed + nbytes;
                } else {
                    a.pk_len[pk] = fixed + nbytes + pbody;
                }
            }
            if (EMIT)  // body pieces follow each header, in block order
                for (int l2 = l0; l2 < l; l2++) {
                    int n2 = 0, len2 = 0;
                    if (own) {
                        n2 = (int)S.nl[l2 * 64 + lane] - (l2 ? (int)S.nl[(l2 - 1) * 64 + lane] : 0);
                        len2 = S.lr[l2 * 64 + lane] - (l2 ? S.lr[(l2 - 1) * 64 + lane] : 0);
                    }
                    const uint32_t lin2 = n2 > 0 ? (uint32_t)len2 : 0u;
                    const uint32_t before = wave_incl_scan(lin2) - lin2;
                    const uint32_t h2 = (uint32_t)__builtin_amdgcn_readlane((int)hdr, l2 - l0);
                    const size_t pk2 = (size_t)pi * L + l2;
                    if (n2 > 0) a.blkdst[(size_t)b * L + l2] = a.pk_off[pk2] + h2 + before;
                }
            wave_lds_sync();
            for (uint32_t i = lane; i < used; i += 64) buf[i] = 0;
            wave_lds_sync();
            used = 0;
            l0 = l;
            if (l == L) break;
        }
        // packet l at buf[used]: the "packet present" bit, then each block's bits
        const uint32_t p = used * 32u;
        if (lane == 0 && nbits > 1) atomicOr(&buf[used], 0x80000000u);
        uint32_t q = p + 1u + off;
        lds_put_bits(buf, q, I, nI);
        q += (uint32_t)nI;
        lds_put_bits(buf, q, Z, nZ);
        q += (uint32_t)nZ;
        lds_put_bits(buf, q, p1v, p1n);
        q += (uint32_t)p1n;
        lds_put_bits(buf, q, (uint64_t)(uint32_t)len, p2n);
        if (lane == l - l0) {
            pws = used;
            pnb = nbits;
            pbody = body;
        }
        used += need;
    }
}

__device__ __forceinline__ int varint_len(uint32_t v) {
    int k = 1;
    while (v >>= 7) k++;
    return k;
}

// One workgroup: each tile-part's size (SOT + PLT + SOD + packets), their
// offsets in code-stream order, and the sums the host needs (part size,
// header bytes, bytes per layer, tier-1 totals); in the device rate loop
// (rate != null) also the loop's step (rate_step).
struct RateStepArgs {
    RateState *rs;
    int64_t *budget;
    RateState *out_rs;
    T2Summary *out_sum;
};
__device__ __forceinline__ void tpart_size(const T2Args &a, int t) {
    const TpDesc d = a.tps[t];
    const size_t p0 = (size_t)d.prec0 * a.L, p1 = (size_t)(d.prec0 + d.nprec) * a.L;
    uint64_t body = 0, plt = 0, seg = 0;
    for (size_t i0 = p0; i0 < p1; i0 += 8) {  // 8 lengths' loads in flight at a time
        uint32_t l8[8];
#pragma unroll
        for (int j = 0; j < 8; j++) l8[j] = a.pk_len[min(i0 + j, p1 - 1)];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const size_t i = i0 + j;
            if (i >= p1) break;
            const uint32_t len = l8[j];
            body += len;
            if (a.plt) {
                const uint64_t k = (uint64_t)varint_len(len);
                if (i == p0 || seg + k > 65532) {
                    if (i != p0) plt += 5 + seg;
                    seg = 0;
                }
                seg += k;
            }
        }
    }
    if (a.plt && p1 > p0) plt += 5 + seg;
    a.tp_hdr[t] = (uint32_t)(14 + plt);
    a.tp_len[t] = (uint32_t)(14 + plt + body);
}

// One workgroup of kTotThreads: tile-part sizes (a thread per tile-part, or
// a contiguous run of them), their offsets by a workgroup scan, and every sum
// the host needs as per-thread partials reduced through one LDS table (a wave
// sum each, then the waves' partials): no thread walks a serial loop over
// the others' results.
constexpr int kTotSums = kMaxLayers + 5;  // layers, tp headers, t1 bytes, passes, decisions, skipped
// what the sizing totals read besides T2Args
struct T2TotalArgs {
    int nblocks;
    const int32_t *lengths;
    const uint8_t *npasses, *pmin;
    const int *t1err;
    const unsigned long long *pool_used;  // decision-stream pool fill (emit_t1_items)
    const uint64_t *kc;  // [group][kMaxLayers]; Kdu-Layer-Info takes each layer's strictest (largest)
    int ngroups;
    const unsigned long long *acc;
    T2Summary *sum;
    RateStepArgs rate;
    uint32_t *ticket;  // k_t2_wave<false> with the totals fused: arrival counter (left 0)
};

// One workgroup of NT threads: tile-part sizes (a thread per tile-part, or a
// contiguous run of them), their offsets by a workgroup scan, and every sum
// the host needs as per-thread partials reduced through one LDS table (a wave
// sum each, then the waves' partials): no thread walks a serial loop over
// the others' results.  Run by k_t2_total, or by the last workgroup of
// k_t2_wave<false> to arrive.  T1: also the tier-1 totals (k_hull has
// already summed them into *sum once per encode; k_t2_total re-sums them).
template <int NT, bool T1>
__device__ __forceinline__ void t2_total_body(const T2Args &a, const T2TotalArgs &ta, uint64_t *wsum,
                                              int64_t (*red)[kTotSums]) {
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int L = a.L;
    const int chunk = (a.ntp + NT - 1) / NT;
    const int t0 = min(a.ntp, tid * chunk), t1 = min(a.ntp, t0 + chunk);
    for (int t = t0; t < t1; t++) tpart_size(a, t);
    uint64_t s = 0, hdr = 0;
    for (int t = t0; t < t1; t++) s += a.tp_len[t];
    uint64_t tot;
    uint64_t o = wg_excl_scan64<NT>(s, wsum, tot);
    if (tid == 0) ta.sum->part_bytes = (int64_t)tot;
    for (int t = t0; t < t1; t++) {
        a.tp_off[t] = o;
        o += a.tp_len[t];
        hdr += a.tp_hdr[t];
    }
    // per-layer packet bytes: precinct-major, a precinct's L lengths per thread
    int64_t lay[kMaxLayers];
#pragma unroll
    for (int l = 0; l < kMaxLayers; l++) lay[l] = 0;
    for (int pq = tid; pq < a.nprec; pq += NT) {
        const uint32_t *pl = a.pk_len + (size_t)pq * L;
#pragma unroll
        for (int l = 0; l < kMaxLayers; l++)
            if (l < L) lay[l] += pl[l];
    }
    // tier-1 totals (acc: decisions per block in the low 40 bits, k_t1_cm3),
    // 4 blocks' loads in flight per thread
    int64_t tb = 0, tp = 0, nd = 0, skipped = 0;
    if (T1)
    for (int b0 = 0; b0 < ta.nblocks; b0 += 4 * NT) {
        int32_t ln[4];
        uint32_t np[4], pm[4];
        unsigned long long kk[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int b = min(b0 + u * NT + tid, ta.nblocks - 1);
            ln[u] = ta.lengths[b];
            np[u] = ta.npasses[b];
            kk[u] = ta.acc[b];
            pm[u] = ta.pmin[b];
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (b0 + u * NT + tid < ta.nblocks) {
                tb += ln[u];
                tp += np[u];
                nd += (int64_t)(kk[u] & ((1ull << 40) - 1ull));
                skipped |= pm[u] > 0;
            }
    }
    // reductions: wave sums, then thread j < kTotSums adds the waves' partials of sum j
    auto wave_put = [&](int j, int64_t v) {
        v = wave_sum64(v);
        if (lane == 0) red[wv][j] = v;
    };
#pragma unroll
    for (int l = 0; l < kMaxLayers; l++)
        if (l < L) wave_put(l, lay[l]);
    wave_put(kMaxLayers + 0, (int64_t)hdr);
    if (T1) {
        wave_put(kMaxLayers + 1, tb);
        wave_put(kMaxLayers + 2, tp);
        wave_put(kMaxLayers + 3, nd);
        wave_put(kMaxLayers + 4, skipped);
    }
    __syncthreads();
    if (tid < (T1 ? kTotSums : kMaxLayers + 1) && (tid >= kMaxLayers || tid < L)) {
        int64_t v = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) v += red[w][tid];
        if (tid < kMaxLayers) ta.sum->layer_bytes[tid] = v;
        else if (tid == kMaxLayers + 0) ta.sum->tp_hdr_bytes = v;
        else if (tid == kMaxLayers + 1) ta.sum->t1_bytes = v;
        else if (tid == kMaxLayers + 2) ta.sum->coded_passes = v;
        else if (tid == kMaxLayers + 3) ta.sum->decisions = v;
        else ta.sum->skipped = v != 0;
    }
    if (tid < L) {
        uint64_t k = 0;
        if (ta.kc)
            for (int g = 0; g < ta.ngroups; g++) k = max(k, ta.kc[(size_t)g * kMaxLayers + tid]);
        ta.sum->kc[tid] = k;
    }
    if (tid == 0) {
        ta.sum->err = *ta.t1err;
        ta.sum->stream_need = ta.pool_used ? (int64_t)*ta.pool_used : 0;
    }
    if (ta.rate.rs) {
        __syncthreads();  // every field of *sum written
        if (tid == 0) rate_step(ta.rate.rs, ta.sum, L, ta.rate.budget, ta.rate.out_rs, ta.rate.out_sum);
    }
}

constexpr int kTotThreads = 1024, kTotWaves = kTotThreads / 64;
__global__ void __launch_bounds__(kTotThreads) k_t2_total(T2Args a, T2TotalArgs ta) {
    __shared__ uint64_t wsum[kTotWaves + 1];
    __shared__ int64_t red[kTotWaves][kTotSums];
    if (a.halt && *a.halt) return;  // the whole workgroup
    t2_total_body<kTotThreads, true>(a, ta, wsum, red);
}

// Packets, a wave per precinct (t2_wave_precinct).  The sizing pass with
// ta.ticket set also runs the totals: every workgroup publishes its packet
// lengths (release, arrival ticket) and the last to arrive acquires them and
// runs t2_total_body -- one launch less per rate iteration (cdna_hip_
// programming.md Guideline 16; no workgroup waits for another).
template <bool EMIT>
__global__ void __launch_bounds__(64 * kT2Waves) k_t2_wave(T2Args a, T2TotalArgs ta) {
    extern __shared__ __attribute__((aligned(16))) uint8_t t2dyn[];  // kT2Waves * t2_lane_bytes(L)
    __shared__ uint64_t wsum[kT2Waves + 1];
    __shared__ int64_t red[kT2Waves][kTotSums];
    __shared__ int last;
    const int wv = threadIdx.x >> 6;
    const int pi = blockIdx.x * kT2Waves + wv;
    if (!EMIT && a.halt && *a.halt) return;  // (the whole grid)
    if (pi < a.nprec) t2_wave_precinct<EMIT>(a, t2_lane(t2dyn, a.L, wv), pi);
    if (EMIT || !ta.ticket) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t t = __hip_atomic_fetch_add(ta.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = t == gridDim.x - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            *ta.ticket = 0u;  // for the next launch
        }
    }
    __syncthreads();
    if (!last) return;
    t2_total_body<64 * kT2Waves, false>(a, ta, wsum, red);
}

// SOT + PLT + SOD of each tile-part, and where each of its packets starts
__global__ void __launch_bounds__(64) k_t2_tp_emit(T2Args a) {
    const int t = blockIdx.x * 64 + threadIdx.x;
    if (t >= a.ntp) return;
    const TpDesc d = a.tps[t];
    uint8_t *p = a.out + a.base + a.tp_off[t];
    const uint32_t psot = a.tp_len[t];
    p[0] = 0xFF; p[1] = 0x90; p[2] = 0; p[3] = 10;
    p[4] = (uint8_t)(d.tile >> 8); p[5] = (uint8_t)d.tile;
    p[6] = (uint8_t)(psot >> 24); p[7] = (uint8_t)(psot >> 16); p[8] = (uint8_t)(psot >> 8); p[9] = (uint8_t)psot;
    p[10] = (uint8_t)d.tpsot;
    p[11] = (uint8_t)d.tnsot;
    p += 12;
    const size_t p0 = (size_t)d.prec0 * a.L, p1 = (size_t)(d.prec0 + d.nprec) * a.L;
    // packet lengths are loaded 8 at a time ahead of the byte stores (a load
    // after a byte store would wait for it: the stores may alias)
    if (a.plt && p1 > p0) {  // PLT segments (A.7.3): lengths as 7-bit groups, <= 65532 bytes each
        size_t i = p0;
        int z = 0;
        uint8_t *hdr = p;
        p += 5;
        uint32_t seg = 0;
        while (i < p1) {
            uint32_t l8[8];
#pragma unroll
            for (int j = 0; j < 8; j++) l8[j] = a.pk_len[min(i + j, p1 - 1)];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (i >= p1) break;
                const uint32_t len = l8[j];
                const int k = varint_len(len);
                if (seg + (uint32_t)k > 65532) {  // close this segment, open the next
                    hdr[0] = 0xFF; hdr[1] = 0x58;
                    hdr[2] = (uint8_t)((3 + seg) >> 8); hdr[3] = (uint8_t)(3 + seg);
                    hdr[4] = (uint8_t)z++;
                    hdr = p;
                    p += 5;
                    seg = 0;
                }
                for (int q = k - 1; q >= 0; q--) *p++ = (uint8_t)(((len >> (7 * q)) & 0x7F) | (q ? 0x80 : 0));
                seg += (uint32_t)k;
                i++;
            }
        }
        hdr[0] = 0xFF; hdr[1] = 0x58;
        hdr[2] = (uint8_t)((3 + seg) >> 8); hdr[3] = (uint8_t)(3 + seg);
        hdr[4] = (uint8_t)z;
    }
    p[0] = 0xFF; p[1] = 0x93;
    p += 2;
    uint64_t o = (uint64_t)(p - a.out);
    for (size_t i0 = p0; i0 < p1; i0 += 8) {
        uint32_t l8[8];
#pragma unroll
        for (int j = 0; j < 8; j++) l8[j] = a.pk_len[min(i0 + j, p1 - 1)];
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (i0 + j < p1) {
                a.pk_off[i0 + j] = o;
                o += l8[j];
            }
    }
}

// code-block bytes into the packet bodies: one wave per block, its layer
// pieces in turn; bytes move in 16-byte vector loads/stores where source and
// destination are both aligned, else one byte per lane
// A wave per block: lanes 0..L-1 read the layers' segment bounds and body
// offsets at once, then each layer's bytes go over as dwords aligned to the
// destination, each built from two source dwords by one v_alignbyte (the
// source reads up to 3 bytes past a segment: t1out carries 64 bytes of slack).
__global__ void __launch_bounds__(256) k_t2_copy(T2Args a, int nblocks, const uint8_t *t1out) {
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (b >= nblocks) return;
    const int L = a.L;
    int r1 = 0, r0 = 0, np = 0, pp = 0;
    uint64_t dst = 0;
    if (lane < L) {
        r1 = a.lrate[(size_t)b * L + lane];
        np = a.nl[(size_t)b * L + lane];
        if (lane) {
            r0 = a.lrate[(size_t)b * L + lane - 1];
            pp = a.nl[(size_t)b * L + lane - 1];
        }
        dst = a.blkdst[(size_t)b * L + lane];
    }
    const uint64_t live = __ballot(lane < L && np > pp);  // layers with bytes of this block
    const uint8_t *src0 = t1out + a.blocks[b].out_off;
    for (uint64_t m = live; m; m &= m - 1) {
        const int l = __builtin_ctzll(m);
        const int s0 = __builtin_amdgcn_readlane(r0, l);
        const int n = __builtin_amdgcn_readlane(r1, l) - s0;
        const uint8_t *s = src0 + s0;
        uint8_t *d = a.out + (((uint64_t)__builtin_amdgcn_readlane((uint32_t)(dst >> 32), l) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((uint32_t)dst, l));
        const int head = min(n, (int)((0u - (uint32_t)(uintptr_t)d) & 3u));
        if (lane < head) d[lane] = s[lane];
        const uint8_t *s4 = s + head;
        uint32_t *d4 = (uint32_t *)(d + head);
        const int nw = (n - head) >> 2;
        const uint32_t sh = (uint32_t)(uintptr_t)s4 & 3u;
        const uint32_t *sa = (const uint32_t *)(s4 - sh);
        for (int i = lane; i < nw; i += 64) d4[i] = __builtin_amdgcn_alignbyte(sa[i + 1], sa[i], sh);
        const int t0 = head + 4 * nw;
        if (lane < n - t0) d[t0 + lane] = s[t0 + lane];
    }
}

// Releases the SDMA copy of the code-stream (GpuEncoder::dma_to_host): the
// stream's earlier kernels have completed (their writes reached memory at
// kernel end), and this system-scope release store sets the copy's
// dependency signal to 0.
__global__ void __launch_bounds__(64) k_release_dma(int64_t *dep) {
    if (threadIdx.x == 0) __hip_atomic_store(dep, (int64_t)0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// --------------------------------------------------------------------------
// Host side (GpuEncoder)
// --------------------------------------------------------------------------
#define HSACHECK(x)                                                                    \
    do {                                                                               \
        hsa_status_t s_ = (x);                                                         \
        if (s_ != HSA_STATUS_SUCCESS) {                                                \
            const char *m_ = "?";                                                      \
            hsa_status_string(s_, &m_);                                                \
            err = std::string(#x) + ": " + m_;                                         \
            return false;                                                              \
        }                                                                              \
    } while (0)

// HSA signal waits take their timeout in system-timestamp ticks
static uint64_t hsa_ticks(uint64_t ns) {
    static const uint64_t freq = [] {
        uint64_t f = 0;
        if (hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &f) != HSA_STATUS_SUCCESS || !f) f = 1000000000ull;
        return f;
    }();
    return (uint64_t)((double)ns * (double)freq / 1e9) + 1;
}

static uint64_t mono_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// one slice of a wait for `sig` to drop below 1 (the copy's completion)
static jp2hip::SliceResult poll_signal(hsa_signal_t sig, uint64_t slice_ns) {
    const hsa_signal_value_t v =
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, hsa_ticks(slice_ns), HSA_WAIT_STATE_BLOCKED);
    return v < 0 ? jp2hip::SliceResult::Error : (v < 1 ? jp2hip::SliceResult::Done : jp2hip::SliceResult::Pending);
}

static constexpr uint64_t kWaitSliceNs = 50ull * 1000 * 1000;          // 50 ms
static constexpr uint64_t kDrainedGraceNs = 20ull * 1000 * 1000 * 1000;  // 20 s

static hsa_status_t first_cpu_agent(hsa_agent_t a, void *out) {
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
        *(hsa_agent_t *)out = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

// SDMA engines differ a lot in their device -> host rate (MI355X box,
// profiles/r05/sdma_engines.txt: engines 0, 2, 3 at 56.6 GB/s, engine 1 --
// the runtime's own pick -- at 30, engines 4-15 at 7-13), so the engines are
// timed once per process and GPU on a 32 MiB copy, and the contexts spread
// over the ones within 10 % of the fastest.
struct DmaGpu {
    std::mutex mu;            // this GPU's probe (other GPUs probe in parallel)
    bool probed = false;
    std::vector<int> fast;    // engine ids within 10 % of the fastest
    std::vector<std::pair<int, double>> rates;  // (engine, GB/s) as probed
    std::atomic<unsigned> next{0};               // round-robin cursor
};
struct DmaEngines {
    std::mutex mu;  // the map only
    std::map<uint64_t, std::unique_ptr<DmaGpu>> gpu;  // GPU agent handle -> its engines
};
static DmaEngines &dma_engines() {
    static DmaEngines *e = new DmaEngines();  // never destroyed: contexts may outlive static teardown
    return *e;
}

static int pick_dma_engine(hsa_agent_t gpu, hsa_agent_t cpu, hsa_signal_t sig) {
    DmaEngines &E = dma_engines();
    DmaGpu *G;
    {
        std::lock_guard<std::mutex> lk(E.mu);
        std::unique_ptr<DmaGpu> &slot = E.gpu[gpu.handle];
        if (!slot) slot.reset(new DmaGpu());
        G = slot.get();
    }
    {
        std::lock_guard<std::mutex> lk(G->mu);  // the first context of this GPU probes; the others wait
        if (!G->probed) {
            uint32_t mask = 0;
            const size_t n = 32u << 20;
            void *d = nullptr, *h = nullptr;
            if (hsa_amd_memory_copy_engine_status(cpu, gpu, &mask) == HSA_STATUS_SUCCESS && mask &&
                hipMalloc(&d, n) == hipSuccess && hipHostMalloc(&h, n, hipHostMallocDefault) == hipSuccess) {
                for (int e = 0; e < 16; e++) {
                    if (!(mask & (1u << e))) continue;
                    double best = 0.0;
                    for (int r = 0; r < 2; r++) {  // the first copy also maps the pages
                        hsa_signal_store_relaxed(sig, 1);
                        const auto t0 = std::chrono::steady_clock::now();
                        if (hsa_amd_memory_async_copy_on_engine(h, cpu, d, gpu, n, 0, nullptr, sig,
                                                                (hsa_amd_sdma_engine_id_t)(1u << e), true) != HSA_STATUS_SUCCESS)
                            break;
                        // nothing else is queued: a probe copy that takes more
                        // than a second is an engine to leave out
                        std::string perr;
                        if (!jp2hip::wait_bounded([&](uint64_t ns) { return poll_signal(sig, ns); },
                                                  [](std::string &) { return jp2hip::StreamState::Drained; }, mono_ns,
                                                  kWaitSliceNs, 1000ull * 1000 * 1000, "DMA engine probe", perr))
                            break;
                        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                        best = std::max(best, n / sec);
                    }
                    if (best > 0.0) G->rates.emplace_back(e, best / 1e9);
                }
                double top = 0.0;
                for (auto &r : G->rates) top = std::max(top, r.second);
                for (auto &r : G->rates)
                    if (r.second >= 0.9 * top) G->fast.push_back(r.first);
            }
            if (d) (void)hipFree(d);
            if (h) (void)hipHostFree(h);
            G->probed = true;  // empty `fast`: the runtime picks the engine
        }
    }
    if (G->fast.empty()) return -1;
    return G->fast[(size_t)(G->next++) % G->fast.size()];
}

// "GPU agent <handle>: engines e,e,.. used of (e rate, ...)" per probed GPU
std::string dma_engine_report() {
    DmaEngines &E = dma_engines();
    std::lock_guard<std::mutex> lk(E.mu);
    std::string out;
    char buf[64];
    for (auto &kv : E.gpu) {
        DmaGpu &G = *kv.second;
        std::lock_guard<std::mutex> lg(G.mu);
        if (!G.probed) continue;
        if (!out.empty()) out += "; ";
        out += "agent " + std::to_string(kv.first) + ": using";
        for (int e : G.fast) out += " " + std::to_string(e);
        if (G.fast.empty()) out += " the runtime's choice";
        out += " of";
        for (auto &r : G.rates) {
            std::snprintf(buf, sizeof buf, " %d:%.1fGB/s", r.first, r.second);
            out += buf;
        }
    }
    return out;
}

bool GpuEncoder::dma_init(std::string &err) {
    if (dma_ok) return true;
    if (!t2out.ptr) {
        err = "dma_init: no device buffer yet";
        return false;
    }
    if (!hsa_up) {  // the HIP runtime has initialised ROCr already; this takes a reference
        HSACHECK(hsa_init());
        hsa_up = true;
    }
    hsa_amd_pointer_info_t pi;
    std::memset(&pi, 0, sizeof pi);
    pi.size = sizeof pi;
    HSACHECK(hsa_amd_pointer_info(t2out.ptr, &pi, nullptr, nullptr, nullptr));
    dma_gpu = pi.agentOwner;
    if (hsa_iterate_agents(first_cpu_agent, &dma_cpu) != HSA_STATUS_INFO_BREAK) {
        err = "dma_init: no CPU agent";
        return false;
    }
    if (!dma_dep.handle) HSACHECK(hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &dma_dep));
    if (!dma_done.handle) HSACHECK(hsa_signal_create(1, 0, nullptr, &dma_done));
    HSACHECK(hsa_amd_signal_value_pointer(dma_dep, &dma_dep_val));
    dma_engine = pick_dma_engine(dma_gpu, dma_cpu, dma_done);
    dma_ok = true;
    return true;
}

// Everything enqueued on the stream so far, then `bytes` from device `src` to
// pinned `host_dst` on a DMA engine; returns when the bytes are in host memory.
bool GpuEncoder::dma_to_host(uint8_t *host_dst, const void *src, size_t bytes, std::string &err) {
    if (!dma_init(err)) return false;
    hsa_signal_store_relaxed(dma_dep, 1);
    hsa_signal_store_relaxed(dma_done, 1);
    hipLaunchKernelGGL(k_release_dma, dim3(1), dim3(64), 0, stream, (int64_t *)dma_dep_val);
    HIPCHECK(hipGetLastError());
    const hsa_status_t s =
        dma_engine >= 0
            ? hsa_amd_memory_async_copy_on_engine(host_dst, dma_cpu, src, dma_gpu, bytes, 1, &dma_dep, dma_done,
                                                  (hsa_amd_sdma_engine_id_t)(1u << dma_engine), true)
            : hsa_amd_memory_async_copy(host_dst, dma_cpu, src, dma_gpu, bytes, 1, &dma_dep, dma_done);
    if (s != HSA_STATUS_SUCCESS) {
        const char *m = "?";
        hsa_status_string(s, &m);
        std::string e2;
        (void)host_wait(e2);  // the stream's kernels still own the buffers
        err = std::string("code-stream copy: hsa_amd_memory_async_copy: ") + m;
        return false;
    }
    waits++;
    // in slices, never unbounded: the copy waits for k_release_dma, which
    // never runs if an earlier launch on the stream failed (host_wait.h)
    hipStream_t st = stream;
    const bool ok = jp2hip::wait_bounded(
        [&](uint64_t ns) { return poll_signal(dma_done, ns); },
        [st](std::string &why) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) return jp2hip::StreamState::Drained;
            if (q == hipErrorNotReady) return jp2hip::StreamState::Running;
            why = hipGetErrorString(q);
            return jp2hip::StreamState::Failed;
        },
        mono_ns, kWaitSliceNs, kDrainedGraceNs, "code-stream copy", err);
    if (!ok) {
        // the copy may still be queued behind its gate, holding both
        // signals: leave them to it (a failure path; a few bytes) and give
        // the next encode fresh ones, so a late release cannot complete a
        // wait that belongs to another copy
        dma_dep.handle = 0;
        dma_done.handle = 0;
        dma_ok = false;
    }
    return ok;
}
T2Args GpuEncoder::t2_args(const Plan &plan) const {
    T2Args a;
    std::memset(&a, 0, sizeof a);
    a.prec = (const PrecDesc *)t2prec.ptr;
    a.nprec = t2_nprec;
    a.tps = (const TpDesc *)t2tp.ptr;
    a.ntp = t2_ntp;
    a.blocks = (const BlockDesc *)blocks.ptr;
    a.P = (const uint8_t *)P.ptr;
    a.nl = (uint8_t *)nl.ptr;
    a.lrate = (int32_t *)lrate.ptr;
    a.nhull = (const uint8_t *)nhull.ptr;
    a.hpass = (const uint8_t *)hpass.ptr;
    a.npasses = (const uint8_t *)npasses.ptr;
    a.hkey = (const uint64_t *)hkey.ptr;
    a.K = (const uint64_t *)thr.ptr;
    a.grp_b0 = (const int32_t *)grptab.ptr;
    a.ngroups = plan.ngroups();
    a.rates = (const int32_t *)rates.ptr;
    a.lossless = plan.rc.rate_bpp <= 0.0;
    a.L = plan.rc.layers;
    a.sop = plan.rc.sop;
    a.eph = plan.rc.eph;
    a.plt = plan.rc.plt;
    a.tt = (uint32_t *)t2tt.ptr;
    a.lblock = (int8_t *)t2lblock.ptr;
    a.incl = (int8_t *)t2incl.ptr;
    a.pk_len = (uint32_t *)t2pklen.ptr;
    a.tp_len = (uint32_t *)t2tplen.ptr;
    a.tp_hdr = (uint32_t *)t2tphdr.ptr;
    a.tp_off = (uint64_t *)t2tpoff.ptr;
    a.pk_off = (uint64_t *)t2pkoff.ptr;
    a.blkdst = (uint64_t *)t2blkdst.ptr;
    a.out = (uint8_t *)t2out.ptr;
    return a;
}

bool GpuEncoder::t2_load(const Plan &plan, const T2Tables &T, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    const int nb = (int)plan.blocks.size();
    const int L = plan.rc.layers;
    t2_nprec = (int)T.prec.size();
    t2_ntp = (int)T.tp.size();
    // k_t2_wave (else the serial k_t2_code + k_apply)
    int max_mb = 0;
    for (const BlockDesc &bd : plan.blocks) max_mb = std::max(max_mb, (int)bd.Mb);
    t2_wave = T.max_prec_blocks <= 64 && max_mb <= kWaveMaxMb;
    const size_t npk = (size_t)t2_nprec * L;
    if (!ensure<PrecDesc>(t2prec, T.prec.size(), err) || !ensure<TpDesc>(t2tp, T.tp.size(), err) ||
        !ensure<uint32_t>(t2tt, (size_t)T.tt_nodes, err) || !ensure<int8_t>(t2lblock, nb, err) ||
        !ensure<int8_t>(t2incl, nb, err) || !ensure<uint32_t>(t2pklen, npk, err) ||
        !ensure<uint64_t>(t2pkoff, npk, err) || !ensure<uint32_t>(t2tplen, T.tp.size(), err) ||
        !ensure<uint32_t>(t2tphdr, T.tp.size(), err) || !ensure<uint64_t>(t2tpoff, T.tp.size(), err) ||
        !ensure<uint64_t>(t2blkdst, (size_t)nb * L, err) || !ensure<T2Summary>(t2sum, 1, err))
        return false;
    if (!h_sum) HIPCHECK(hipHostMalloc((void **)&h_sum, sizeof(T2Summary), hipHostMallocDefault));
    if (!t2ticket.ptr) {  // k_t2_wave<false>'s arrival counter: zero once, left zero by every launch
        if (!ensure<uint32_t>(t2ticket, 1, err)) return false;
        HIPCHECK(hipMemsetAsync(t2ticket.ptr, 0, sizeof(uint32_t), stream));
    }
    if (plan.gen && plan.gen == t2_gen) return true;  // resident (same plan, same tables)
    t2_gen = 0;
    if (!h2d(t2prec.ptr, T.prec.data(), sizeof(PrecDesc) * T.prec.size(), err) ||
        !h2d(t2tp.ptr, T.tp.data(), sizeof(TpDesc) * T.tp.size(), err))
        return false;
    t2_gen = plan.gen;
    return true;
}

void GpuEncoder::t2_size_launch(const Plan &plan, bool with_kc, const int *halt, RateState *rs,
                                RateState *out_rs) {
    const int nb = (int)plan.blocks.size();
    T2Args a = t2_args(plan);
    a.halt = halt;
    RateStepArgs ra;
    ra.rs = rs;
    ra.budget = (int64_t *)budget.ptr;
    ra.out_rs = out_rs;
    ra.out_sum = out_rs ? (T2Summary *)(out_rs + 1) : nullptr;
#ifndef JP2HIP_REPEAT_STAGE
#define JP2HIP_REPEAT_STAGE 0  // stage-cost experiments only (kernels.hip)
#endif
    T2TotalArgs ta;
    ta.nblocks = nb;
    ta.lengths = (const int32_t *)lengths.ptr;
    ta.npasses = (const uint8_t *)npasses.ptr;
    ta.pmin = (const uint8_t *)pmin.ptr;
    ta.t1err = (const int *)this->err.ptr;
    ta.pool_used = mqspan.ptr ? (const unsigned long long *)mqspan.ptr + 2 : nullptr;
    ta.kc = with_kc ? (const uint64_t *)thr.ptr + (size_t)plan.ngroups() * kMaxLayers : (const uint64_t *)nullptr;
    ta.ngroups = plan.ngroups();
    ta.acc = (const unsigned long long *)ordkey.ptr;
    ta.sum = (T2Summary *)t2sum.ptr;
    ta.rate = ra;
    ta.ticket = nullptr;
    for (int rep_ = 0; rep_ < (JP2HIP_REPEAT_STAGE == 5 ? 2 : 1); rep_++) {
        if (t2_nprec && t2_wave) {
            // the totals run in the last workgroup to finish (no k_t2_total launch)
            ta.ticket = (uint32_t *)t2ticket.ptr;
            hipLaunchKernelGGL(k_t2_wave<false>, dim3((t2_nprec + kT2Waves - 1) / kT2Waves), dim3(64 * kT2Waves),
                               kT2Waves * t2_lane_bytes(a.L), stream, a, ta);
        } else {
            ta.ticket = nullptr;
            if (t2_nprec) hipLaunchKernelGGL(k_t2_code<false>, dim3((t2_nprec + 63) / 64), dim3(64), 0, stream, a);
            hipLaunchKernelGGL(k_t2_total, dim3(1), dim3(kTotThreads), 0, stream, a, ta);
        }
    }
}

bool GpuEncoder::t2_size(const Plan &plan, bool with_kc, bool profile, StageTimes &st, T2Summary &sum,
                         std::string &err) {
    HIPCHECK(hipSetDevice(device));
    HIPCHECK(hipEventRecord(ev[8], stream));
    t2_size_launch(plan, with_kc, nullptr);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(h_sum, t2sum.ptr, sizeof(T2Summary), hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipEventRecord(ev[9], stream));
    if (!host_wait(err)) return false;
    sum = *h_sum;
    if (profile) {
        float t;
        HIPCHECK(hipEventElapsedTime(&t, ev[6], ev[7]));
        st.pcrd += t;
        HIPCHECK(hipEventElapsedTime(&t, ev[8], ev[9]));
        st.t2 += t;
    }
    return true;
}

bool GpuEncoder::t2_reserve(uint64_t part_bytes, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    return ensure<uint8_t>(t2out, part_bytes, err);
}

bool GpuEncoder::t2_emit(const Plan &plan, uint64_t base, uint64_t part_bytes, uint8_t *host_dst, bool profile,
                         StageTimes &st, std::string &err) {
    HIPCHECK(hipSetDevice(device));
    const int nb = (int)plan.blocks.size();
    if (!ensure<uint8_t>(t2out, base + part_bytes, err)) return false;
    T2Args a = t2_args(plan);
    a.base = base;
    HIPCHECK(hipEventRecord(ev[8], stream));
    if (t2_ntp) hipLaunchKernelGGL(k_t2_tp_emit, dim3((t2_ntp + 63) / 64), dim3(64), 0, stream, a);
    if (t2_nprec && t2_wave)
        hipLaunchKernelGGL(k_t2_wave<true>, dim3((t2_nprec + kT2Waves - 1) / kT2Waves), dim3(64 * kT2Waves),
                           kT2Waves * t2_lane_bytes(a.L), stream, a, T2TotalArgs{});
    else if (t2_nprec)
        hipLaunchKernelGGL(k_t2_code<true>, dim3((t2_nprec + 63) / 64), dim3(64), 0, stream, a);
    if (nb) hipLaunchKernelGGL(k_t2_copy, dim3((nb + 3) / 4), dim3(256), 0, stream, a, nb, (const uint8_t *)t1out.ptr);
    HIPCHECK(hipGetLastError());
    // host_dst is pinned (api.cpp out_alloc)
#if defined(JP2HIP_DIAG_NO_D2H)  // diagnostic builds only: the code-stream never leaves the GPU (output invalid)
    HIPCHECK(hipEventRecord(ev[9], stream));
    if (!host_wait(err)) return false;
    (void)host_dst;
#elif !defined(JP2HIP_D2H_BLIT)
    if (part_bytes) {
        // on a DMA engine, released by the stream (dma_to_host): no blit
        // kernel competes with the other contexts' kernels for CUs
        if (!dma_to_host(host_dst, (const uint8_t *)t2out.ptr + base, part_bytes, err)) return false;
        HIPCHECK(hipEventRecord(ev[9], stream));
        if (profile && !host_wait(err)) return false;  // (the events below must be complete)
    } else {
        HIPCHECK(hipEventRecord(ev[9], stream));
        if (!host_wait(err)) return false;
    }
#else  // A/B builds: the HIP runtime's copy (a blit kernel for pinned memory)
    if (part_bytes)
        HIPCHECK(hipMemcpyAsync(host_dst, (const uint8_t *)t2out.ptr + base, part_bytes, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipEventRecord(ev[9], stream));
    if (!host_wait(err)) return false;
#endif
    if (profile) {
        float t;
        HIPCHECK(hipEventElapsedTime(&t, ev[8], ev[9]));
        st.d2h += t;
    }
    return true;
}

}  // namespace jp2hip
