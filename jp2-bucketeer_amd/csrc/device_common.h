// device_common.h -- device helpers shared by the stage kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "jp2hip_internal.h"

namespace jp2hip {

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

// The same quantities in 32-bit arithmetic for planes q <= 14: |error| below
// plane q is < 2^(q+1) half-units (the residual 2(v mod 2^q) + 1 - 2^q once
// significant, 2v + 1 < 2^(q+1) before), so its square is < 2^30.
__device__ __forceinline__ uint32_t err_small(uint32_t v, int q, bool lossless) {
    const int32_t d = lossless ? 0 : 1;
    if ((v >> q) != 0) {
        if (lossless && q == 0) return 0u;
        const int32_t e = 2 * (int32_t)(v & ((1u << q) - 1u)) + d - (1 << q);
        return (uint32_t)(e < 0 ? -e : e);
    }
    return 2u * v + (uint32_t)d;
}
__device__ __forceinline__ int64_t dist_gain_small(uint32_t v, int p, bool lossless) {  // p <= 13
    const uint32_t e1 = err_small(v, p + 1, lossless), e0 = err_small(v, p, lossless);
    return (int64_t)(e1 * e1) - (int64_t)(e0 * e0);
}

// Deadzone quantisation of one final DWT coefficient (Annex E.1; oracle
// quantise): the index min(floor(|x| / Delta), 2^Mb - 1) -- |x| for the
// reversible path -- with the coefficient's sign bit at bit `sbit` (15: the
// 16-bit plane, 31: the 32-bit one).  The sign of a zero index is stored as
// the coefficient had it and never coded.
// (The float product is non-negative, so the truncating conversion is the
// floor: one v_mul with the |x| source modifier and one v_cvt.)
template <bool REV>
__device__ __forceinline__ uint32_t quant_mag(int32_t x, float inv, uint32_t lim) {
    uint32_t m;
    if (REV) m = (uint32_t)abs(x);
    else m = (uint32_t)(__builtin_fabsf(__int_as_float(x)) * inv);
    return min(m, lim);
}
template <bool REV>
__device__ __forceinline__ uint32_t quant_sm(int32_t x, float inv, uint32_t lim, int sbit) {
    return quant_mag<REV>(x, inv, lim) | (((uint32_t)x >> 31) << sbit);
}

// Whole-wave lane shifts by DPP (wave_shr:1 / wave_shl:1, GFX9 family): a
// VALU move, not an LDS-crossbar ds_bpermute with its latency.  Lane 0
// (shr) / lane 63 (shl) receive 0.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) {  // lane i <- lane i-1
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t wave_shl1(uint32_t x) {  // lane i <- lane i+1
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, true);
}
__device__ __forceinline__ uint64_t wave_shr1(uint64_t x) {
    return ((uint64_t)wave_shr1((uint32_t)(x >> 32)) << 32) | wave_shr1((uint32_t)x);
}
__device__ __forceinline__ uint64_t wave_shl1(uint64_t x) {
    return ((uint64_t)wave_shl1((uint32_t)(x >> 32)) << 32) | wave_shl1((uint32_t)x);
}

// inclusive prefix sum over the 64 lanes of a wave (DPP row shifts, then the
// row_bcast15 / row_bcast31 steps across rows)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t n) {
    int v = (int)n;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
    return (uint32_t)v;
}
// OR over the wave (every lane), by the same DPP steps
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t n) {
    int v = (int)n;
    v |= __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
    v |= __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
    v |= __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
    v |= __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
    v |= __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
    v |= __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
    return (uint32_t)__builtin_amdgcn_readlane(v, 63);
}
// the wave's total (every lane), by the DPP scan and lane 63
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t n) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(n), 63);
}
// 64-bit total: the same scan on both halves, the carries of the low half
// added into the high one
__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
    uint64_t x = (uint64_t)v;
#define JP2HIP_SCAN64_STEP(ctl, rm)                                                                            \
    {                                                                                                          \
        const uint32_t lo_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, ctl, rm, 0xf, false);   \
        const uint32_t hi_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), ctl, rm, 0xf, false); \
        x += ((uint64_t)hi_ << 32) | lo_;                                                                      \
    }
    JP2HIP_SCAN64_STEP(0x111, 0xf)
    JP2HIP_SCAN64_STEP(0x112, 0xf)
    JP2HIP_SCAN64_STEP(0x114, 0xf)
    JP2HIP_SCAN64_STEP(0x118, 0xf)
    JP2HIP_SCAN64_STEP(0x142, 0xa)
    JP2HIP_SCAN64_STEP(0x143, 0xc)
#undef JP2HIP_SCAN64_STEP
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
// exclusive scan of NT threads (every thread calls it);
// wsum: NT/64 + 1 words of LDS; `tot` = the workgroup's sum
template <int NT>
__device__ __forceinline__ uint32_t wg_excl_scan(uint32_t n, uint32_t *wsum, uint32_t &tot) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(n);
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t w = threadIdx.x < NT / 64 ? wsum[threadIdx.x] : 0u;
        const uint32_t wi = wave_incl_scan(w);
        if (threadIdx.x < NT / 64) wsum[threadIdx.x] = wi - w;
        if (threadIdx.x == NT / 64 - 1) wsum[NT / 64] = wi;
    }
    __syncthreads();
    const uint32_t ex = wsum[wv] + inc - n;
    tot = wsum[NT / 64];
    __syncthreads();  // wsum is reused by the next call
    return ex;
}
// 64-bit variants (shuffle steps; offsets that may pass 4 GiB)
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, o, 64);
        const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), o, 64);
        if (lane >= o) v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}
template <int NT>
__device__ __forceinline__ uint64_t wg_excl_scan64(uint64_t n, uint64_t *wsum, uint64_t &tot) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t inc = wave_incl_scan64(n);
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint64_t w = threadIdx.x < NT / 64 ? wsum[threadIdx.x] : 0ull;
        const uint64_t wi = wave_incl_scan64(w);
        if (threadIdx.x < NT / 64) wsum[threadIdx.x] = wi - w;
        if (threadIdx.x == NT / 64 - 1) wsum[NT / 64] = wi;
    }
    __syncthreads();
    const uint64_t ex = wsum[wv] + inc - n;
    tot = wsum[NT / 64];
    __syncthreads();
    return ex;
}

// The rate-control group of block b (Plan::grp_b0: ngroups + 1 ascending
// block indices): the last g with grp_b0[g] <= b
__device__ __forceinline__ int block_group(const int32_t *grp_b0, int ngroups, int b) {
    int lo = 0, hi = ngroups - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (grp_b0[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// --------------------------------------------------------------------------
// Device rate loop (RateState, jp2hip_internal.h): the same arithmetic as the
// oracle's loop (oracle_encode, rate_bpp > 0).  One step, after a tier-2
// sizing pass summarised in `sum`: stop when the code-stream fits the target
// (or after 8 iterations), else lower the budget.  Each step that runs also
// leaves the state and the summary it decided on in host-mapped memory
// (out_rs, out_sum): the host reads them after its wait, no copy launches.
// --------------------------------------------------------------------------
__device__ __forceinline__ void rate_budgets(const RateState &r, int L, int64_t *budget) {
    const int64_t b = r.budget < 0 ? 0 : r.budget;
    for (int l = 0; l < L; l++) budget[l] = b >> (L - 1 - l);
}
__device__ __forceinline__ void rate_step(RateState *rs, const T2Summary *sum, int L, int64_t *budget,
                                          RateState *out_rs, T2Summary *out_sum) {
    RateState r = *rs;
    if (r.halt) return;
    if (sum->err) {  // tier-1 overflow: the host reports it
        r.halt = 1;
    } else if (r.it == 0 && r.skip_target > 0 && sum->skipped && sum->t1_bytes < r.skip_target) {
        r.safety = 1;  // slope prediction's safety net: the host re-runs the front
        r.halt = 1;
    } else {
        r.iters++;
        r.cs_bytes = r.fixed + sum->part_bytes;
        if (r.cs_bytes <= r.target || r.it == 7) {
            r.halt = 1;
        } else {
            // exponential back-off + 1/16 of the overshoot + 64 B, as the oracle
            const int64_t over = r.cs_bytes - r.target;
            r.budget -= (over << r.it) + (over >> 4) + 64;
            if (r.budget < 0) r.budget = 0;
            r.it++;
            rate_budgets(r, L, budget);
        }
    }
    *rs = r;
    *out_rs = r;
    *out_sum = *sum;
}

// Files each block's coded planes in k_t1_cm3's per-depth work lists
// (T1ItemArgs, gpu_encoder.h); called by every thread of a thread-per-block
// kernel of NT threads (`valid` false past the last block).  The workgroup
// counts its entries per depth (a ballot per wave and depth), one lane per
// depth reserves the workgroup's run of each list with one atomic -- all
// depths' atomics in flight together, not one round trip per depth and wave
// -- and every block writes its entries at its rank inside the run.
struct ItemScratch {
    uint32_t cnt[16][64];  // [wave][depth] entries; then the wave's offset in the list
};
// bytes reserved per (block, plane) for the three passes' decisions:
// at most w*h coding decisions + w*h sign decisions + 3 per run-length column
// (each pass is padded to a 16-byte boundary; the MQ kernel prefetches one
// 16-byte chunk past the end of a pass)
__host__ __device__ __forceinline__ uint32_t plane_stream_cap(int w, int h) {
    return ((uint32_t)(11 * w * h) / 4 + 128 + 15) & ~15u;
}


// Also places each block's decision-stream slot: c coded planes x
// plane_stream_cap bytes, carved from the pool (a.pool_cap bytes) by one
// atomic per wave on a.pool_used, which ends at the bytes the encode
// needed.  A block that does not fit is coded as empty and sets
// kErrSlotPool; the host then grows the pool to a.pool_used and encodes
// again (GpuEncoder::run_front), so no output is ever made from a short pool.
template <int NT, typename ItemArgs>
__device__ __forceinline__ void emit_t1_items(const ItemArgs &a, int b, bool valid, int P, int pmin, ItemScratch &sc) {
    static_assert(NT % 64 == 0 && NT / 64 <= 16, "emit_t1_items: 64..1024 threads");
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t c = valid ? (uint32_t)(P - pmin) : 0u;
    {
        uint32_t need = 0;
        if (c) {
            const BlockDesc d = a.blocks[b];
            need = c * plane_stream_cap(d.w, d.h);
        }
        uint32_t x = need;  // inclusive scan over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
            if (lane >= o) x += y;
        }
        const uint32_t wtot = (uint32_t)__shfl((int)x, 63, 64);
        unsigned long long wbase = 0;
        if (lane == 63 && wtot) wbase = atomicAdd(a.pool_used, (unsigned long long)wtot);
        wbase = ((unsigned long long)(uint32_t)__shfl((int)(uint32_t)(wbase >> 32), 63, 64) << 32) |
                (uint32_t)__shfl((int)(uint32_t)wbase, 63, 64);
        const unsigned long long base = wbase + (x - need);
        if (c) {
            if (base + need > a.pool_cap) {
                c = 0;  // no room: coded as an empty block; the host re-encodes
                atomicOr(a.err, kErrSlotPool);
            } else {
                a.slot_off[b] = base;
            }
        }
    }
    if (valid) {
        a.acc[b] = (unsigned long long)c << 40;
        if (c == 0) {
            a.npasses[b] = 0;
            a.lengths[b] = 0;
        }
    }
    uint32_t cw = c;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cw = max(cw, (uint32_t)__shfl_xor((int)cw, o, 64));
    const int kw = min(__builtin_amdgcn_readfirstlane((int)cw), a.kmax);
    const uint64_t lt = (1ull << lane) - 1ull;
    // this wave's entries per depth (depths >= kw: none)
    for (int k = lane; k < 64; k += 64) sc.cnt[wv][k] = 0u;
    for (int k = 0; k < kw; k++) {
        const uint64_t m = __ballot(c > (uint32_t)k);
        if (lane == 0) sc.cnt[wv][k] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // lane k: depth k's run for the workgroup
        const int k = threadIdx.x;
        uint32_t tot = 0, wc[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) {
            wc[w] = sc.cnt[w][k];
            tot += wc[w];
        }
        uint32_t base = (tot && k < a.kmax) ? atomicAdd(&a.dfill[k], tot) : 0u;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            sc.cnt[w][k] = base;
            base += wc[w];
        }
    }
    __syncthreads();
    for (int k = 0; k < kw; k++) {
        const uint64_t m = __ballot(c > (uint32_t)k);
        if (c > (uint32_t)k) a.dlist[(size_t)k * a.nb + sc.cnt[wv][k] + (uint32_t)__popcll(m & lt)] = b;
    }
}

}  // namespace jp2hip
