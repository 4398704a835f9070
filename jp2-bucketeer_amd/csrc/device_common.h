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

__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        int lo = __shfl_xor((int)(uint32_t)v, o, 64);
        int hi = __shfl_xor((int)(uint32_t)((uint64_t)v >> 32), o, 64);
        v += (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
    }
    return v;
}


}  // namespace jp2hip
