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
