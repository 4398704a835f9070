// split.cpp -- exact global PCRD thresholds for a tile-split encode
// (one oversized image, contiguous bands of tile rows per
// GPU).  Host-only: no device code, so the exchange is testable on CPU.
//
// Single-image rule (kernels.hip k_thresh, oracle/jp2_oracle.c
// select_threshold): walk the hull segments of every code-block in
// decreasing slope-key order and take whole equal-key groups while the
// running byte total fits the layer budget; the threshold K is the last key
// taken.  Equivalently, with S(k) = bytes of segments whose key >= k (monotone
// non-increasing), the included set is {key >= K'} for
//     K' = min { k : S(k) <= budget },
// since no key lies strictly between the last group taken and the next one.
// S(k) is a sum over ranks, so K' is found by bisection over the 64-bit key
// space with one all-reduce(sum) of `layers` int64 per step (64 steps, all
// layers at once).  Every rank sees the same sums, so every rank ends with
// the same K' and the split encode includes exactly the passes the
// single-GPU encode does.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "jp2hip.h"
#include "jp2hip_internal.h"

namespace {

// bytes of this rank's segments with key >= k (keys descending, cum inclusive)
int64_t bytes_at_least(const uint64_t *keys, const int64_t *cum, int64_t n, uint64_t k) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = lo + ((hi - lo) >> 1);
        if (keys[mid] >= k) lo = mid + 1;
        else hi = mid;
    }
    return lo ? cum[lo - 1] : 0;
}

}  // namespace

extern "C" {

void jp2hip_split_rows(int32_t height, int32_t tile_h, int32_t flush_period, int32_t rank, int32_t world,
                       int32_t *row0, int32_t *row1) {
    int tr0 = 0, tr1 = 0;
    if (tile_h > 0 && height > 0 && world > 0 && rank >= 0 && rank < world)
        jp2hip::split_tile_rows((height + tile_h - 1) / tile_h, tile_h, height, flush_period, rank, world, tr0, tr1);
    if (row0) *row0 = (int32_t)std::min<int64_t>(height, (int64_t)tr0 * tile_h);
    if (row1) *row1 = (int32_t)std::min<int64_t>(height, (int64_t)tr1 * tile_h);
}

int jp2hip_split_thresholds(const uint64_t *keys, const int64_t *cum, int64_t nseg, const int64_t *budgets,
                            int32_t layers, const jp2hip_split *split, uint64_t *K) {
    if (layers <= 0 || layers > 64 || !budgets || !K || (nseg > 0 && (!keys || !cum))) return -1;
    // positive finite doubles: bit patterns order like the values and stay
    // below 0x7FF0000000000000; one past that includes nothing
    const uint64_t kNone = 0x7FF0000000000001ull;
    std::vector<uint64_t> lo((size_t)layers, 0), hi((size_t)layers, kNone);
    std::vector<int64_t> v((size_t)layers);
    for (;;) {
        bool open = false;
        for (int l = 0; l < layers; l++) {
            const uint64_t mid = lo[l] + ((hi[l] - lo[l]) >> 1);
            v[l] = lo[l] < hi[l] ? bytes_at_least(keys, cum, nseg, mid) : 0;
            open = open || lo[l] < hi[l];
        }
        if (!open) break;  // identical on every rank: same sums, same bounds
        if (split && split->world > 1) {
            if (!split->allreduce_sum || split->allreduce_sum(split->user, v.data(), layers) != 0) return -2;
        }
        for (int l = 0; l < layers; l++) {
            if (lo[l] >= hi[l]) continue;
            const uint64_t mid = lo[l] + ((hi[l] - lo[l]) >> 1);
            if (v[l] <= budgets[l]) hi[l] = mid;
            else lo[l] = mid + 1;
        }
    }
    for (int l = 0; l < layers; l++) K[l] = lo[l];
    return 0;
}

}  // extern "C"
