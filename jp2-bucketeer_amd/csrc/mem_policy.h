// A context's device-memory decisions, as pure functions (api.cpp EncodeEnd
// uses them; tests/host/test_mem_policy.cpp checks them on the CPU).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace jp2hip {

constexpr size_t kNeedHistory = 8;                   // encodes the usual image is taken over
constexpr size_t kReleaseSlack = (size_t)256 << 20;  // bytes above twice the usual

// Record what one encode needed (the last kNeedHistory are kept).
inline void record_need(std::vector<size_t> &needs, size_t need) {
    if (!need) return;
    needs.push_back(need);
    if (needs.size() > kNeedHistory) needs.erase(needs.begin());
}

// The bytes a context may keep after an encode (`needs` ends with that
// encode's): the explicit soft limit if one is set (> 0), else twice the
// larger of the recent needs' median and the previous encode's need, plus
// kReleaseSlack; SIZE_MAX when there is nothing to go by.  So a lone outsized
// image is released after it, and a lasting shift to larger images costs one
// release, not one per encode until the median catches up.
inline size_t keep_limit(const std::vector<size_t> &needs, int64_t soft) {
    if (soft > 0) return (size_t)soft;
    if (needs.empty()) return SIZE_MAX;
    std::vector<size_t> v = needs;
    std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
    const size_t prev = needs.size() >= 2 ? needs[needs.size() - 2] : 0;
    return 2 * std::max(v[v.size() / 2], prev) + kReleaseSlack;
}

}  // namespace jp2hip
