// CPU unit test of the release-after-encode rule (csrc/mem_policy.h).
#include "mem_policy.h"

#include <cstdio>

static int failures = 0;
#define CHECK(c)                                                     \
    do {                                                             \
        if (!(c)) {                                                  \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            failures++;                                              \
        }                                                            \
    } while (0)

int main() {
    using namespace jp2hip;
    const size_t GB = (size_t)1 << 30;
    std::vector<size_t> needs;
    CHECK(keep_limit(needs, 0) == SIZE_MAX);            // nothing to go by: keep
    CHECK(keep_limit(needs, 5 * (int64_t)GB) == 5 * GB);  // an explicit soft limit wins
    record_need(needs, 0);
    CHECK(needs.empty());  // a failed or empty encode records nothing
    // steady large masters: their own footprint is always kept
    for (int i = 0; i < 3; i++) record_need(needs, 17 * GB);
    CHECK(keep_limit(needs, 0) >= 17 * GB + 17 * GB / 8);
    // a C2 pool, then one C5-class master: released after it
    needs.clear();
    for (int i = 0; i < 3; i++) record_need(needs, 2 * GB);
    record_need(needs, 42 * GB);
    CHECK(keep_limit(needs, 0) == 4 * GB + kReleaseSlack);
    // a second one in a row is kept: a lasting shift costs one release
    record_need(needs, 42 * GB);
    CHECK(keep_limit(needs, 0) == 84 * GB + kReleaseSlack);
    // back to the small images: kept for one more encode, released after two
    record_need(needs, 2 * GB);
    CHECK(keep_limit(needs, 0) == 84 * GB + kReleaseSlack);
    record_need(needs, 2 * GB);
    CHECK(keep_limit(needs, 0) == 4 * GB + kReleaseSlack);
    // the history keeps the last 8 only: after 8 masters the pool is theirs
    for (int i = 0; i < 8; i++) record_need(needs, 42 * GB);
    CHECK(needs.size() == kNeedHistory);
    CHECK(keep_limit(needs, 0) == 84 * GB + kReleaseSlack);
    // half small, half large: the median is the upper middle, large kept
    needs.clear();
    for (int i = 0; i < 4; i++) {
        record_need(needs, 17 * GB);
        record_need(needs, 2 * GB);
    }
    CHECK(keep_limit(needs, 0) == 34 * GB + kReleaseSlack);
    if (failures) return 1;
    std::printf("MEM POLICY OK\n");
    return 0;
}
