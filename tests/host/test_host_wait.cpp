// CPU unit test of jp2hip::wait_bounded (csrc/host_wait.h), the sliced wait
// dma_to_host uses for the code-stream copy.
#include "host_wait.h"

#include <cstdio>
#include <cstdlib>
#include <string>

using jp2hip::SliceResult;
using jp2hip::StreamState;

static int failures = 0;
#define CHECK(c)                                                     \
    do {                                                             \
        if (!(c)) {                                                  \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            failures++;                                              \
        }                                                            \
    } while (0)

struct Sim {
    int polls = 0, done_at = -1, error_at = -1, drain_at = -1, fail_at = -1;
    uint64_t clock = 0;
    SliceResult poll(uint64_t ns) {
        clock += ns;  // a slice that times out costs its length
        ++polls;
        if (error_at >= 0 && polls >= error_at) return SliceResult::Error;
        if (done_at >= 0 && polls >= done_at) return SliceResult::Done;
        return SliceResult::Pending;
    }
    StreamState state(std::string &why) {
        if (fail_at >= 0 && polls >= fail_at) {
            why = "an illegal memory access was encountered";
            return StreamState::Failed;
        }
        if (drain_at >= 0 && polls >= drain_at) return StreamState::Drained;
        return StreamState::Running;
    }
};

static bool run(Sim &s, std::string &err, uint64_t grace = 1000) {
    return jp2hip::wait_bounded([&](uint64_t ns) { return s.poll(ns); },
                                [&](std::string &why) { return s.state(why); }, [&] { return s.clock; }, 10, grace,
                                "code-stream copy", err);
}

int main() {
    {  // completes at once
        Sim s;
        s.done_at = 1;
        std::string e;
        CHECK(run(s, e) && s.polls == 1 && e.empty());
    }
    {  // a long encode: the stream runs for 100 000 slices, then the copy completes
        Sim s;
        s.done_at = 100000;
        std::string e;
        CHECK(run(s, e) && s.polls == 100000);
    }
    {  // the stream fails before the gate kernel runs: error at once, with its reason
        Sim s;
        s.fail_at = 3;
        std::string e;
        CHECK(!run(s, e) && s.polls == 3);
        CHECK(e.find("stream failed") != std::string::npos && e.find("illegal memory access") != std::string::npos);
    }
    {  // drained but the copy never signals: fails after the grace period, not before
        Sim s;
        s.drain_at = 5;
        std::string e;
        CHECK(!run(s, e, 1000));
        CHECK(e.find("timed out") != std::string::npos);
        CHECK(s.polls >= 5 + 100 && s.polls <= 5 + 102);  // 1000 ns of 10 ns slices after draining
    }
    {  // drained, then the copy completes inside the grace period
        Sim s;
        s.drain_at = 2;
        s.done_at = 50;
        std::string e;
        CHECK(run(s, e, 1000));
    }
    {  // the copy engine reports an error
        Sim s;
        s.error_at = 4;
        std::string e;
        CHECK(!run(s, e) && e.find("copy engine reported an error") != std::string::npos);
    }
    if (failures) return 1;
    std::printf("HOST WAIT OK\n");
    return 0;
}
