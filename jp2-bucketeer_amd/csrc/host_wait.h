// Bounded host waits on a completion that a device stream triggers (VERDICT
// r5 item 6). The code-stream D2H is an SDMA copy gated on a signal that the
// stream's last kernel releases (t2_device.hip dma_to_host). If that kernel
// never runs -- an earlier launch on the stream failed -- an unbounded wait
// on the copy's completion signal would block the caller forever, and the
// converter contract (every failure an IOException, AbstractConverter.java:
// 33-35) needs an error instead. So the wait runs in slices; between slices
// it asks the stream for its state:
//   - the stream failed            -> fail at once with the stream's error;
//   - the stream drained (every kernel done, the gate released) but the
//     copy still has not signalled after `drained_grace_ns` -> fail;
//   - the stream is still running  -> keep waiting: a long encode (a C5-class
//     image) is not an error.
// No HIP or HSA types here, so the loop is unit-tested on the CPU
// (tests/host/test_host_wait.cpp).
#pragma once

#include <cstdint>
#include <string>

namespace jp2hip {

enum class StreamState { Running, Drained, Failed };

enum class SliceResult { Done, Pending, Error };

// poll(slice_ns) -> SliceResult: waits at most about slice_ns for the
//   completion; Error when the completion itself reports a failure.
// state(why) -> StreamState: the stream's state; on Failed, `why` says why.
// now_ns() -> monotonic nanoseconds.
template <class Poll, class State, class Clock>
bool wait_bounded(Poll &&poll, State &&state, Clock &&now_ns, uint64_t slice_ns, uint64_t drained_grace_ns,
                  const char *what, std::string &err) {
    uint64_t drained_at = 0;
    bool drained = false;
    for (;;) {
        const SliceResult r = poll(slice_ns);
        if (r == SliceResult::Done) return true;
        if (r == SliceResult::Error) {
            err = std::string(what) + " failed (the copy engine reported an error)";
            return false;
        }
        std::string why;
        const StreamState s = state(why);
        if (s == StreamState::Failed) {
            err = std::string(what) + " abandoned: the stream failed before releasing it: " + why;
            return false;
        }
        if (s == StreamState::Drained) {
            const uint64_t t = now_ns();
            if (!drained) {
                drained = true;
                drained_at = t;
            } else if (t - drained_at > drained_grace_ns) {
                err = std::string(what) + " timed out: the stream drained but the copy never completed";
                return false;
            }
        } else {
            drained = false;
        }
    }
}

}  // namespace jp2hip
