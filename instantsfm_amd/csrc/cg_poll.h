// Host poll policy of the two-level CG (ba_kernels.hip run_solve): no stream sync inside the CG.  The lead workgroup
// of k_tl_pc publishes {iterations started, status} into host-mapped memory; the host keeps about `ahead` iterations
// queued, one at a time, and stops when the status word turns non-zero.  Plain C++ (no HIP types) so the policy,
// including its deadline, is unit-tested on the CPU (tests/test_cg_poll.py builds tests/cpp/cg_poll_test.cpp).
//
// Deadline: if neither the progress word nor the status changes for `stall_s` seconds of wall clock, the poll gives up
// (CgPoll::kStalled) instead of spinning forever on a CG launch that never publishes (a hung kernel, or a fault that
// does not surface as a stream error).  A live CG iteration takes ~10-20 us, so any stall of seconds is a failure.
// Multi-rank, the stall clock only starts once the work queued in front of the CG (the cross-rank exchange) has
// completed; that gate has its own, longer deadline `gate_s` (a peer that died or never sends its exchange would
// otherwise keep the gate shut forever): past it the poll returns CgPoll::kGateStalled.
#pragma once
#include <chrono>
#include <cstdlib>
#include <string>

namespace insfm {

struct CgPoll {
    enum Result { kDone = 0, kDrained = 1, kEnqueueError = -1, kStreamError = -2, kStalled = -3, kGateStalled = -4 };
    int enq = 0;            // iterations enqueued so far
    int last_reached = 0;   // last progress word seen
    long spins = 0;
    double stalled_s = 0.0; // wall-clock seconds without progress when the poll stopped
    int extra_ahead = 0;    // the caller may raise it (e.g. while it issues other work from pause()) to keep more queued
};

// Default stall limit (seconds); the environment variable INSFM_CG_STALL_S overrides it.
inline double cg_stall_limit_s(const char* env_value) {
    if (env_value && *env_value) {
        char* end = nullptr;
        const double v = std::strtod(env_value, &end);
        if (end != env_value && v > 0.0) return v;
    }
    return 10.0;
}

// Deadline of the multi-rank gate (the exchange in front of the CG): six stall limits.
inline double cg_gate_limit_s(double stall_s) { return 6.0 * stall_s; }

// status():  the published status word (0 running, non-zero finished)
// reached(): the published count of iterations started
// enqueue(from, to) -> int: launch iterations [from, to); non-zero = error (returned as kEnqueueError, code in *rc)
// query() -> int: 0 = stream drained, 1 = still running, negative = stream error
// now() -> double seconds (monotonic)
// pause(): a CPU relax hint
// started(): whether the work queued in front of the CG has completed; until it has, the deadline clock does not run
//   (multi-rank: the first CG launch waits for the cross-rank exchange, i.e. for the slowest peer, which is not a
//   stall of this device); it must open within gate_s seconds of the poll's start
template <class Status, class Reached, class Enqueue, class Query, class Now, class Pause, class Started>
int cg_poll(CgPoll& s, int limit, int ahead, double stall_s, double gate_s, Status status, Reached reached,
            Enqueue enqueue, Query query, Now now, Pause pause, Started started, int* rc) {
    const double t_start = now();
    double t_progress = t_start;
    bool live = false;
    for (;;) {
        if (status() != 0) return CgPoll::kDone;
        const int r = reached();
        if (r != s.last_reached) {
            s.last_reached = r;
            t_progress = now();
        }
        if (s.enq < limit && r >= s.enq - ahead - s.extra_ahead) {
            const int to = s.enq + 1 < limit ? s.enq + 1 : limit;
            if ((*rc = enqueue(s.enq, to)) != 0) return CgPoll::kEnqueueError;
            s.enq = to;
            continue;
        }
        if ((++s.spins & 255) == 0) {
            const int q = query();
            if (q == 0) {  // drained: everything enqueued has run
                if (status() != 0) return CgPoll::kDone;
                if (s.enq >= limit) return CgPoll::kDrained;
                const int to = s.enq + 8 < limit ? s.enq + 8 : limit;
                if ((*rc = enqueue(s.enq, to)) != 0) return CgPoll::kEnqueueError;
                s.enq = to;
                t_progress = now();
                continue;
            }
            if (q < 0) return CgPoll::kStreamError;
            if (!live) {
                live = started();
                if (!live) {
                    t_progress = now();
                    if (t_progress - t_start > gate_s) {
                        s.stalled_s = t_progress - t_start;
                        return CgPoll::kGateStalled;
                    }
                }
            }
            const double dt = now() - t_progress;
            if (dt > stall_s) {
                s.stalled_s = dt;
                return CgPoll::kStalled;
            }
        }
        pause();
    }
}

template <class Status, class Reached, class Enqueue, class Query, class Now, class Pause>
int cg_poll(CgPoll& s, int limit, int ahead, double stall_s, Status status, Reached reached, Enqueue enqueue,
            Query query, Now now, Pause pause, int* rc) {
    return cg_poll(s, limit, ahead, stall_s, stall_s, status, reached, enqueue, query, now, pause, [] { return true; },
                   rc);
}

inline double wall_seconds() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace insfm
