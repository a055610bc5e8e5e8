// CPU unit test of the two-level CG host poll policy (instantsfm_amd/csrc/cg_poll.h): a simulated device drives the
// progress / status words; prints one line per case, checked by tests/test_cg_poll.py.
#include <cstdio>

#include "../../instantsfm_amd/csrc/cg_poll.h"

using namespace insfm;

struct FakeDevice {
    int reached = 0, status = 0, converge_at = -1, enqueued = 0;
    bool hung = false;
    int stream_error_after = -1, enqueue_error_at = -1;
    long polls = 0;
    // the device starts one queued iteration every 3 polls unless hung
    void tick() {
        ++polls;
        if (hung || polls % 3) return;
        if (reached < enqueued) {
            ++reached;
            if (converge_at >= 0 && reached >= converge_at) status = 1;
        }
    }
};

static int run(FakeDevice& d, int limit, int ahead, double stall_s, CgPoll& s) {
    int rc = 0;
    double fake_t = 0.0;
    return cg_poll(
        s, limit, ahead, stall_s, [&] { d.tick(); return d.status; }, [&] { return d.reached; },
        [&](int from, int to) {
            if (d.enqueue_error_at >= 0 && to > d.enqueue_error_at) return -7;
            d.enqueued = to;
            (void)from;
            return 0;
        },
        [&] {
            if (d.stream_error_after >= 0 && d.polls > d.stream_error_after) return -1;
            return d.reached >= d.enqueued ? 0 : 1;
        },
        [&] { fake_t += 1e-4; return fake_t; }, [] {}, &rc) == CgPoll::kEnqueueError ? 1000 + rc : 0;
}

int main() {
    {   // converges at 30: done, never more than `ahead` + 1 queued beyond what the device started
        FakeDevice d; d.converge_at = 30; CgPoll s;
        int rc = 0;
        double fake_t = 0.0;
        int maxq = 0;
        const int r = cg_poll(
            s, 502, 2, 10.0, [&] { d.tick(); return d.status; }, [&] { return d.reached; },
            [&](int, int to) { d.enqueued = to; if (to - d.reached > maxq) maxq = to - d.reached; return 0; },
            [&] { return d.reached >= d.enqueued ? 0 : 1; }, [&] { fake_t += 1e-4; return fake_t; }, [] {}, &rc);
        std::printf("converge result=%d reached=%d enq=%d maxq=%d\n", r, d.reached, s.enq, maxq);
    }
    {   // hung device: no progress ever -> stalled after the limit, not an endless spin
        FakeDevice d; d.hung = true; CgPoll s; s.enq = 4; d.enqueued = 4;
        int rc = 0;
        double fake_t = 0.0;
        const int r = cg_poll(
            s, 502, 2, 0.5, [&] { d.tick(); return d.status; }, [&] { return d.reached; },
            [&](int, int to) { d.enqueued = to; return 0; }, [&] { return 1; },
            [&] { fake_t += 1e-4; return fake_t; }, [] {}, &rc);
        std::printf("hung result=%d stalled_s=%.3f enq=%d\n", r, s.stalled_s, s.enq);
    }
    {   // gated: the work in front of the CG (a peer's exchange) completes only after 2 s of fake time; the deadline
        // (0.5 s) counts from then on, so the poll stalls ~0.5 s after the gate opened, not 0.5 s after the start
        FakeDevice d; d.hung = true; CgPoll s; s.enq = 4; d.enqueued = 4;
        int rc = 0;
        double fake_t = 0.0, opened = -1.0;
        const int r = cg_poll(
            s, 502, 2, 0.5, 3.0, [&] { d.tick(); return d.status; }, [&] { return d.reached; },
            [&](int, int to) { d.enqueued = to; return 0; }, [&] { return 1; },
            [&] { fake_t += 1e-4; return fake_t; }, [] {},
            [&] { const bool o = fake_t >= 2.0; if (o && opened < 0) opened = fake_t; return o; }, &rc);
        std::printf("gated result=%d stalled_s=%.3f end=%.3f opened=%.3f\n", r, s.stalled_s, fake_t, opened);
    }
    {   // gate never opens (a peer died before its exchange): the gate deadline (3 s) ends the poll with kGateStalled
        FakeDevice d; d.hung = true; CgPoll s; s.enq = 4; d.enqueued = 4;
        int rc = 0;
        double fake_t = 0.0;
        const int r = cg_poll(
            s, 502, 2, 0.5, 3.0, [&] { d.tick(); return d.status; }, [&] { return d.reached; },
            [&](int, int to) { d.enqueued = to; return 0; }, [&] { return 1; },
            [&] { fake_t += 1e-4; return fake_t; }, [] {}, [] { return false; }, &rc);
        std::printf("gate_never result=%d stalled_s=%.3f end=%.3f\n", r, s.stalled_s, fake_t);
    }
    {   // status never set, device drains everything: stops at the launch limit
        FakeDevice d; CgPoll s;
        const int r = [&] {
            int rc = 0; double t = 0.0;
            return cg_poll(s, 40, 2, 10.0, [&] { d.tick(); return d.status; }, [&] { return d.reached; },
                           [&](int, int to) { d.enqueued = to; return 0; },
                           [&] { return d.reached >= d.enqueued ? 0 : 1; }, [&] { t += 1e-4; return t; }, [] {}, &rc);
        }();
        std::printf("drained result=%d reached=%d enq=%d\n", r, d.reached, s.enq);
    }
    {   // stream error surfaces
        FakeDevice d; d.hung = true; d.stream_error_after = 100; CgPoll s; s.enq = 4; d.enqueued = 4;
        const int r = [&] {
            int rc = 0; double t = 0.0;
            return cg_poll(s, 502, 2, 10.0, [&] { d.tick(); return d.status; }, [&] { return d.reached; },
                           [&](int, int to) { d.enqueued = to; return 0; },
                           [&] { return d.polls > d.stream_error_after ? -1 : 1; }, [&] { t += 1e-4; return t; },
                           [] {}, &rc);
        }();
        std::printf("stream_error result=%d\n", r);
    }
    {   // enqueue error code is passed through
        FakeDevice d; d.converge_at = 50; d.enqueue_error_at = 10; CgPoll s;
        const int code = run(d, 502, 2, 10.0, s);
        std::printf("enqueue_error code=%d\n", code);
    }
    std::printf("limit default=%.1f env=%.2f bad=%.1f gate=%.1f\n", cg_stall_limit_s(nullptr), cg_stall_limit_s("0.25"),
                cg_stall_limit_s("x"), cg_gate_limit_s(10.0));
    return 0;
}
