"""CPU unit test of the two-level CG host poll policy (instantsfm_amd/csrc/cg_poll.h, used by ba_kernels.hip
run_solve): progress, convergence, the launch limit, stream errors, and the wall-clock stall deadline that turns a
CG launch that never publishes into INSFM_BA_EHIP instead of an endless spin."""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def poll_out(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("poll") / "cg_poll_test")
    subprocess.run([cxx, "-std=c++17", "-O1", "-Wall", "-Werror", "-o", exe,
                    os.path.join(REPO, "tests", "cpp", "cg_poll_test.cpp")], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=60).stdout
    return {ln.split()[0]: dict(re.findall(r"(\w+)=(-?[\d.]+)", ln)) for ln in out.splitlines()}


def test_converges_with_bounded_queue(poll_out):
    c = poll_out["converge"]
    assert int(c["result"]) == 0 and int(c["reached"]) == 30
    assert int(c["maxq"]) <= 3  # `ahead` (2) + the one being started


def test_hung_device_stalls_out(poll_out):
    h = poll_out["hung"]
    assert int(h["result"]) == -3
    assert 0.5 <= float(h["stalled_s"]) < 0.6


def test_drained_stops_at_limit(poll_out):
    d = poll_out["drained"]
    assert int(d["result"]) == 1 and int(d["enq"]) == 40 and int(d["reached"]) == 40


def test_stream_error_and_enqueue_error(poll_out):
    assert int(poll_out["stream_error"]["result"]) == -2
    assert int(poll_out["enqueue_error"]["code"]) == 1000 - 7


def test_stall_limit_env(poll_out):
    lim = poll_out["limit"]
    assert float(lim["default"]) == 10.0 and float(lim["env"]) == 0.25 and float(lim["bad"]) == 10.0
    assert float(lim["gate"]) == 60.0


def test_deadline_starts_after_the_gate(poll_out):
    """Multi-rank: the CG waits for the cross-rank exchange (the slowest peer); the stall clock starts only once the
    work queued in front of the CG has completed, so a peer that is seconds behind is not reported as a hung device."""
    g = poll_out["gated"]
    assert int(g["result"]) == -3
    assert float(g["opened"]) >= 2.0
    assert 0.5 <= float(g["stalled_s"]) < 0.6
    assert float(g["end"]) >= 2.5


def test_gate_that_never_opens_ends_the_poll(poll_out):
    """A peer that dies before its exchange keeps the multi-rank gate shut: the poll must still end (kGateStalled,
    -4) once the gate deadline passes, not spin forever with the stall clock held at zero."""
    g = poll_out["gate_never"]
    assert int(g["result"]) == -4
    assert 3.0 <= float(g["stalled_s"]) < 3.1
    assert 3.0 <= float(g["end"]) < 3.2
