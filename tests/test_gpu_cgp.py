"""The persistent register-resident CG (ba_cgp.h k_tl_cgp) against the launch-per-iteration two-level CG.

Both run the same pipelined two-level recurrence (oracle/ba_oracle.c ora_pcg) with the additive coarse correction
(precond 1: the launch path has no A-DEF2 form) in non-deterministic mode (per-cluster atomic partial sums); they differ only in the summation order inside S~ m, so LM trajectories agree to rounding:
losses within 1e-8 relative, PCG iteration counts within one per step.  INSFM_DIAG is read once per process, so each
path runs in its own process (tools/cgp_check.py).  The oracle parity of the path itself is test_gpu_parity.py's
test_solve_parity / test_step_parity (non-deterministic D = 8 cases run k_tl_cgp where it is eligible).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(diag, *extra, scenes="small,fine,config2"):
    env = dict(os.environ, INSFM_DIAG=diag)
    p = subprocess.run([sys.executable, os.path.join(REPO, "tools", "cgp_check.py"), "--scenes", scenes,
                        "--steps", "4", *extra], capture_output=True, text=True, timeout=170, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])["scenes"]


def test_cgp_matches_launch_path():
    a, b = run(""), run("no_cgp")
    assert a["fine"]["nc"] * 9 > 512  # the coarse vector spans more than two LDS fills per thread
    for name in a:
        sa, sb = a[name], b[name]
        assert sa["D"] == 8
        assert not any(sa["failed"]) and not any(sb["failed"]), (name, sa, sb)
        # k_tl_cgp: one CG launch per solve (trial); the launch path: one per iteration and more
        assert sa["launches"] == sa["trials"], (name, sa)
        assert all(l > t for l, t in zip(sb["launches"], sb["trials"])), (name, sb)
        for k, (la, lb) in enumerate(zip(sa["losses"], sb["losses"])):
            assert abs(la - lb) <= 1e-8 * abs(lb), (name, k, la, lb)
        assert all(abs(x - y) <= 1 for x, y in zip(sa["iters"], sb["iters"])), (name, sa["iters"], sb["iters"])


def test_cgp_deterministic_variant():
    """deterministic=True runs the fixed-order k_tl_cgp (no atomics: every workgroup run stores its partials in a
    parity buffer before the grid barrier, and after it every workgroup sums each cluster's runs itself in run order):
    two runs of each scene are bitwise equal, one launch per solve, and the launch path's deterministic CG agrees to
    rounding (losses 1e-8, PCG iterations within one per step)."""
    a = run("", "--det", "--repeat", "2", scenes="small,config2")
    b = run("no_cgp", "--det", scenes="small,config2")
    for name in ("small", "config2"):
        s1, s2, sb = a[name], a[name + "#1"], b[name]
        assert s1["launches"] == s1["trials"], s1
        assert s1["losses_hex"] == s2["losses_hex"] and s1["params_sha"] == s2["params_sha"], (s1, s2)
        for la, lb in zip(s1["losses"], sb["losses"]):
            assert abs(la - lb) <= 1e-8 * abs(lb), (name, la, lb)
        assert all(abs(x - y) <= 1 for x, y in zip(s1["iters"], sb["iters"])), (s1["iters"], sb["iters"])


def test_cgp_deterministic_adef2_bitwise():
    """the fixed-order A-DEF2 k_tl_cgp (path 5, the product default precond 2 in deterministic mode
    and on every rank of a multi-rank run) is bitwise reproducible run to run, one launch per solve, and agrees with
    the atomic A-DEF2 form (path 4) to rounding: losses 1e-8, PCG iterations within one per step."""
    a = run("", "--det", "--repeat", "2", "--precond", "2", scenes="small,config2")
    b = run("", "--precond", "2", scenes="small,config2")
    for name in ("small", "config2"):
        s1, s2, sb = a[name], a[name + "#1"], b[name]
        assert s1["path"] == 5 and sb["path"] == 4, (s1, sb)
        assert s1["launches"] == s1["trials"], s1
        assert s1["losses_hex"] == s2["losses_hex"] and s1["params_sha"] == s2["params_sha"], (s1, s2)
        assert not any(s1["failed"]) and not any(sb["failed"]), (s1, sb)
        for la, lb in zip(s1["losses"], sb["losses"]):
            assert abs(la - lb) <= 1e-8 * abs(lb), (name, la, lb)
        assert all(abs(x - y) <= 1 for x, y in zip(s1["iters"], sb["iters"])), (s1["iters"], sb["iters"])


def test_cgp_abort_falls_back_to_launch_path():
    """A k_tl_cgp whose grid barrier times out (INSFM_DIAG=cgp_fault: the process's first launch, the warm-up step's,
    loses a workgroup at iteration 2 as if another process held its CU) raises the abort word; every workgroup leaves
    without touching the CG vectors, the host repeats that solve on the launch path from the basis and keeps the
    handle there.  The run then follows the launch path's trajectory (losses 1e-9 against INSFM_DIAG=no_cgp)."""
    env = dict(os.environ, INSFM_DIAG="cgp_fault")
    p = subprocess.run([sys.executable, os.path.join(REPO, "tools", "cgp_check.py"), "--scenes", "config2", "--steps",
                        "4"], capture_output=True, text=True, timeout=170, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "grid barrier timed out" in p.stderr, p.stderr[-3000:]
    a = json.loads(p.stdout.strip().splitlines()[-1])["scenes"]["config2"]
    b = run("no_cgp", scenes="config2")["config2"]
    assert not any(a["failed"]), a
    assert all(l > t for l, t in zip(a["launches"], a["trials"])), a  # launch path after the abort
    for la, lb in zip(a["losses"], b["losses"]):
        assert abs(la - lb) <= 1e-9 * abs(lb), (la, lb)
