"""The persistent register-resident CG (ba_cgp.h k_tl_cgp) against the launch-per-iteration two-level CG.

Both run the same pipelined two-level recurrence (oracle/ba_oracle.c ora_pcg) in non-deterministic mode (per-cluster
atomic partial sums); they differ only in the summation order inside S~ m, so LM trajectories agree to rounding:
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


def run(diag):
    env = dict(os.environ, INSFM_DIAG=diag)
    p = subprocess.run([sys.executable, os.path.join(REPO, "tools", "cgp_check.py"), "--scenes", "small,fine,config2",
                        "--steps", "4"], capture_output=True, text=True, timeout=170, env=env, cwd=REPO)
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
