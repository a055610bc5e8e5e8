"""Track-sharded multi-rank LM on the GPU (2 ranks sharing one MI355X through gloo) vs the single-GPU LM."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("extra", [["--small", "--steps", "5"], ["--config", "2", "--steps", "3"], ["--gp", "--steps", "6"]])
def test_two_ranks_match_single_gpu(extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(REPO, "tools", "dist_check.py"), "--backend", "gloo",
           "--same-device", *extra]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["loss_rel"] < 1e-9, out
    assert out["cams_rel"] < 1e-7 and out["points_rel"] < 1e-7, out
    assert out["cams_equal_across_ranks"], out
    assert abs(out["rmse"] - out["ref_rmse"]) < 1e-6, out
    if "scales_rel" in out:
        assert out["scales_rel"] < 1e-7, out
