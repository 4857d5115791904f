"""Examples run end-to-end (BASELINE config #1: minGPT-small DP world_size=2 on CPU/gloo)."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_mingpt_dp2_cpu_gloo(tmp_path):
    snap = tmp_path / "snap.pt"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29633", os.path.join(ROOT, "examples/mingpt/main.py"),
           "--cpu", "--max_iters", "40", "--max_epochs", "1", "--snapshot_path", str(snap)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    m = re.search(r"final train loss ([0-9.]+) val loss ([0-9.]+)", out.stdout)
    assert m, out.stdout[-2000:]
    assert float(m.group(1)) < 2.5  # char vocab ~ 20: ln(20)=3.0 at init
