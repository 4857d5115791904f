"""scripts/run_dist_test.py (collective smoke tests of every dist wrapper) under
torch.distributed.run with gloo, world size 2 and 4, on the CPU."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4])
def test_run_dist_test_gloo(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "scripts", "run_dist_test.py"), "--backend", "gloo"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "ALL 17 PASSED" in r.stdout, r.stdout[-4000:]
