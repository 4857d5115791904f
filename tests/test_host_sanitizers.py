"""Host-code sanitizers (SURVEY.md §5.2 "optional -fsanitize=address builds"): the
launch planning and validation code of the HIP kernels (csrc/wgrad_gemm.hip tail split,
csrc/flash_attn.hip dK/dV split, csrc/rmsnorm.hip) compiled with
``-Xarch_host -fsanitize=address,undefined`` -- host only: GPU ASan is not available
on this fleet -- into tests/native/host_checks.cpp and run on the CPU.  Every entry
point it calls returns before a kernel launch, so no GPU is needed."""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_host_launch_planning_under_asan_ubsan(tmp_path):
    exe = tmp_path / "host_checks"
    san = []
    for s in ("-fsanitize=address", "-fsanitize=undefined", "-fno-sanitize-recover=all"):
        san += ["-Xarch_host", s]
    # device code at the shipped -O3: the hand-placed buffer descriptors of csrc/wgrad4.hip need
    # the uniformity analysis -O1 skips (only host code is sanitized and run here)
    cmd = [HIPCC, "--offload-arch=gfx950", "-O1", "-Xarch_device", "-O3", "-g", "-std=c++17", *san,
           f"-I{ROOT / 'csrc'}",
           str(ROOT / "csrc/wgrad_gemm.hip"), str(ROOT / "csrc/wgrad4.hip"), str(ROOT / "csrc/flash_attn.hip"), str(ROOT / "csrc/rmsnorm.hip"),
           str(ROOT / "tests/native/host_checks.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
