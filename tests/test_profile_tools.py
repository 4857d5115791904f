"""The trace tools the round-6 profiles rest on (tools/rocpd_summary.py, tools/trace_overlap.py),
on a synthetic rocpd-style SQLite ``kernels`` table with known answers: step windows from the
AdamW launches, per-class milliseconds, busy union, and the side-stream interference sum."""
from __future__ import annotations

import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MS = 1_000_000  # ns


def _db(tmp_path, steps=4, period_ms=100):
    """Each step k at t = k * period: AdamW 0-4 ms (side stream); under it one forward GEMM
    of 3 ms (its clean length elsewhere is 1 ms); then three clean 1-ms GEMMs and a 2-ms
    flash forward back to back."""
    rows = []
    for k in range(steps):
        t = k * period_ms * MS
        rows.append(("void adamw_kernel<float, unsigned short>(float*)", t, t + 4 * MS))
        rows.append(("Custom_Cijk_Alik_Bljk_BBS_BH_MT256x256x64", t + MS // 2, t + MS // 2 + 3 * MS))
        for j in range(3):
            s = t + 10 * MS + j * MS
            rows.append(("Custom_Cijk_Alik_Bljk_BBS_BH_MT256x256x64", s, s + MS))
        rows.append(("void flash_fwd_kernel<128, true, 1>(AttnParams)", t + 13 * MS, t + 15 * MS))
    path = tmp_path / "run_results.db"
    c = sqlite3.connect(path)
    c.execute("create table kernels (name text, start integer, end integer)")
    c.executemany("insert into kernels values (?, ?, ?)", rows)
    c.commit()
    c.close()
    return str(path)


def _run(tool, *args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", tool), *args], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_rocpd_summary_windows_and_classes(tmp_path):
    db = _db(tmp_path)
    out = _run("rocpd_summary.py", db, "--steps", "2", "--csv", str(tmp_path / "k.csv"))
    head = out.splitlines()[0]
    assert "100.00 ms/step wall" in head  # window = end of AdamW group 1 .. end of group 3
    # per step in the window: GEMMs 3 + 3 x 1 = 6 ms, flash fwd 2 ms, AdamW 4 ms (next step's)
    assert any(line.split()[0] == "gemm_bf16(fwd+dgrad)" and abs(float(line.split()[1]) - 6.0) < 1e-6
               for line in out.splitlines()[1:])
    assert any(line.split()[0] == "flash_fwd" and abs(float(line.split()[1]) - 2.0) < 1e-6
               for line in out.splitlines()[1:])
    assert (tmp_path / "k.csv").read_text().startswith("Name,Class,CallsPerStep,MsPerStep,AvgUs")


def test_trace_overlap_prices_the_side_stream(tmp_path):
    db = _db(tmp_path)
    out = _run("trace_overlap.py", db, "--steps", "2")
    # the overlapped GEMM ran 3 ms against a 1-ms clean mean: 2 ms extra per step
    line = next(x for x in out.splitlines() if x.startswith("extra time of overlapped"))
    assert abs(float(line.split(":")[1].split()[0]) - 2.0) < 1e-6
    assert "side-stream (AdamW + grad-norm) busy 4.00 ms/step" in out
