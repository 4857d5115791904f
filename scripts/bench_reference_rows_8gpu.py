#!/usr/bin/env python3
"""Replay the reference's published 8-device table (the reference's
README.md:48-139 rows, driven there by scripts/benchmark_comprehensive.py:54-173 and
scripts/benchmark_moe.sh:44-50) on one MI355X node, row by row, with the SAME model,
parallel layout, micro-batch, gradient accumulation, sequence length and activation
checkpointing, and write one JSONL line per row with the reference's tok/s/GPU next
to ours.

Differences that make our rows do MORE work than the reference's (BASELINE.md caveat
flags, kept in each line): CP rows run real ring / all-gather attention ([CP]: the
reference's was chunk-local), SP rows run real sequence parallelism ([SP]), DP+GA
rows all-reduce and step ([GA]), EP rows back-propagate through the all-to-all
([EP]); our timing is the full step (clip + AdamW included).

  python scripts/bench_reference_rows_8gpu.py --list
  python scripts/bench_reference_rows_8gpu.py --gpus 8 --out gpurun_out/reference_rows_8gpu.jsonl
  python scripts/bench_reference_rows_8gpu.py --filter 'qwen3-8b' --dry-run
  python scripts/bench_reference_rows_8gpu.py --smoke --filter 'tp4-pp2|ep2-tp4'   # CPU/gloo, tiny models
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.realpath(__file__)))

# (model, layout, mbs, ga, seq, gc, reference tok/s/GPU, reference MFU %, flags, README line)
ROWS = [
    ("qwen3-0.6b", "dp8", 2, 2, 2048, False, 16422, 38.0, "GA", 48),
    ("qwen3-0.6b", "cp2-dp4", 1, 1, 4096, False, 9218, 26.4, "CP", 49),
    ("qwen3-0.6b", "sp-tp2-dp4", 2, 1, 2048, False, 8136, 18.8, "SP", 50),
    ("qwen3-0.6b", "tp2-dp4", 2, 1, 2048, False, 8035, 18.6, "", 51),
    ("qwen3-0.6b", "cp4-dp2", 1, 1, 8192, True, 6829, 27.1, "CP", 52),
    ("qwen3-0.6b", "tp2-cp2-dp2", 1, 1, 4096, False, 5340, 15.3, "CP", 53),
    ("qwen3-0.6b", "tp4-dp2", 2, 1, 2048, False, 4514, 10.4, "", 54),
    ("qwen3-1.7b", "dp8", 1, 2, 2048, True, 6792, 36.1, "GA", 60),
    ("qwen3-1.7b", "cp4-dp2", 1, 1, 8192, True, 5096, 35.5, "CP", 61),
    ("qwen3-1.7b", "cp2-dp4", 1, 1, 4096, True, 4891, 28.7, "CP", 62),
    ("qwen3-1.7b", "tp2-dp4", 1, 1, 2048, False, 3932, 20.9, "", 63),
    ("qwen3-1.7b", "sp-tp2-dp4", 1, 1, 2048, False, 3769, 20.0, "SP", 64),
    ("qwen3-1.7b", "tp4-dp2", 1, 1, 2048, False, 2440, 13.0, "", 65),
    ("qwen3-4b", "cp2-dp4", 1, 1, 4096, True, 2719, 35.8, "CP", 71),
    ("qwen3-4b", "dp8", 1, 1, 2048, True, 2706, 31.8, "", 72),
    ("qwen3-4b", "sp-tp2-dp4", 1, 1, 2048, True, 1994, 23.4, "SP", 73),
    ("qwen3-4b", "tp2-dp4", 1, 1, 2048, True, 1984, 23.3, "", 74),
    ("qwen3-4b", "tp2-cp2-dp2", 1, 1, 4096, True, 1952, 25.7, "CP", 75),
    ("qwen3-4b", "tp4-dp2", 1, 1, 2048, False, 1629, 19.1, "", 76),
    ("qwen3-8b", "tp2-cp2-dp2", 1, 1, 4096, True, 1406, 31.0, "CP", 82),
    ("qwen3-8b", "sp-tp2-dp4", 1, 1, 2048, True, 1405, 29.0, "SP", 83),
    ("qwen3-8b", "tp2-dp4", 1, 1, 2048, True, 1391, 28.7, "", 84),
    ("qwen3-8b", "tp8", 1, 1, 4096, True, 1175, 25.9, "", 85),
    ("qwen3-8b", "tp4-dp2", 1, 1, 2048, True, 998, 20.6, "", 86),
    ("qwen3-8b", "tp8", 1, 1, 2048, False, 868, 17.9, "", 87),
    ("qwen3-8b", "tp4-pp2", 1, 1, 2048, True, 793, 16.3, "", 88),
    ("qwen3-8b", "cp2-dp4", 1, 1, 4096, True, None, None, "CP,OOM", 89),
    ("qwen3-14b", "tp4-cp2", 1, 1, 4096, True, 871, 33.6, "CP,DP1", 98),
    ("qwen3-14b", "tp4-dp2", 1, 1, 2048, False, 818, 29.9, "", 99),
    ("qwen3-14b", "tp4-dp2", 1, 1, 2048, True, 718, 26.2, "", 100),
    ("qwen3-14b", "sp-tp4-dp2", 1, 1, 2048, True, 712, 26.1, "SP", 101),
    ("qwen3-14b", "sp-tp8", 1, 1, 2048, False, 651, 23.8, "SP", 102),
    ("qwen3-14b", "tp8", 1, 1, 2048, False, 650, 23.8, "", 103),
    ("qwen3-14b", "tp4-pp2", 1, 1, 2048, True, 565, 20.7, "", 104),
    ("qwen3-14b", "tp8", 1, 1, 2048, True, 514, 18.8, "", 105),
    ("qwen3-32b", "tp8", 2, 1, 2048, True, 377, 30.9, "", 114),
    ("qwen3-32b", "tp8", 1, 1, 4096, True, 369, 32.1, "", 115),
    ("qwen3-32b", "tp8", 1, 1, 2048, False, 369, 30.2, "", 116),
    ("qwen3-32b", "sp-tp8", 1, 1, 2048, False, 365, 29.9, "SP", 117),
    ("qwen3-32b", "tp4-pp2", 1, 1, 2048, False, 295, 24.2, "", 118),
    ("qwen3-32b", "tp4-pp2", 1, 1, 2048, True, 295, 24.1, "", 119),
    ("qwen3-32b", "tp8", 1, 1, 2048, True, 292, 23.9, "", 120),
    ("qwen3-32b", "sp-tp8", 1, 1, 2048, True, 289, 23.6, "SP", 121),
    ("qwen3-30b-a3b", "ep2-tp4", 1, 1, 4096, False, 327, 3.8, "EP", 131),
    ("qwen3-30b-a3b", "ep2-tp4", 1, 1, 2048, False, 233, 2.3, "EP", 132),
    ("qwen3-30b-a3b", "ep4-tp2", 1, 1, 2048, False, 229, 2.2, "EP", 133),
    ("qwen3-30b-a3b", "ep2-tp4", 1, 1, 4096, True, 180, 2.1, "EP", 134),
    ("qwen3-30b-a3b", "ep2-tp4", 2, 1, 2048, True, 176, 1.7, "EP", 135),
    ("qwen3-30b-a3b", "ep4-tp2", 1, 1, 2048, True, 127, 1.2, "EP", 136),
    ("qwen3-30b-a3b", "sp-ep2-tp4", 1, 1, 2048, True, 118, 1.1, "EP,SP", 137),
    ("qwen3-30b-a3b", "ep2-tp4", 1, 1, 2048, True, 114, 1.1, "EP", 138),
    ("qwen3-30b-a3b", "ep2-tp4", 1, 2, 2048, True, 110, 1.1, "EP", 139),
]


def parse_layout(layout: str) -> dict:
    """'sp-tp2-cp2-dp2' -> {tp: 2, cp: 2, dp: 2, pp: 1, ep: 1, sp: True}."""
    out = dict(dp=1, tp=1, pp=1, cp=1, ep=1, sp=False)
    for part in layout.split("-"):
        if part == "sp":
            out["sp"] = True
            continue
        m = re.fullmatch(r"(dp|tp|pp|cp|ep)(\d+)", part)
        if not m:
            raise ValueError(f"bad layout piece {part!r} in {layout!r}")
        out[m.group(1)] = int(m.group(2))
    return out


def rows(gpus: int, pattern: str | None) -> list[dict]:
    out = []
    for model, layout, mbs, ga, seq, gc, ref, ref_mfu, flags, line in ROWS:
        lay = parse_layout(layout)
        mp = lay["tp"] * lay["pp"] * lay["cp"] * lay["ep"]
        if lay["dp"] * mp != 8:
            raise AssertionError(f"{model} {layout}: not an 8-device layout")
        name = f"{model}-{layout}-mbs{mbs}-ga{ga}-s{seq}" + ("-gc" if gc else "")
        if pattern and not re.search(pattern, name):
            continue
        if gpus % mp:
            continue
        out.append(dict(name=name, model=model, layout=layout, mbs=mbs, ga=ga, seq=seq, gc=gc,
                        reference_tok_s_per_gpu=ref, reference_mfu_pct=ref_mfu, flags=flags,
                        reference_source=f"README.md:{line}", **lay))
    return out


def build_cmd(r: dict, gpus: int, steps: int, warmup: int, smoke: bool, rehearse: bool = False) -> list[str]:
    model = r["model"]
    seq, mbs, ga = r["seq"], r["mbs"], r["ga"]
    if r["pp"] > 1 and ga < r["pp"]:
        ga = r["pp"]  # our 1F1B needs >= pp micro-batches in flight (noted in the output line)
    if smoke:
        model = "tiny-moe-8h" if "a3b" in model else "tiny-qwen3-8h"
        seq = min(seq, 64 * r["cp"])
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--model", model,
           "--micro_batch_size", str(mbs), "--grad_acc", str(ga), "--seq_len", str(seq),
           "--tp", str(r["tp"]), "--pp", str(r["pp"]), "--cp", str(r["cp"]), "--ep", str(r["ep"]),
           "--steps", str(steps), "--warmup", str(warmup)]
    if r["sp"]:
        cmd.append("--sp")
    if r["gc"]:
        cmd.append("--gc")
    if smoke:
        cmd += ["--backend", "gloo"]
    if rehearse:  # 8 ranks on ONE GPU over gloo, the real model cut to 2 layers per stage (invalid)
        cmd += ["--backend", "gloo", "--layers", str(2 * r["pp"])]
    return cmd


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--filter", default=None, help="regex over row names")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "reference_rows_8gpu.jsonl"))
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--smoke", action="store_true",
                    help="CPU/gloo plumbing check: tiny models, short sequences (results invalid)")
    ap.add_argument("--rehearse", action="store_true",
                    help="8 ranks on ONE GPU over gloo, real models cut to 2 layers per stage (results invalid)")
    ap.add_argument("--timeout", type=int, default=1200)
    a = ap.parse_args()
    todo = rows(a.gpus, a.filter)
    if a.list or a.dry_run:
        for r in todo:
            print(r["name"], " ".join(build_cmd(r, a.gpus, a.steps, a.warmup, a.smoke)) if a.dry_run else "")
        return 0
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    failures = 0
    with open(a.out, "a") as f:
        for r in todo:
            cmd = build_cmd(r, a.gpus, a.steps, a.warmup, a.smoke, a.rehearse)
            t0 = time.time()
            env = dict(os.environ, MASTER_ADDR="127.0.0.1")
            if a.rehearse:
                # 8 processes time-slice ONE GPU: an xGMI collective waits for peers that are
                # descheduled, so the 2 s production wait bound is raised
                env.update(ST_GPU_OVERSUBSCRIBE="1", OMP_NUM_THREADS="2", ST_XGMI_TIMEOUT_S="60")
            try:
                p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=a.timeout)
                rc, text = p.returncode, p.stdout + p.stderr
            except subprocess.TimeoutExpired as e:
                rc, text = 124, (e.stdout or "") if isinstance(e.stdout, str) else ""
            ours = None
            for line in reversed(text.splitlines()):
                if line.startswith("{") and '"metric"' in line:
                    ours = json.loads(line)
                    break
            rec = dict(r, rc=rc, wall_s=round(time.time() - t0, 1), smoke=a.smoke, rehearse=a.rehearse,
                       ours_tok_s_per_gpu=ours.get("tokens_per_s_per_gpu") if ours else None,
                       ours_mfu_pct=ours.get("mfu_pct") if ours else None, ours=ours)
            if ours and r["reference_tok_s_per_gpu"]:
                rec["ours_over_reference"] = round(ours["tokens_per_s_per_gpu"] / r["reference_tok_s_per_gpu"], 3)
            if rc != 0:
                rec["tail"] = text[-2000:]
                failures += 1
                with open(os.path.splitext(os.path.abspath(a.out))[0] + f"_{r['name']}.log", "w") as lf:
                    lf.write(text)  # the whole output: the failing rank's error is rarely in the tail
            f.write(json.dumps(rec) + "\n")
            f.flush()
            print(f"{r['name']}: rc={rc} ours={rec['ours_tok_s_per_gpu']} ref={r['reference_tok_s_per_gpu']}",
                  flush=True)
            if rc in (124, 137, -9) and not (a.smoke or a.rehearse):
                break  # a hung or killed run: stop, read what it left
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
