#!/usr/bin/env python3
"""Multi-configuration benchmark driver (reference: scripts/benchmark_comprehensive.py,
scripts/benchmark_all.py, scripts/benchmark_moe.sh).

Runs ``bench.py`` under torchrun for a grid of model x parallel layouts on one
node, parses the JSON line each run prints, and appends it to an incremental
results file (re-runs skip finished configs unless --force).  Layouts are the
reference's families -- pure DP, TP+DP, PP+DP, CP+DP, SP, mixed TP/PP/CP, EP
for MoE -- generated per model instead of a hand-copied list, plus the MI355X
options the reference lacks (ZeRO-1, CP transport).

  python scripts/benchmark_sweep.py --list
  python scripts/benchmark_sweep.py --gpus 8 --filter '8b' --steps 10 --out bench_results.jsonl
  python scripts/benchmark_sweep.py --dry-run --filter 'qwen3-0.6b-.*tp2'
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

# model -> (micro_batch, seq, activation checkpointing)
MODELS = {
    "qwen3-0.6b": (4, 4096, False),
    "qwen3-1.7b": (4, 4096, False),
    "qwen3-4b": (2, 4096, False),
    "qwen3-8b": (2, 4096, False),
    "llama3-8b": (2, 4096, False),
    "qwen3-14b": (1, 4096, True),
    "qwen3-32b": (1, 4096, True),
    "llama3-70b": (1, 4096, True),
}
MOE_MODELS = {"qwen3-30b-a3b": (1, 4096, True), "mixtral-8x7b": (1, 4096, True)}

# (suffix, tp, pp, cp, ep, sp, extra) with dp = gpus / (tp*pp*cp*ep)
DENSE_LAYOUTS = [
    ("dp", 1, 1, 1, 1, False, {}),
    ("dp-zero0", 1, 1, 1, 1, False, {"zero": 0}),
    ("tp2-dp", 2, 1, 1, 1, False, {}),
    ("tp4-dp", 4, 1, 1, 1, False, {}),
    ("tp8", 8, 1, 1, 1, False, {}),
    ("sp-tp2-dp", 2, 1, 1, 1, True, {}),
    ("pp2-dp", 1, 2, 1, 1, False, {}),
    ("pp4-dp", 1, 4, 1, 1, False, {}),
    ("cp2-dp", 1, 1, 2, 1, False, {"seq": 8192}),
    ("cp4-dp-ring", 1, 1, 4, 1, False, {"seq": 16384, "cp_comm": "ring"}),
    ("cp4-dp-ulysses", 1, 1, 4, 1, False, {"seq": 16384, "cp_comm": "ulysses"}),
    ("cp8-32k", 1, 1, 8, 1, False, {"seq": 32768, "mbs": 1}),
    ("tp2-pp2-dp", 2, 2, 1, 1, False, {}),
    ("tp2-cp2-dp", 2, 1, 2, 1, False, {"seq": 8192}),
    ("tp2-pp2-cp2", 2, 2, 2, 1, False, {"seq": 8192}),
]
MOE_LAYOUTS = [
    ("ep8", 1, 1, 1, 8, False, {}),
    ("ep4-dp", 1, 1, 1, 4, False, {}),
    ("ep2-tp2-dp", 2, 1, 1, 2, False, {}),
]


def build_configs(gpus: int) -> list[dict]:
    out = []
    for models, layouts in ((MODELS, DENSE_LAYOUTS), (MOE_MODELS, MOE_LAYOUTS)):
        for m, (mbs, seq, gc) in models.items():
            for suffix, tp, pp, cp, ep, sp, extra in layouts:
                mp = tp * pp * cp * ep
                if gpus % mp:
                    continue
                out.append(dict(name=f"{m}-{suffix}".replace("-dp", f"-dp{gpus // mp}"), model=m, tp=tp, pp=pp,
                                cp=cp, ep=ep, sp=sp, mbs=extra.get("mbs", mbs), seq=extra.get("seq", seq), gc=gc,
                                cp_comm=extra.get("cp_comm", "allgather"), zero=extra.get("zero", 1)))
    return out


def build_cmd(c: dict, gpus: int, steps: int, warmup: int, port: int) -> list[str]:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(gpus), "--steps", str(steps), "--warmup", str(warmup), "--model", c["model"],
           "--micro_batch_size", str(c["mbs"]), "--seq_len", str(c["seq"]), "--tp", str(c["tp"]), "--pp", str(c["pp"]),
           "--cp", str(c["cp"]), "--ep", str(c["ep"]), "--cp_comm", c["cp_comm"], "--zero", str(c["zero"])]
    if c["sp"]:
        cmd.append("--sp")
    if c["gc"]:
        cmd.append("--gc")
    return cmd


def parse_result(stdout: str) -> dict | None:
    """The last JSON object line bench.py printed (rank 0)."""
    for line in reversed(stdout.strip().splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            try:
                return json.loads(line)
            except json.JSONDecodeError:
                continue
    return None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--filter", default="", help="regex on config names")
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--force", action="store_true", help="re-run configs already in --out")
    ap.add_argument("--out", default=os.path.join(ROOT, "bench_results.jsonl"))
    ap.add_argument("--timeout", type=int, default=1800)
    ap.add_argument("--port", type=int, default=29511)
    args = ap.parse_args(argv)
    cfgs = [c for c in build_configs(args.gpus) if re.search(args.filter, c["name"])]
    if args.list:
        for c in cfgs:
            print(f"{c['name']:36s} tp{c['tp']} pp{c['pp']} cp{c['cp']} ep{c['ep']} sp={int(c['sp'])} "
                  f"mbs={c['mbs']} seq={c['seq']} gc={int(c['gc'])} cp_comm={c['cp_comm']} zero={c['zero']}")
        return 0
    done = set()
    if os.path.exists(args.out) and not args.force:
        with open(args.out) as f:
            for line in f:
                try:
                    done.add(json.loads(line)["sweep_name"])
                except (json.JSONDecodeError, KeyError):
                    pass
    for i, c in enumerate(cfgs):
        cmd = build_cmd(c, args.gpus, args.steps, args.warmup, args.port + i % 50)
        if args.dry_run:
            print(" ".join(cmd))
            continue
        if c["name"] in done:
            print(f"[skip] {c['name']} (in {args.out})")
            continue
        t0 = time.time()
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        try:
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=args.timeout, env=env, cwd=ROOT)
            res = parse_result(p.stdout)
            status = "ok" if (p.returncode == 0 and res) else f"failed rc={p.returncode}"
            err = "" if status == "ok" else (p.stderr or "")[-2000:]
        except subprocess.TimeoutExpired:
            res, status, err = None, "timeout", ""
        rec = dict(sweep_name=c["name"], status=status, wall_s=round(time.time() - t0, 1), config=c,
                   result=res, stderr_tail=err)
        with open(args.out, "a") as f:
            f.write(json.dumps(rec) + "\n")
        msg = (f"{res['tokens_per_s_per_gpu']:.0f} tok/s/GPU, MFU {res['mfu_pct']:.1f}%" if res else err[-300:])
        print(f"[{status}] {c['name']}: {msg}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
