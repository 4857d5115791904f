#!/usr/bin/env python3
"""Single-GPU sweep of micro-batch x sequence length x activation checkpointing.

Reference: tools/bench_single.py:30-111 (bs / seq / GC / fused sweep on one NPU)
and scripts/sweep_mfu.sh.  Each point is one ``bench.py`` child process (a point
that runs out of memory cannot take the sweep down); results are appended to a
JSONL file as they finish, so an interrupted sweep keeps what it measured.

  python tools/bench_single.py --model llama3-8b --mbs 1,2,4 --seq 2048,4096,8192 --gc 0,1 \\
      --out gpurun_out/sweep_single.jsonl
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--mbs", default="1,2")
    ap.add_argument("--seq", default="2048,4096")
    ap.add_argument("--gc", default="0")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--timeout", type=int, default=600)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sweep_single.jsonl"))
    ap.add_argument("--dry-run", action="store_true")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    grid = list(itertools.product([int(x) for x in args.mbs.split(",")], [int(x) for x in args.seq.split(",")],
                                  [int(x) for x in args.gc.split(",")]))
    rc_all = 0
    for mbs, seq, gc in grid:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--model", args.model, "--micro_batch_size", str(mbs),
               "--seq_len", str(seq), "--steps", str(args.steps), "--warmup", str(args.warmup)]
        if gc:
            cmd.append("--gc")
        if args.dry_run:
            print(" ".join(cmd))
            continue
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=args.timeout, cwd=ROOT)
            line = next((l for l in reversed(r.stdout.splitlines()) if l.startswith("{")), None)
            rec = json.loads(line) if line and r.returncode == 0 else {"error": (r.stderr or r.stdout)[-800:]}
        except subprocess.TimeoutExpired:
            rec = {"error": f"timeout after {args.timeout}s"}
        rec.update(sweep={"model": args.model, "mbs": mbs, "seq": seq, "gc": bool(gc)})
        rc_all |= "error" in rec
        with open(args.out, "a") as f:
            f.write(json.dumps(rec) + "\n")
        short = {k: rec.get(k) for k in ("tokens_per_s_per_gpu", "mfu_pct", "ms_per_step", "max_mem_gb", "error")}
        print(json.dumps({"mbs": mbs, "seq": seq, "gc": bool(gc), **short}), flush=True)
    return 1 if rc_all else 0


if __name__ == "__main__":
    sys.exit(main())
