#!/usr/bin/env python3
"""Per-step kernel breakdown from a rocprofv3 ``--kernel-trace`` database.

rocprofv3 (ROCm 7) writes a rocpd SQLite file (``*_results.db``).  This reads its
``kernels`` view, keeps the dispatches of the last ``--steps`` optimizer steps
(step boundaries = the fused AdamW launches, csrc/adamw.hip), groups kernels into
classes (forward / dgrad / wgrad GEMMs, flash attention, AdamW, norms, ...), and
prints per-step milliseconds, the device-busy union (time with >= 1 kernel
running) and the idle remainder of the wall window.

  python tools/rocpd_summary.py gpurun_out/prof/run_results.db --steps 3 --csv profiles/x.csv
  python tools/rocpd_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 3   # csv output format
"""
from __future__ import annotations

import argparse
import csv
import re
import sqlite3
import sys

CLASSES = [  # (class, regex on the kernel name), first match wins
    ("gemm_wgrad_hip", r"wgrad8_kernel|wgrad_gemm_kernel|wgrad_tail_reduce|wgrad4_kernel|wgrad4_tail_reduce"),
    ("gemm_hip(gemm4w)", r"gemm4[a-z_]*kernel|gemm4[bdef]"),
    ("gemm_fp32_out(wgrad_hipblaslt)", r"Cijk_.*_BSS_|Cijk_.*BBS_BS_"),
    ("gemm_bf16(fwd+dgrad)", r"Cijk_"),
    ("grouped_gemm(experts)", r"grouped|Grouped"),
    ("moe_route/permute/combine", r"moe_|topk|permute|combine|gather_rows"),
    ("flash_fwd", r"flash_fwd"),
    ("flash_bwd", r"flash_bwd"),
    ("adamw", r"adamw_kernel|adamw_wt_kernel"),
    ("grad_norm", r"sumsq_kernel|sum_partials_kernel"),
    ("rmsnorm", r"rmsnorm|colsum_kernel"),
    ("swiglu", r"swiglu"),
    ("rope", r"rope_kernel|qknorm_rope"),
    ("xent", r"xent_"),
    ("transpose(W^T)", r"transpose_kernel|transpose"),
    ("embedding", r"embedding|index_add|indexSelect|index_select"),
    ("copy/fill/elementwise", r"copyBuffer|FillFunctor|elementwise|CatArray|fill"),
]


def classify(name: str) -> str:
    for cls, rx in CLASSES:
        if re.search(rx, name):
            return cls
    return "other"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=3, help="timed steps at the end of the run")
    ap.add_argument("--csv", default="", help="write per-kernel stats of the window here")
    ap.add_argument("--gap_ms", type=float, default=50.0,
                    help="AdamW launches further apart than this start a new step (below the step time)")
    args = ap.parse_args()
    if args.db.endswith(".csv"):  # rocprofv3 --output-format csv: *_kernel_trace.csv
        with open(args.db, newline="") as f:
            rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                           for r in csv.DictReader(f)), key=lambda r: r[1])
    else:
        c = sqlite3.connect(args.db)
        rows = c.execute("select name, start, end from kernels order by start").fetchall()
    ad = [(s, e) for n, s, e in rows if "adamw_kernel" in n or "adamw_wt_kernel" in n]
    if len(ad) < args.steps + 1:
        print("not enough AdamW launches to find step boundaries", file=sys.stderr)
        return 1
    # group AdamW launches into steps (arenas of one step launch back to back)
    groups = [[ad[0]]]
    for s, e in ad[1:]:
        if s - groups[-1][-1][1] > args.gap_ms * 1e6:  # far apart: a new step
            groups.append([(s, e)])
        else:
            groups[-1].append((s, e))
    if len(groups) < args.steps + 1:
        print(f"found {len(groups)} steps, need {args.steps + 1}", file=sys.stderr)
        return 1
    t0 = max(e for _, e in groups[-args.steps - 1])
    t1 = max(e for _, e in groups[-1])
    win = [(n, s, e) for n, s, e in rows if s >= t0 and e <= t1]
    wall = (t1 - t0) / 1e6 / args.steps
    # union of busy intervals
    busy, cur_s, cur_e = 0, None, None
    for _, s, e in sorted(win, key=lambda r: r[1]):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    per_cls, per_k = {}, {}
    for n, s, e in win:
        d = (e - s) / 1e6
        k = classify(n)
        per_cls[k] = per_cls.get(k, 0.0) + d
        st = per_k.setdefault(n, [0, 0.0])
        st[0] += 1
        st[1] += d
    total = sum(per_cls.values())
    print(f"window: last {args.steps} steps, {wall:.2f} ms/step wall, device busy (union) "
          f"{busy / 1e6 / args.steps:.2f} ms/step, idle {wall - busy / 1e6 / args.steps:.2f} ms/step, "
          f"sum of kernel durations {total / args.steps:.2f} ms/step (overlap {total / args.steps - busy / 1e6 / args.steps:.2f})")
    for k, v in sorted(per_cls.items(), key=lambda kv: -kv[1]):
        print(f"  {k:34s} {v / args.steps:8.2f} ms/step  {100 * v / total:5.1f} %")
    if args.csv:
        with open(args.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Class", "CallsPerStep", "MsPerStep", "AvgUs"])
            for n, (cnt, d) in sorted(per_k.items(), key=lambda kv: -kv[1][1]):
                w.writerow([n[:200], classify(n), cnt / args.steps, round(d / args.steps, 3), round(d / cnt * 1e3, 2)])
    return 0


if __name__ == "__main__":
    sys.exit(main())
