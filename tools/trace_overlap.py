#!/usr/bin/env python3
"""What the side-stream optimizer costs the kernels it overlaps, from one rocprofv3 trace.

For the last ``--steps`` steps of a ``--kernel-trace`` database (step windows as in
tools/rocpd_summary.py), every kernel is tagged "overlapped" when more than half of its
duration falls inside the union of the AdamW / grad-norm (side-stream) kernels, else
"clean".  Per kernel name: mean duration clean vs overlapped, and the EXTRA time the
overlapped launches took beyond the clean mean -- summed, the interference the side stream
puts on the step's critical path ("which kernels grow and which AdamW
buckets they overlap").

  python tools/trace_overlap.py gpurun_out/x/run_results.db --steps 2 [--top 25]
"""
from __future__ import annotations

import argparse
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocpd_summary import classify  # noqa: E402

SIDE = ("adamw_kernel", "adamw_wt_kernel", "sumsq_kernel", "sum_partials_kernel")


def _union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _overlap(s, e, uni, start_idx):
    tot, i = 0, start_idx
    while i < len(uni) and uni[i][1] <= s:
        i += 1
    j = i
    while j < len(uni) and uni[j][0] < e:
        tot += min(e, uni[j][1]) - max(s, uni[j][0])
        j += 1
    return tot, i


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--gap_ms", type=float, default=50.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    ad = [(s, e) for n, s, e in rows if "adamw_kernel" in n or "adamw_wt_kernel" in n]
    groups = [[ad[0]]]
    for s, e in ad[1:]:
        if s - groups[-1][-1][1] > a.gap_ms * 1e6:
            groups.append([(s, e)])
        else:
            groups[-1].append((s, e))
    if len(groups) < a.steps + 1:
        print(f"found {len(groups)} steps, need {a.steps + 1}", file=sys.stderr)
        return 1
    t0 = max(e for _, e in groups[-a.steps - 1])
    t1 = max(e for _, e in groups[-1])
    win = [(n, s, e) for n, s, e in rows if s >= t0 and e <= t1]
    side = _union([(s, e) for n, s, e in win if any(k in n for k in SIDE)])
    side_ms = sum(e - s for s, e in side) / 1e6 / a.steps
    stats = {}  # name -> [clean n, clean sum, ov n, ov sum]
    idx = 0
    for n, s, e in win:
        if any(k in n for k in SIDE):
            continue
        ov, idx = _overlap(s, e, side, idx)
        st = stats.setdefault(n, [0, 0.0, 0, 0.0])
        if 2 * ov > (e - s):
            st[2] += 1
            st[3] += (e - s) / 1e6
        else:
            st[0] += 1
            st[1] += (e - s) / 1e6
    rows_out, extra_total, per_cls = [], 0.0, {}
    for n, (cn, cs, on, os_) in stats.items():
        if on == 0:
            continue
        if cn == 0:  # never ran clean: no baseline for this name
            rows_out.append((0.0, n, cn, None, on, os_ / on))
            continue
        mc = cs / cn
        extra = os_ - on * mc
        extra_total += extra
        k = classify(n)
        per_cls[k] = per_cls.get(k, 0.0) + extra
        rows_out.append((extra, n, cn, mc, on, os_ / on))
    print(f"window: {a.steps} steps; side-stream (AdamW + grad-norm) busy {side_ms:.2f} ms/step")
    print(f"extra time of overlapped main-stream kernels over their clean mean: "
          f"{extra_total / a.steps:.2f} ms/step")
    for k, v in sorted(per_cls.items(), key=lambda kv: -kv[1]):
        print(f"  {k:34s} {v / a.steps:+8.2f} ms/step")
    print(f"\n{'extra ms/step':>13} {'clean n':>7} {'clean us':>9} {'ovl n':>6} {'ovl us':>9}  kernel")
    for extra, n, cn, mc, on, mo in sorted(rows_out, key=lambda r: -r[0])[: a.top]:
        mcs = f"{mc * 1e3:9.1f}" if mc is not None else "        -"
        print(f"{extra / a.steps:13.3f} {cn:7d} {mcs} {on:6d} {mo * 1e3:9.1f}  {n[:90]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
