#!/usr/bin/env python3
"""Summarise rocprofv3 ``--pmc`` runs per kernel (MFMA utilisation, LDS bank
conflicts, HBM bytes / bandwidth).

Each counter group is collected in its own rocprofv3 run (``--pmc`` together
with ``--kernel-trace`` only); point this at the output directories:

  python tools/pmc_summary.py gpurun_out/pmc_mfma gpurun_out/pmc_lds gpurun_out/pmc_hbm > profiles/x.md

Derived numbers per kernel (summed over its dispatches, then averaged):
  * mfma_busy %   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
  * clock GHz     = GRBM_GUI_ACTIVE / 8 / kernel time (the clock the kernel actually ran at)
  * bf16 TF/s     = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 / kernel time
  * lds_conflict  = SQ_LDS_BANK_CONFLICT / (SQ_LDS_IDX_ACTIVE - SQ_LDS_BANK_CONFLICT)  (cycles / access-cycle)
  * HBM GB/s      = (FETCH_SIZE + WRITE_SIZE) KiB / kernel time
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict

SIMDS = 1024   # 256 CUs x 4 SIMDs
XCDS = 8       # GRBM_GUI_ACTIVE comes back summed over the 8 XCDs


def _short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0][:70]


def load(dirs):
    vals = defaultdict(lambda: defaultdict(float))   # kernel -> counter -> sum
    disp = defaultdict(set)                          # kernel -> dispatch ids (per run dir)
    dur = defaultdict(float)                         # kernel -> ns (from the run with kernel traces)
    ndur = defaultdict(int)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = _short(row["Kernel_Name"])
                    vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
                    disp[(k, row["Counter_Name"])].add((f, row["Dispatch_Id"]))
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = _short(row["Kernel_Name"])
                    dur[k] += float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
                    ndur[k] += 1
    return vals, disp, dur, ndur


def main(argv):
    dirs = argv[1:] or ["gpurun_out"]
    vals, disp, dur, ndur = load(dirs)
    rows = []
    for k, c in vals.items():
        def n(name):
            return max(1, len(disp.get((k, name), ())))

        def per(name):
            return c[name] / n(name) if name in c else None

        t_ns = dur[k] / ndur[k] if ndur.get(k) else None
        r = {"kernel": k, "dispatches": ndur.get(k, 0), "avg_us": t_ns / 1e3 if t_ns else None}
        busy, gui = per("SQ_VALU_MFMA_BUSY_CYCLES"), per("GRBM_GUI_ACTIVE")
        if busy is not None and gui:
            r["mfma_busy_%"] = 100 * busy / (gui / XCDS * SIMDS)
            if t_ns:
                r["clock_GHz"] = gui / XCDS / t_ns
        mops = per("SQ_INSTS_VALU_MFMA_MOPS_BF16")
        if mops is not None and t_ns:
            r["bf16_TFps"] = mops * 512 / t_ns / 1e3
        bc, ia = per("SQ_LDS_BANK_CONFLICT"), per("SQ_LDS_IDX_ACTIVE")
        if bc is not None and ia:
            r["lds_conflict"] = bc / max(1.0, ia - bc)
        fs, ws = per("FETCH_SIZE"), per("WRITE_SIZE")
        rd, rd32, wr, wr64 = (per(x) for x in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_WRREQ_sum",
                                               "TCC_EA0_WRREQ_64B_sum"))
        if fs is None and None not in (rd, rd32, wr, wr64):  # raw L2->memory requests: 64 B reads, 32/64 B writes
            fs = ((rd - rd32) * 64 + rd32 * 32) / 1024
            ws = ((wr - wr64) * 32 + wr64 * 64) / 1024
        if fs is not None and ws is not None:
            r["hbm_MB"] = (fs + ws) * 1024 / 1e6
            if t_ns:
                r["hbm_GBps"] = (fs + ws) * 1024 / t_ns
        rows.append(r)
    rows.sort(key=lambda r: -(r["avg_us"] or 0) * max(1, r["dispatches"]))
    cols = ["kernel", "dispatches", "avg_us", "clock_GHz", "mfma_busy_%", "bf16_TFps", "lds_conflict", "hbm_MB", "hbm_GBps"]
    print("| " + " | ".join(cols) + " |")
    print("|" + "---|" * len(cols))
    for r in rows:
        cells = []
        for col in cols:
            v = r.get(col)
            cells.append("" if v is None else (f"{v:.3g}" if isinstance(v, float) else str(v)))
        print("| " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main(sys.argv)
