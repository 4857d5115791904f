#!/usr/bin/env python3
"""Per-kernel PMC rows from rocprofv3 ``--pmc`` passes (one sub-directory ``pmc_*`` per pass
under ROOT), grouped by (kernel, grid size): duration, MFMA busy, clock, HBM fetch / write,
L2 hit, wait and VALU shares.

  python tools/pmc_by_grid.py ROOT [REGEX]      (REGEX: kernels to keep, default "flash")
"""
import csv, glob, sys, collections, re
root = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else "flash")
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = {}
for d in glob.glob(root + "/pmc_*"):
    for f in glob.glob(d + "/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if not pat.search(n): continue
            short = re.sub(r"\(anonymous namespace\)::", "", n).split("(")[0].replace("void ", "")
            short = short if len(short) <= 45 else short[:20] + ".." + short[-23:]
            key = (short, int(r["Grid_Size"]))
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur.setdefault((d, r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            vals[key]["_dur_" + d].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for key in sorted(vals):
    c = vals[key]
    def avg(n): 
        v = c.get(n); return sum(v)/len(v) if v else None
    # mean duration over every dispatch of the group (all passes): persistent kernels share one
    # grid over many shapes, so a min would pair one shape's time with another's counters
    durs = [x for k in c if k.startswith("_dur_") for x in c[k]]
    t = sum(durs) / len(durs) if durs else None
    busy, gui = avg("SQ_VALU_MFMA_BUSY_CYCLES"), avg("GRBM_GUI_ACTIVE")
    fetch, write = avg("FETCH_SIZE"), avg("WRITE_SIZE")
    hit, miss = avg("TCC_HIT_sum"), avg("TCC_MISS_sum")
    wc, wi = avg("SQ_WAVE_CYCLES"), avg("SQ_WAIT_INST_ANY")
    av = avg("SQ_ACTIVE_INST_VALU")
    n = max((len(c[k]) for k in c if k.startswith("_dur_")), default=0)
    out = f"{key[0]:45s} grid {key[1]:8d} n {n:4d} t {t/1e3 if t else 0:8.1f}us"
    if busy and gui: out += f" mfma {100*busy/(gui/8*1024):5.1f}% clk {gui/8/t:4.2f}"
    if fetch is not None: out += f" fetch {fetch/1024:8.1f}MB"
    if write is not None: out += f" write {write/1024:8.1f}MB"
    if fetch is not None and write is not None and t: out += f" {((fetch+write)*1024)/t:6.0f}GB/s"
    if hit is not None and miss is not None: out += f" L2hit {100*hit/max(1,hit+miss):5.1f}%"
    if wc and wi: out += f" wait/wave {100*wi/wc:5.1f}%"
    if wc and av: out += f" valu/wave {100*av/wc:5.1f}%"
    print(out)
