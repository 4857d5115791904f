#!/usr/bin/env python3
"""Static instruction mix of the gfx950 kernels in a hipcc ``-S`` listing.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc --cuda-device-only -S csrc/flash_attn.hip -o /tmp/fa.s
  python tools/isa_stats.py /tmp/fa.s [name-filter ...]

Per kernel: total instructions and counts by class (MFMA, AGPR moves, LDS,
VMEM, waitcnt, SALU, v_mov, other VALU), plus the same for the innermost
loop bodies (basic blocks that branch back to themselves or to an earlier
label) -- the numbers that matter for an MFMA-paced loop.
"""
from __future__ import annotations

import re
import sys
from collections import Counter


def classify(op: str) -> str:
    if "mfma" in op:
        return "mfma"
    if op.startswith("v_accvgpr"):
        return "accmov"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_mov") or op.startswith("v_pk_mov"):
        return "vmov"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt")):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    return "other"


def kernels(text: str):
    for m in re.finditer(r"^(\S+):\s*(?:;.*)?$", text, re.M):
        name = m.group(1)
        if name.startswith(".") or not name.startswith("_Z"):
            continue
        end = text.find(".Lfunc_end", m.end())
        yield name, text[m.end():end]


def main():
    path, filters = sys.argv[1], sys.argv[2:]
    text = open(path).read()
    for name, body in kernels(text):
        if filters and not any(f in name for f in filters):
            continue
        total = Counter()
        blocks, cur, label = [], [], None
        labels_seen = []
        for raw in body.split("\n"):
            line = raw.split(";")[0].strip()
            if not line or line.startswith("."):
                if line.startswith(".LBB") and line.endswith(":"):
                    blocks.append((label, cur))
                    label, cur = line[:-1], []
                    labels_seen.append(label)
                continue
            op = line.split()[0]
            total[classify(op)] += 1
            cur.append(line)
        blocks.append((label, cur))
        print(f"{name[:90]}\n  all : {sum(total.values())} {dict(total)}")
        order = {l: i for i, l in enumerate(labels_seen)}
        for lab, ins in blocks:
            if not ins or lab is None:
                continue
            last = ins[-1].split()
            if last[0].startswith("s_cbranch") or last[0] == "s_branch":
                tgt = last[-1]
                if tgt in order and order[tgt] <= order[lab]:
                    # loop: collect blocks from target to here
                    i0, i1 = order[tgt], order[lab]
                    c = Counter()
                    for l2, ins2 in blocks:
                        if l2 in order and i0 <= order[l2] <= i1:
                            for x in ins2:
                                c[classify(x.split()[0])] += 1
                    print(f"  loop {tgt}->{lab}: {sum(c.values())} {dict(c)}")


if __name__ == "__main__":
    main()
