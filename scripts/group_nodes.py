#!/usr/bin/env python3
"""Group a node list into racks / islands and write one node file per group.

Reference: scripts/group_nodes.py:10-71 (rack grouping helper for the multi-node
launcher).  A node's group is the regex capture ``--pattern`` applied to its
hostname (default: the hostname without its trailing number, e.g.
``mi355x-r07-n03`` -> ``mi355x-r07-n``), or a fixed ``--size`` chunking of the
list order.  Output: ``<outdir>/group_<k>.txt`` files usable as
``scripts/launch_multi_nodes.sh`` node lists, and a JSON summary on stdout.

  python scripts/group_nodes.py node_list.txt --outdir groups/
  python scripts/group_nodes.py node_list.txt --size 4 --outdir groups/
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
from collections import OrderedDict


def group_nodes(nodes: list[str], pattern: str = r"^(.*?)(\d+)$", size: int = 0) -> "OrderedDict[str, list[str]]":
    out: "OrderedDict[str, list[str]]" = OrderedDict()
    if size > 0:
        for i in range(0, len(nodes), size):
            out[f"chunk{i // size}"] = nodes[i: i + size]
        return out
    rx = re.compile(pattern)
    for n in nodes:
        m = rx.match(n)
        key = m.group(1) if m else n
        out.setdefault(key, []).append(n)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("node_list")
    ap.add_argument("--pattern", default=r"^(.*?)(\d+)$")
    ap.add_argument("--size", type=int, default=0)
    ap.add_argument("--outdir", default="node_groups")
    args = ap.parse_args()
    with open(args.node_list) as f:
        nodes = [l.split("#", 1)[0].strip() for l in f]
    nodes = [n for n in nodes if n]
    groups = group_nodes(nodes, args.pattern, args.size)
    os.makedirs(args.outdir, exist_ok=True)
    summary = {}
    for k, (name, ns) in enumerate(groups.items()):
        path = os.path.join(args.outdir, f"group_{k}.txt")
        with open(path, "w") as f:
            f.write("\n".join(ns) + "\n")
        summary[name] = {"file": path, "nodes": ns}
    print(json.dumps(summary, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
