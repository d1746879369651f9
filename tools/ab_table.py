#!/usr/bin/env python3
"""Per-layer table of a tools/ab_layers.sh output (one column per library run, in run order).
usage: python tools/ab_table.py gpurun_out/ab_TAG.txt"""
import re
import sys


def main(path):
    txt = open(path).read()
    cols, rows = [], {}
    for b in re.split(r"\n(?=\[)", txt):
        lines = b.strip().splitlines()
        if not lines or not lines[0].startswith("["):
            continue
        tag = lines[0].split("]")[0][1:]
        n = sum(1 for c in cols if c.split("#")[0] == tag)
        tag = f"{tag}#{n}" if n else tag
        cols.append(tag)
        total = re.search(r"total ([\d.]+) ms", lines[0])
        rows.setdefault("TOTAL ms", {})[tag] = float(total.group(1)) * 1000 if total else 0.0
        for ln in lines[1:]:
            m = re.match(r"\s+(\S+)\s+(\S+)\s+([\d.]+) us", ln)
            if m:
                rows.setdefault(m.group(1), {})[tag] = float(m.group(3))
    print(f"{'layer (us)':30s}" + "".join(f"{c:>11s}" for c in cols))
    for k, v in rows.items():
        print(f"{k:30s}" + "".join(f"{v.get(c, 0):11.1f}" for c in cols))


if __name__ == "__main__":
    main(sys.argv[1])
