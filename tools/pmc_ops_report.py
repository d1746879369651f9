#!/usr/bin/env python3
"""Per-tile PMC summary of tools/pmc_ops.sh output: the conv kernel's last dispatch per pass.
usage: python tools/pmc_ops_report.py gpurun_out/pmcops_TAG"""
import csv
import glob
import os
import re
import sys
from collections import OrderedDict, defaultdict


def last_dispatch(d):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        return None
    disp = OrderedDict()
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "_ZN3ore" not in n and "ore::" not in n or "pack" in n or "ktab" in n or "wino_u" in n:
            continue
        e = disp.setdefault(int(r["Dispatch_Id"]), {"name": n, "dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                    "vgpr": r["VGPR_Count"], "agpr": r["Accum_VGPR_Count"],
                                                    "lds": r.get("LDS_Block_Size", r.get("Lds_Size", ""))})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(disp.values())[-1] if disp else None


def main():
    base = sys.argv[1]
    tiles = defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(base, "t*_p*"))):
        m = re.match(r"t(-?\d+)_p(\d+)$", os.path.basename(d))
        if not m or not os.path.isdir(d):
            continue
        r = last_dispatch(d)
        if r:
            tiles[int(m.group(1))].update(r)
    print(f"{'tile':>4s} {'us':>7s} {'waves':>7s} {'valu/w':>7s} {'mfma/w':>7s} {'lds/w':>6s} {'vmr/w':>6s} {'salu/w':>6s} "
          f"{'mfma%':>6s} {'wait%':>6s} {'waitI%':>6s} {'ldsbc/w':>7s} {'GHz':>5s} {'v/a':>7s} kernel")
    for t, r in sorted(tiles.items()):
        w = max(r.get("SQ_WAVES", 1), 1)
        dur = r.get("dur", 1) / 1e3
        busy = r.get("GRBM_GUI_ACTIVE", 0)
        clk = busy / 8 if busy else dur * 1e3 * 2.1
        mf = 100.0 * r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * clk) if clk else 0
        wc = r.get("SQ_WAVE_CYCLES", 0)
        wa = 100.0 * r.get("SQ_WAIT_ANY", 0) / wc if wc else 0
        wi = 100.0 * r.get("SQ_WAIT_INST_ANY", 0) / wc if wc else 0
        name = re.sub(r"^_ZN3ore", "", r["name"])[:60]
        print(f"{t:4d} {dur:7.1f} {w:7.0f} {r.get('SQ_INSTS_VALU', 0) / w:7.0f} {r.get('SQ_INSTS_MFMA', 0) / w:7.0f} "
              f"{r.get('SQ_INSTS_LDS', 0) / w:6.0f} {r.get('SQ_INSTS_VMEM_RD', 0) / w:6.0f} {r.get('SQ_INSTS_SALU', 0) / w:6.0f} "
              f"{mf:6.1f} {wa:6.1f} {wi:6.1f} {r.get('SQ_LDS_BANK_CONFLICT', 0) / w:7.0f} "
              f"{(busy / 8 / (dur * 1e3)) if busy else 0:5.2f} {r.get('vgpr', '')}/{r.get('agpr', '')} {name}")


if __name__ == "__main__":
    main()
