#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py: per-kernel-class launches and
average duration, next to bench.py's own HIP-event figure (roofline.per_launch_avg_us).
usage: python tools/prof_summary.py <run_kernel_stats.csv> [bench_json] > profiles/rNN_prof_summary.txt"""
import csv
import json
import sys

CLASSES = [("conv (f32 MFMA)", "conv_gemm_kernel"), ("conv (f16 MFMA)", "conv_f16_kernel"),
           ("conv (window)", "conv_win_kernel"), ("maxpool", "maxpool"), ("gap", "gap_kernel"),
           ("softmax", "softmax_kernel"), ("pack/ktab (load time)", "pack_"), ("ktab", "ktab_kernel")]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    print(f"{'class':24s} {'launches':>9s} {'total ms':>10s} {'avg us':>9s}")
    for label, key in CLASSES:
        sel = [r for r in rows if key in r["Name"]]
        if not sel:
            continue
        calls = sum(int(r["Calls"]) for r in sel)
        tot = sum(float(r["TotalDurationNs"]) for r in sel)
        print(f"{label:24s} {calls:9d} {tot / 1e6:10.3f} {tot / calls / 1e3:9.2f}")
    if len(sys.argv) > 2:
        b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
        r = b.get("roofline", {})
        print(f"\nbench.py (HIP events, same run): conv per_launch_avg_us = {r.get('per_launch_avg_us')}, "
              f"achieved {r.get('achieved')} {r.get('unit')} = {r.get('frac')} of {r.get('peak')}")
    print("\nper-kernel rows:")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        print(f"  {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} us  {r['Name'][:110]}")


if __name__ == "__main__":
    main()
