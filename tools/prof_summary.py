#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py: per-kernel-class launches and
average duration, next to bench.py's own HIP-event figure (roofline.per_launch_avg_us).
usage: python tools/prof_summary.py <run_kernel_stats.csv> [bench_json] > profiles/rNN_prof_summary.txt

With run_kernel_trace.csv beside the stats file, the classes are also computed over the timed
steps only (the last `steps` x per-step dispatches of the run: autotune candidates and warm-up runs
excluded), which is what bench.py's per_launch_avg_us measures."""
import csv
import json
import os
import sys

CLASSES = [("conv (f32 MFMA)", ("conv_gemm_kernel", "conv_stream_kernel", "conv_stream1x1_persist_kernel", "fire_kernel", "conv_pool_stream_kernel",
                                "conv_wino32_kernel", "conv_wino16_kernel", "conv_winol_kernel", "fire_wino_kernel",
                                "conv_win_pool_f32_kernel", "conv_band_pool_f32_kernel", "fire_pool_kernel", "pool_conv1x1_f32_kernel",
                                "conv1x1_gap_f32_kernel")),
           ("conv (f16 MFMA)", ("conv_f16_kernel", "conv_f16_dma_kernel", "conv_f16_epool", "fire_f16_kernel",
                                "fire_pool_f16_kernel", "conv_pair_pool_f16_kernel", "conv1x1_gap_f16_kernel")),
           ("conv (window)", "conv_win_kernel"), ("maxpool", "maxpool"), ("gap", ("gap_kernel", "gap_nhwc_kernel")),
           ("softmax", "softmax_kernel"), ("pack/ktab (load time)", "pack_"), ("ktab", "ktab_kernel")]


def hit(key, name):
    return any(k in name for k in key) if isinstance(key, tuple) else key in name


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    print(f"{'class':24s} {'launches':>9s} {'total ms':>10s} {'avg us':>9s}")
    for label, key in CLASSES:
        sel = [r for r in rows if hit(key, r["Name"])]
        if not sel:
            continue
        calls = sum(int(r["Calls"]) for r in sel)
        tot = sum(float(r["TotalDurationNs"]) for r in sel)
        print(f"{label:24s} {calls:9d} {tot / 1e6:10.3f} {tot / calls / 1e3:9.2f}")
    trace = os.path.join(os.path.dirname(sys.argv[1]), "run_kernel_trace.csv")
    bench = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]) if len(sys.argv) > 2 else None
    last = []
    if os.path.exists(trace) and bench:
        disp = [r for r in csv.DictReader(open(trace)) if "ore::" in r["Kernel_Name"] or "_ZN3ore" in r["Kernel_Name"]]
        disp.sort(key=lambda r: int(r["Dispatch_Id"]))
        # dispatches per step: the distance between the last two softmax launches (every step ends
        # with the softmax)
        sm = [i for i, r in enumerate(disp) if "softmax" in r["Kernel_Name"]]
        per = sm[-1] - sm[-2] if len(sm) >= 2 else 31
        last = disp[-per * int(bench["steps"]):]
        print(f"\ntimed steps only (last {len(last)} dispatches = {bench['steps']} steps x {per}):")
        for label, key in CLASSES:
            sel = [r for r in last if hit(key, r["Kernel_Name"])]
            if sel:
                tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel)
                print(f"{label:24s} {len(sel):9d} {tot / 1e6:10.3f} {tot / len(sel) / 1e3:9.2f}")
    if bench:
        b = bench
        r = b.get("roofline", {})
        cc = r.get("conv_class", r)
        print(f"\nbench.py (HIP events, same run): conv class per_launch_avg_us = {cc.get('per_launch_avg_us')}, "
              f"achieved {cc.get('achieved')} {cc.get('unit', 'TFLOP/s')} = {cc.get('frac')} of {cc.get('peak')}")
        if "launch_us" in r:  # round 5: the dominant launch, which the rocprof row of its kernel must agree with
            print(f"bench.py dominant launch: {r.get('kernel')}: {r.get('launch_us')} us, achieved {r.get('achieved')} "
                  f"{r.get('unit')} = {r.get('frac')} of {r.get('peak')}")
            kern = {"epool band f32": "conv_band_pool_f32_kernel", "epool window f32": "conv_win_pool_f32_kernel",
                    "first conv pool f16": "conv_pair_pool_f16_kernel", "epool band f16": "conv_band_pool_f16_kernel"}
            names = [k for t, k in kern.items() if f"tile '{t}'" in str(r.get("kernel"))] or list(kern.values())
            dom = [x for x in rows if any(k in x["Name"] for k in names)]
            for x in dom:
                print(f"rocprofv3 row of that kernel: {int(x['Calls'])} calls, average {float(x['AverageNs']) / 1e3:.2f} us "
                      f"({x['Name'][:90]})")
            # round 6: the same kernel over the timed steps only (the stats row also averages the autotune's
            # candidate runs and the warm-up)
            tl = [q for q in last if any(k in q["Kernel_Name"] for k in names)]
            if tl:
                tot = sum(int(q["End_Timestamp"]) - int(q["Start_Timestamp"]) for q in tl)
                print(f"rocprofv3, that kernel over the timed steps only: {len(tl)} launches, average "
                      f"{tot / len(tl) / 1e3:.2f} us")
    print("\nper-kernel rows:")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        print(f"  {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} us  {r['Name'][:110]}")


if __name__ == "__main__":
    main()
