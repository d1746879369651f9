#!/usr/bin/env python3
"""Per-layer view of a rocprofv3 kernel trace of bench.py: the ore kernels of one step recur in
a fixed order, so dispatch i of the ore kernels belongs to graph step (i mod steps_per_pass).
Prints avg duration per step position with the step's algorithmic FLOP and bytes (B=256).
usage: python tools/prof_layers.py gpurun_out/prof_xxx/run_kernel_trace.csv [batch]"""
import csv
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "onnx-rusty-inference-engine_amd"))


def main():
    path = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    rows = [r for r in csv.DictReader(open(path)) if "ore::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    from ore import squeezenet, onnx_wire
    m = onnx_wire.decode_model(squeezenet.build(224))
    # kernels per pass: convs (relu fused), 3 pools, gap, softmax = 26 + 3 + 2 = 31
    per = 31
    n = len(rows) // per
    rows = rows[len(rows) - n * per:]
    names = []
    for node in m.graph.node:
        if node.op_type in ("Conv", "MaxPool", "GlobalAveragePool", "Softmax"):
            names.append(node.name)
    agg = {}
    for i, r in enumerate(rows):
        k = i % per
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg.setdefault(k, []).append(d)
    tot = 0.0
    for k in range(per):
        ds = sorted(agg[k])
        med = ds[len(ds) // 2] / 1e3
        tot += med
        kn = rows[k]["Kernel_Name"].replace("void ore::", "").replace("(ore::ConvParams)", "")[:48]
        print(f"{k:2d} {names[k] if k < len(names) else '?':24s} {kn:48s} {med:9.1f} us")
    print(f"sum of medians {tot / 1e3:.3f} ms over {n} passes")


if __name__ == "__main__":
    main()
