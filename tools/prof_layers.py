#!/usr/bin/env python3
"""Per-layer view of a rocprofv3 kernel trace of bench.py: the ore kernels of one step recur in
a fixed order, so dispatch i of the ore kernels belongs to graph step (i mod steps_per_pass).
Prints the median duration per step position with the layer's algorithmic FLOP and bytes at
batch B, the achieved TFLOP/s and GB/s, and `eff` = max(FLOP / mfma_peak, bytes / hbm) /
duration against the MEASURED peaks (profiles/r01_peaks.txt: f32 MFMA 143.5 TFLOP/s, f16 MFMA
2040 TFLOP/s; HBM 5.0 TB/s streaming).
usage: python tools/prof_layers.py gpurun_out/prof_xxx/run_kernel_trace.csv [batch] [--f16] [--passes N]"""
import csv
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "onnx-rusty-inference-engine_amd"))

HBM = 5.0e12


def geometry():
    """(name, kind, M, C, k, H_in, H_out) per launched layer of SqueezeNet-1.0 @224."""
    from ore import onnx_wire, squeezenet
    m = onnx_wire.decode_model(squeezenet.build(224))
    init = {t.name: t for t in m.graph.initializer}
    inp = m.graph.input[0].name
    C, HW = {inp: 3}, {inp: 224}
    out = []
    for n in m.graph.node:
        a = {at.name: at for at in n.attribute}
        if n.op_type == "Conv":
            w = list(init[n.input[1]].dims)
            x = n.input[0]
            k = w[2]
            pads = list(a["pads"].ints) if "pads" in a else [0] * 4
            s = list(a["strides"].ints)[0] if "strides" in a else 1
            ho = (HW[x] + pads[0] + pads[2] - k) // s + 1
            C[n.output[0]], HW[n.output[0]] = w[0], ho
            out.append((n.name, "conv", w[0], w[1], k, HW[x], ho))
        elif n.op_type == "MaxPool":
            x = n.input[0]
            pads = list(a["pads"].ints) if "pads" in a else [0] * 4
            ho = (HW[x] + pads[0] + pads[2] - 3) // 2 + 1
            C[n.output[0]], HW[n.output[0]] = C[x], ho
            out.append((n.name, "pool", C[x], C[x], 3, HW[x], ho))
        elif n.op_type == "Concat":
            C[n.output[0]], HW[n.output[0]] = C[n.input[0]] + C[n.input[1]], HW[n.input[0]]
        elif n.op_type in ("GlobalAveragePool", "Softmax"):
            x = n.input[0]
            out.append((n.name, "gap" if n.op_type == "GlobalAveragePool" else "softmax", C[x], C[x], 0, HW[x], 1))
            C[n.output[0]], HW[n.output[0]] = C[x], 1
        else:
            C[n.output[0]], HW[n.output[0]] = C.get(n.input[0]), HW.get(n.input[0])
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path = args[0]
    B = int(args[1]) if len(args) > 1 else 256
    f16 = "--f16" in sys.argv
    es = 2 if f16 else 4
    peak = 2040e12 if f16 else 143.5e12
    rows = [r for r in csv.DictReader(open(path))
            if ("ore::" in r["Kernel_Name"] or "_ZN3ore" in r["Kernel_Name"]) and "pack" not in r["Kernel_Name"] and "ktab" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    geo = geometry()
    if any("nchw_to_nhwc" in r["Kernel_Name"] for r in rows[-64:]):  # f16: the first conv's input conversion
        geo.insert(0, ("to_nhwc4", "cvt", 4, 3, 0, 224, 224))
    # kernels per pass from the period of the name sequence; one fewer than the layer list = pool1
    # fused into conv1 (ORE_FUSE_CONV_POOL)
    names = [r["Kernel_Name"] for r in rows]
    period = next((q for q in (len(geo), len(geo) - 1)
                   if len(names) >= 3 * q and names[-q:] == names[-2 * q:-q] == names[-3 * q:-2 * q]), len(geo))
    if period == len(geo) - 1:
        k1 = next(i for i, g in enumerate(geo) if g[0] == "conv1")
        name, kind, M, C, kk, H, Ho = geo[k1]
        pool = geo[k1 + 1]
        geo[k1] = ("conv1+pool1", "conv", M, C, kk, H, Ho, pool[6])
        del geo[k1 + 1]
    per = len(geo)
    n = len(rows) // per
    if "--passes" in sys.argv:
        n = min(n, int(sys.argv[sys.argv.index("--passes") + 1]))
    rows = rows[len(rows) - n * per:]
    agg = {}
    for i, r in enumerate(rows):
        agg.setdefault(i % per, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = tot_ideal = conv_t = conv_f = 0.0
    print(f"{'layer':22s} {'M':>5s} {'C':>4s} k {'H':>3s}->{'Ho':>3s} {'us':>8s} {'TF/s':>7s} {'GB/s':>6s} {'ideal':>7s} {'eff':>5s}  kernel")
    for k in range(per):
        ds = sorted(agg[k])
        d = ds[len(ds) // 2] / 1e3
        name, kind, M, C, kk, H, Ho = geo[k][:7]
        Hout = geo[k][7] if len(geo[k]) > 7 else Ho  # stored plane (the pooled one when fused)
        in_es = 4 if (k == 0 or kind in ("softmax", "cvt")) else es
        out_es = 4 if kind in ("gap", "softmax") else es
        if kind == "conv" and name.startswith("conv1") and geo[0][1] == "cvt":
            in_es, C = 2, 4  # reads the NHWC4 f16 copy
        fl = 2.0 * M * C * kk * kk * Ho * Ho * B if kind == "conv" else 0.0
        if name.startswith("conv1") and geo[0][1] == "cvt":
            fl = 2.0 * M * 3 * kk * kk * Ho * Ho * B
        by = B * (in_es * C * H * H + out_es * M * Hout * Hout)
        ideal = max(fl / peak, by / HBM) * 1e6
        tot += d
        tot_ideal += ideal
        if kind == "conv":
            conv_t += d
            conv_f += fl
        kn = rows[k]["Kernel_Name"].replace("void ore::", "").split("(")[0][:44]
        tf = f"{fl / d / 1e6:7.1f}" if fl else f"{'':7s}"
        print(f"{name:22s} {M:5d} {C:4d} {kk} {H:3d}->{Ho:3d} {d:8.1f} {tf} {by / d / 1e3:6.0f} {ideal:7.1f} {ideal / d:5.2f}  {kn}")
    print(f"sum of medians {tot / 1e3:.3f} ms over {n} passes; ideal {tot_ideal / 1e3:.3f} ms "
          f"(eff {tot_ideal / tot:.2f}); conv {conv_t / 1e3:.3f} ms = {conv_f / conv_t / 1e6:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
