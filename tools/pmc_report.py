#!/usr/bin/env python3
"""Per-layer PMC table from tools/pmc.sh output (the last SqueezeNet pass of each counter pass).
usage: python tools/pmc_report.py gpurun_out/pmc_TAG [--json profiles/pmc_traffic_f32.json]

--json writes the HBM traffic per launch of the conv kernel class (FETCH_SIZE x2 + WRITE_SIZE,
the guide's gfx950 correction), which bench.py reports as roofline.traffic."""
import csv
import glob
import os
import sys
from collections import OrderedDict, defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "onnx-rusty-inference-engine_amd"))
PER = 31  # set by main() from the kernel-name period of the trace


def layer_names(period):
    """Layer names per launched kernel: pool1 fused into conv1 (ORE_FUSE_CONV_POOL) and the f16
    input conversion change the count; decided from the trace's period."""
    from ore import onnx_wire, squeezenet
    m = onnx_wire.decode_model(squeezenet.build(224))
    names = [n.name for n in m.graph.node if n.op_type in ("Conv", "MaxPool", "GlobalAveragePool", "Softmax")]
    if period == len(names) + 1:
        names.insert(0, "to_nhwc")
    if period in (len(names) - 1, len(names)) and "pool1" in names and period == len(names) - 1:
        names[names.index("conv1")] = "conv1+pool1"
        names.remove("pool1")
    if period == len(names) - 1 and "to_nhwc" in names:  # f16 conversion + fused pool (not built)
        names.remove("to_nhwc")
    return names


def period_of(d):
    """Kernels per bench step from the repetition of the ore kernel names."""
    f = os.path.join(d, "run_counter_collection.csv")
    disp = OrderedDict()
    for r in csv.DictReader(open(f)):
        if ("ore::" in r["Kernel_Name"] or "_ZN3ore" in r["Kernel_Name"]) and "pack_" not in r["Kernel_Name"] and \
                "ktab" not in r["Kernel_Name"]:
            disp.setdefault(int(r["Dispatch_Id"]), r["Kernel_Name"])
    names = list(disp.values())
    for q in range(20, 40):
        if len(names) >= 2 * q and names[-q:] == names[-2 * q:-q]:
            return q
    return 31


def load(d):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        return None
    disp = OrderedDict()
    for r in csv.DictReader(open(f)):
        if ("ore::" not in r["Kernel_Name"] and "_ZN3ore" not in r["Kernel_Name"]) or "pack_" in r["Kernel_Name"] or \
                "ktab" in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"name": r["Kernel_Name"], "dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                "vgpr": r["VGPR_Count"], "agpr": r["Accum_VGPR_Count"], "grid": int(r["Grid_Size"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = list(disp.values())
    return rows[len(rows) - PER:]


def main():
    global PER
    base = sys.argv[1]
    json_out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    first = sorted(d for d in glob.glob(os.path.join(base, "p*")) if os.path.isdir(d))
    steps = None
    if os.path.exists(os.path.join(base, "steps.json")):  # bench.py --dump-steps: the plan's own names
        import json
        steps = json.load(open(os.path.join(base, "steps.json")))
        PER = len(steps)
        names = [s["name"] for s in steps]
    else:
        PER = period_of(first[0]) if first else 31
        names = layer_names(PER)
    merged = [defaultdict(float) for _ in range(PER)]
    for d in sorted(glob.glob(os.path.join(base, "p*"))):
        if not os.path.isdir(d):
            continue
        rows = load(d)
        if not rows:
            continue
        for i, r in enumerate(rows):
            for k, v in r.items():
                if k in ("name", "vgpr", "agpr"):
                    merged[i][k] = v
                elif k in ("dur", "grid"):
                    merged[i].setdefault(k, v)
                else:
                    merged[i][k] = v
    hdr = f"{'layer':22s} {'us':>7s} {'waves':>7s} {'valu/w':>7s} {'mfma/w':>7s} {'lds/w':>6s} {'vmr/w':>6s} {'vmw/w':>6s} {'mfma%':>6s} {'wait%':>6s} {'fetchMB':>8s} {'writeMB':>8s} {'GHz':>5s} {'v/a':>7s}"
    print(hdr)
    for i in range(PER):
        r = merged[i]
        w = max(r.get("SQ_WAVES", 1), 1)
        dur = r.get("dur", 1) / 1e3
        busy = r.get("GRBM_GUI_ACTIVE", 0)
        mf = r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        # MFMA busy fraction: busy cycles summed over SIMDs (1024 SIMDs) vs kernel cycles
        clk = busy / 8 if busy else dur * 1e3 * 2.1
        mfpct = 100.0 * mf / (1024 * clk) if clk else 0
        wc = r.get("SQ_WAVE_CYCLES", 0)
        waitpct = 100.0 * r.get("SQ_WAIT_ANY", 0) / wc if wc else 0
        hit, miss = r.get("TCC_HIT_sum", 0), r.get("TCC_MISS_sum", 0)
        print(f"{names[i]:22s} {dur:7.1f} {w:7.0f} {r.get('SQ_INSTS_VALU', 0) / w:7.0f} {r.get('SQ_INSTS_MFMA', 0) / w:7.0f} "
              f"{r.get('SQ_INSTS_LDS', 0) / w:6.0f} {r.get('SQ_INSTS_VMEM_RD', 0) / w:6.0f} {r.get('SQ_INSTS_VMEM_WR', 0) / w:6.0f} "
              f"{mfpct:6.1f} {waitpct:6.1f} {2 * r.get('FETCH_SIZE', 0) / 1024:8.1f} {r.get('WRITE_SIZE', 0) / 1024:8.1f} "
              f"{(busy / 8 / (dur * 1e3)) if busy else 0:5.2f} {r.get('vgpr', '')}/{r.get('agpr', '')}")
    if json_out:
        import json
        if steps:
            conv = [r for r, st in zip(merged, steps) if st["op"] == "Conv"]
        else:
            conv = [r for r in merged if "conv" in str(r.get("name", "")) or "fire_kernel" in str(r.get("name", ""))]
        fetch = sum(2 * r.get("FETCH_SIZE", 0) * 1024 for r in conv)  # KB -> B, x2 gfx950 correction
        write = sum(r.get("WRITE_SIZE", 0) * 1024 for r in conv)
        out = {"kernel_class": "conv", "launches": len(conv), "hbm_bytes_per_launch": (fetch + write) / max(len(conv), 1),
               "fetch_bytes_per_launch": fetch / max(len(conv), 1), "write_bytes_per_launch": write / max(len(conv), 1),
               "algorithmic_bytes_per_launch": (sum(st["bytes"] for st in steps if st["op"] == "Conv") / max(len(conv), 1)
                                                if steps else None),
               "source": base, "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, FETCH_SIZE x2 (gfx950)"}
        if steps:  # per launch, in the plan's step order (bench.py reports the dominant launch's traffic)
            out["per_step"] = [{"name": st["name"], "op": st["op"], "algorithmic_bytes": st["bytes"],
                                "hbm_bytes": 2 * r.get("FETCH_SIZE", 0) * 1024 + r.get("WRITE_SIZE", 0) * 1024,
                                "fetch_bytes": 2 * r.get("FETCH_SIZE", 0) * 1024, "write_bytes": r.get("WRITE_SIZE", 0) * 1024}
                               for r, st in zip(merged, steps)]
        for key, fn in (("lib_sha256", "lib.sha256"), ("commit", "commit")):  # the build the passes ran (tools/pmc.sh)
            if os.path.exists(os.path.join(base, fn)):
                out[key] = open(os.path.join(base, fn)).read().strip()
        with open(json_out, "w") as f:
            json.dump(out, f, indent=1)
        print(f"wrote {json_out}: {out['hbm_bytes_per_launch'] / 1e6:.1f} MB per conv launch")


if __name__ == "__main__":
    main()
