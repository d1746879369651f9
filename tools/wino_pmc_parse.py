import csv, glob, sys, collections
for tag in sys.argv[1:]:
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(f"gpurun_out/wpmc_{tag}/p*/run_counter_collection.csv")):
        rows = list(csv.DictReader(open(f)))
        # per dispatch sum counter values for conv kernels
        disp = collections.defaultdict(dict)
        for r in rows:
            if "conv" not in r["Kernel_Name"] or "pack" in r["Kernel_Name"] or "ktab" in r["Kernel_Name"]: continue
            d = r["Dispatch_Id"]; disp[d][r["Counter_Name"]] = disp[d].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
        ds = sorted(disp, key=int)[-3:]
        for d in ds:
            for k, v in disp[d].items(): vals[k].append(v)
    kt = list(csv.DictReader(open(glob.glob(f"gpurun_out/wpmc_{tag}/p1/run_kernel_trace.csv")[0])))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in kt if "conv" in r["Kernel_Name"] and "pack" not in r["Kernel_Name"]]
    print(tag, "kernel", [r["Kernel_Name"][:60] for r in kt if "conv" in r["Kernel_Name"]][-1], "us", [round(x,1) for x in durs[-3:]])
    v = {k: sum(x) / len(x) for k, x in vals.items()}
    for k in sorted(v): print(f"  {k:28s} {v[k]:.4g}")
    w = v.get("SQ_WAVES", 1)
    if "SQ_WAVE_CYCLES" in v:
        print("  per wave: cycles", v["SQ_WAVE_CYCLES"] / w * 4 if False else v["SQ_WAVE_CYCLES"] / w, "wait_any%", 100 * v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"], "wait_inst%", 100 * v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"], "active%", 100 * v["SQ_ACTIVE_INST_ANY"] / v["SQ_WAVE_CYCLES"])
    if "SQ_INSTS_MFMA" in v:
        print("  per wave: valu", v["SQ_INSTS_VALU"] / w, "mfma", v["SQ_INSTS_MFMA"] / w, "vmr", v["SQ_INSTS_VMEM_RD"] / w, "vmw", v["SQ_INSTS_VMEM_WR"] / w, "salu", v["SQ_INSTS_SALU"] / w)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in v and "SQ_BUSY_CYCLES" in v:
        print("  mfma busy / busy", v["SQ_VALU_MFMA_BUSY_CYCLES"] / v["SQ_BUSY_CYCLES"])
