import csv, json, sys, glob
tag = sys.argv[1]
for l in open(f"gpurun_out/{tag}/bench.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"]["vcpus_per_gpu"], d["config"]["workload"][:12], "Mpkt/s", d["value"], "launch_ms", d["roofline"]["avg_launch_ms"],
              "Ginsn/s", round(d["insns_per_s"] / 1e9, 1), "ok", d["status_ok_frac"], d["counters_sum"])
for f in sorted(glob.glob(f"gpurun_out/{tag}/pmc_*/a_counter_collection.csv")):
    agg = {}
    for r in csv.DictReader(open(f)):
        if "mimic_xdp" in r["Kernel_Name"]:
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    a = {k: sum(v) / len(v) for k, v in agg.items()}
    w = a.get("SQ_WAVES", 1)
    print(f.split("/")[-2], {k: round(v / w, 1) for k, v in a.items() if k != "SQ_WAVES"}, "per wave")
