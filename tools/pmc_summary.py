#!/usr/bin/env python3
"""Summarise rocprofv3 runs of one bench config into profiles/<tag>_pmc_<config>.json.

Input (tools/profile.sh): under DIR, one rocprofv3 output directory per pass:
  kt_<cfg>     --kernel-trace --stats            (kernel time)
  fetch_<cfg>  --pmc FETCH_SIZE                  (HBM read bytes, KiB per dispatch)
  write_<cfg>  --pmc WRITE_SIZE                  (HBM write bytes, KiB per dispatch)
  req_<cfg>    --pmc TCC_EA0_RDREQ{,_32B,_64B,_128B}_sum   (read requests by size)
  sq_<cfg>     --pmc SQ_* + GRBM_GUI_ACTIVE      (instruction mix, VALU busy)
Per-dispatch values are averaged over the engine kernel's dispatches of the bench's timed region:
the first --skip dispatches (the bench's warmup; for cfg 4 the first one inserts every flow) are
left out.  FETCH_SIZE is
also reported doubled (MI355X_MICROARCH.md: on gfx950 it counts 1/2 of wide streaming reads);
`bytes_per_launch` = doubled FETCH + WRITE, an upper estimate for this kernel's mixed-width
loads.  With the request-size pass, read bytes are counted exactly instead
(32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B, when those three partition RDREQ) and
`bytes_per_launch` is that + WRITE.  The summary is keyed to the kernel source hash, packets and vCPUs of the run, which is
how bench.py finds it.
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def col(r, *names):
    for n in names:
        if n in r:
            return r[n]
    raise KeyError(names)


def counters(d, kernel, skip=0, keep=None):
    """counter name -> mean over the kernel's dispatches (after the first `skip`) of the
    per-dispatch value"""
    per = {}
    for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
        if kernel not in col(r, "Kernel_Name", "Kernel-Name", "KernelName"):
            continue
        disp = col(r, "Dispatch_Id", "Dispatch-Id", "Correlation_Id")
        name = col(r, "Counter_Name", "Counter-Name")
        per.setdefault(name, {}).setdefault(disp, 0.0)
        per[name][disp] += float(col(r, "Counter_Value", "Counter-Value"))
    out = {}
    for k, v in per.items():
        vals = [v[d] for d in sorted(v, key=lambda x: int(x))][skip:]
        vals = vals[:keep] if keep else vals
        if vals:
            out[k] = sum(vals) / len(vals)
    return out


def kernel_stats(d, kernel, skip=0, keep=None):
    """rocprofv3's --stats line for the kernel (every dispatch), plus the mean / median of the
    per-dispatch durations of the kernel trace after the first `skip` dispatches (timed_*)"""
    out = None
    for r in rows(os.path.join(d, "**", "*kernel_stats.csv")):
        if r.get("Name") == kernel:
            out = {"calls": int(r["Calls"]), "all_avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                   "max_ns": float(r["MaxNs"])}
            break
    durs = []
    for r in rows(os.path.join(d, "**", "*kernel_trace.csv")):
        if col(r, "Kernel_Name", "Kernel-Name", "KernelName").startswith(kernel):
            durs.append((int(col(r, "Dispatch_Id", "Correlation_Id")), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    durs = [x for _, x in sorted(durs)][skip:]
    durs = durs[:keep] if keep else durs
    if out is not None and durs:
        srt = sorted(durs)
        out["timed_launches"] = len(durs)
        out["avg_ns"] = sum(durs) / len(durs)
        out["median_ns"] = float(srt[len(srt) // 2])
    elif out is not None:
        out["avg_ns"] = out["all_avg_ns"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--dir", required=True)
    ap.add_argument("--tag", default="r02")
    ap.add_argument("--kernel", default="mimic_jit_kernel")
    ap.add_argument("--packets", type=int, default=0)
    ap.add_argument("--vcpus", type=int, default=0)
    ap.add_argument("--out", default="")
    ap.add_argument("--command", default="")
    ap.add_argument("--skip", type=int, default=2, help="leading dispatches to leave out (the bench's warmup)")
    ap.add_argument("--keep", type=int, default=10, help="dispatches kept after --skip (the bench's timed steps; "
                                                         "its trailing per-batch step-count launches are left out)")
    ap.add_argument("--batches", type=int, default=0, help="batches the bench rotated over (0: its default)")
    ap.add_argument("--sched", default="interleaved")
    ap.add_argument("--per-launch", type=int, default=1, help="batches one launch ran (bench.py --many K)")
    ap.add_argument("--name", default="", help="the pass directories' suffix (default: the config)")
    ap.add_argument("--spread", action="store_true", help="the run used the spread kernel (its source hash)")
    ap.add_argument("--own", action="store_true", help="... in its owned form (engine 'spread_own')")
    a = ap.parse_args()
    import bench

    cfg = bench.CONFIGS[a.config]
    n = a.packets or cfg["packets"]
    vcpus = a.vcpus or cfg.get("vcpus") or max(64, n // 4)
    c = a.config
    nm = a.name or c
    ks = kernel_stats(os.path.join(a.dir, f"kt_{nm}"), a.kernel, a.skip, a.keep)
    fetch = counters(os.path.join(a.dir, f"fetch_{nm}"), a.kernel, a.skip, a.keep).get("FETCH_SIZE")
    write = counters(os.path.join(a.dir, f"write_{nm}"), a.kernel, a.skip, a.keep).get("WRITE_SIZE")
    sq = counters(os.path.join(a.dir, f"sq_{nm}"), a.kernel, a.skip, a.keep)
    req = counters(os.path.join(a.dir, f"req_{nm}"), a.kernel, a.skip, a.keep)
    out = {"config": c, "round": a.tag, "kernel": a.kernel,
           "kernel_src_hash": bench.kernel_src_hash_of(c, vcpus if (a.spread or a.own) else 0, a.own),
           "spread": a.spread or a.own, "spread_own": a.own,
           "packets": n, "vcpus": vcpus, "batches": a.batches or bench.default_batches(c, n),
           "schedule": a.sched, "batches_per_launch": a.per_launch, "kernel_stats": ks}
    if fetch is not None and write is not None:
        out["fetch_size_kib_per_launch"] = fetch
        out["write_size_kib_per_launch"] = write
        out["raw_bytes_per_launch"] = int((fetch + write) * 1024)
        out["bytes_per_launch"] = int((2 * fetch + write) * 1024)
        out["correction"] = ("FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 FETCH_SIZE counts 1/2 of wide "
                             "streaming reads); this kernel mixes 8-B and narrower loads, so true read bytes lie "
                             "between the raw and the doubled value")
    if req and fetch is not None and write is not None:
        g = lambda k: req.get(f"TCC_EA0_RDREQ{k}_sum", req.get(f"TCC_EA0_RDREQ{k}", 0.0))
        n_all, n32, n64, n128 = g(""), g("_32B"), g("_64B"), g("_128B")
        out["read_requests_per_launch"] = {"all": n_all, "32B": n32, "64B": n64, "128B": n128}
        rest = n_all - n32 - n64 - n128
        if n_all and abs(rest) <= 0.01 * n_all:   # the sizes partition the requests: exact read bytes
            rd = 32 * n32 + 64 * n64 + 128 * n128
            out["read_bytes_per_launch"] = int(rd)
            out["bytes_per_launch"] = int(rd + write * 1024)
            out["correction"] = ("read bytes from the request counts by size (TCC_EA0_RDREQ_32B/_64B/_128B); "
                                 "FETCH_SIZE tallies 128-byte requests at 64 B")
        else:
            out["read_requests_unpartitioned"] = rest
    if sq:
        out["sq_per_launch"] = sq
        waves = sq.get("SQ_WAVES") or 0
        if waves:
            out["sq_per_wave"] = {k: v / waves for k, v in sq.items() if k.startswith("SQ_") and k != "SQ_WAVES"}
        grbm = sq.get("GRBM_GUI_ACTIVE")
        if grbm and "SQ_ACTIVE_INST_VALU" in sq:
            # gfx94x VALUBusy formula (no gfx950 section in ROCm 7.2): SQ_ACTIVE_INST_VALU counts
            # quad-cycles; 1024 SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs
            out["valu_busy"] = round(sq["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (grbm / 8), 4)
        if sq.get("SQ_WAVE_CYCLES"):
            out["active_inst_frac_of_wave_cycles"] = round(sq.get("SQ_ACTIVE_INST_ANY", 0) / sq["SQ_WAVE_CYCLES"], 4)
    if a.command:
        out["command"] = a.command
    path = a.out or os.path.join(ROOT, "profiles", f"{a.tag}_pmc_{nm}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out)[:600])


if __name__ == "__main__":
    main()
