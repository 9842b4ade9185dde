#!/usr/bin/env python3
"""Summarize a rocprofv3 run directory (scripts/profile.sh output) into profiles/<tag>/.

Writes:
  kernel_stats.csv      copy of the --kernel-trace --stats summary (avg duration per kernel)
  pmc_summary.json      per-launch PMC values of the named kernel + derived HBM traffic,
                        instruction mix and clock (gfx950 corrections per MI355X_MICROARCH.md)
  bench.json            the bench.py JSON line of the default run
"""
import argparse
import collections
import csv
import json
import os
import shutil

ap = argparse.ArgumentParser()
ap.add_argument("src", help="gpurun_out/<tag> directory")
ap.add_argument("dst", help="profiles/<tag> directory")
ap.add_argument("--kernel", default="otr_kernel<1, false, false, psg::NoHook, false>")
ap.add_argument("--process-rounds", type=float, default=1e7 * 64 * 20, help="process-rounds per launch")
ap.add_argument("--bytes-per-pr", type=float, default=24.0)
args = ap.parse_args()

os.makedirs(args.dst, exist_ok=True)
stats = os.path.join(args.src, "kt", "run_kernel_stats.csv")
avg_ns = None
if os.path.exists(stats):
    shutil.copy(stats, os.path.join(args.dst, "kernel_stats.csv"))
    for r in csv.DictReader(open(stats)):
        if args.kernel in r["Name"]:
            avg_ns = float(r["AverageNs"])

per = collections.defaultdict(list)
meta = {}
durs = []
for d in sorted(os.listdir(args.src)):
    f = os.path.join(args.src, d, "run_counter_collection.csv")
    if not d.startswith("pmc") or not os.path.exists(f):
        continue
    by_dispatch = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if args.kernel not in r["Kernel_Name"]:
            continue
        by_dispatch[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        by_dispatch[r["Dispatch_Id"]]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
                                  "SGPR_Count")}
    for disp, vals in by_dispatch.items():
        for k, v in vals.items():
            per[k].append(v)

avg = {k: sum(v) / len(v) for k, v in per.items()}
out = {"kernel": args.kernel, "kernel_trace_avg_ns": avg_ns, "dispatch_meta": meta,
       "pmc_per_launch": {k: v for k, v in avg.items() if not k.startswith("_")}}
if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    # FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE counts half of wide coalesced reads
    fetch = avg["FETCH_SIZE"] * 1024 * 2
    write = avg["WRITE_SIZE"] * 1024
    alg_bytes = args.process_rounds * args.bytes_per_pr
    dur = (avg_ns or avg.get("_dur")) / 1e9
    out["hbm"] = {
        "fetch_bytes_corrected": fetch,
        "write_bytes": write,
        "traffic_bytes": fetch + write,
        "traffic_GBps": (fetch + write) / dur / 1e9,
        "algorithmic_bytes": alg_bytes,  # SURVEY §8d streamed-state bookkeeping, not a bandwidth
        "traffic_over_algorithmic": (fetch + write) / alg_bytes,
        "note": "FETCH_SIZE doubled (gfx950 half-count of wide coalesced reads); reads here are 4 B/lane "
                "(uncalibrated width), so the read side is bounded by [FETCH_SIZE, 2*FETCH_SIZE]",
    }
if "GRBM_GUI_ACTIVE" in avg and avg_ns:
    out["clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / avg_ns
if "SQ_INSTS_VALU" in avg:
    inst_rounds = args.process_rounds / 64
    out["per_instance_round"] = {k: avg[k] / inst_rounds for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS")
                                 if k in avg}
    if avg_ns and "GRBM_GUI_ACTIVE" in avg:
        cycles = avg["GRBM_GUI_ACTIVE"] / 8
        out["issue_utilization"] = {
            "valu_of_1per2cyc_per_SIMD": avg["SQ_INSTS_VALU"] / (256 * 4 * cycles / 2),
            "salu_of_1per_cyc_per_CU": avg["SQ_INSTS_SALU"] / (256 * cycles),
        }
bench = os.path.join(args.src, "bench_default.log")
if os.path.exists(bench):
    for line in open(bench):
        if line.startswith("{"):
            b = json.loads(line)
            json.dump(b, open(os.path.join(args.dst, "bench.json"), "w"), indent=1)
            out["workload"] = {k: b["config"].get(k) for k in ("n", "rounds", "instances_per_gpu", "value_range")}
sha = os.path.join(args.src, "lib_sha256.txt")
if os.path.exists(sha):  # the libpsg.so the profile ran (bench.py checks it against its own)
    out["lib_sha256"] = open(sha).read().strip()
json.dump(out, open(os.path.join(args.dst, "pmc_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
