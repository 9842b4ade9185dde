#!/usr/bin/env python3
"""Per-kernel PMC summary of a scripts/pmc_wide.sh run (several kernels, one process each pass).

usage: summarize_pmc.py SRC DST --kernel 'NAME_SUBSTR[#k]=instances,rounds,n[,bytes_per_pr]' ...
(#k: only the k-th dispatch of that kernel in each pass, 0-based, e.g. one row of a sweep)

Writes DST/kernel_stats.csv (the --kernel-trace --stats summary) and DST/pmc_summary.json:
per kernel, the per-launch counters, the instruction mix per instance-round, the issue
utilisation of each pipe, the wave-cycle split (issuing / issue-stalled / parked), LDS
bank-conflict share and HBM traffic (gfx950 corrections as in summarize_profile.py:
FETCH_SIZE doubled, SQ_* cycle counters in quad-cycles, GRBM_GUI_ACTIVE summed over 8 XCDs).
"""
import argparse
import collections
import csv
import json
import os
import shutil

CUS = 256

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("dst")
ap.add_argument("--kernel", action="append", required=True)
args = ap.parse_args()

kernels = []
for spec in args.kernel:
    name, nums = spec.rsplit("=", 1)
    nth = None
    if "#" in name:
        name, k = name.rsplit("#", 1)
        nth = int(k)
    v = [float(x) for x in nums.split(",")]
    kernels.append((name, v[0], int(v[1]), int(v[2]), v[3] if len(v) > 3 else None, nth))
label = {id(k): k[0] + ("" if k[5] is None else f"#{k[5]}") for k in kernels}  # one entry per spec

os.makedirs(args.dst, exist_ok=True)
stats = os.path.join(args.src, "kt", "run_kernel_stats.csv")
avg_ns = {}
if os.path.exists(stats):
    shutil.copy(stats, os.path.join(args.dst, "kernel_stats.csv"))
    for r in csv.DictReader(open(stats)):
        for k in kernels:
            if k[0] in r["Name"] and k[5] is None:
                avg_ns[label[id(k)]] = float(r["AverageNs"])

# the nth dispatch of a kernel (name#k) is timed from the kernel-trace pass's own per-dispatch
# records (the same command, so the same dispatch sequence), never from the PMC passes'
# timestamps: counter collection stretches a dispatch (c10_pmc's KSet entry read 2.77 GHz)
trace = os.path.join(args.src, "kt", "run_kernel_trace.csv")
if os.path.exists(trace):
    rows = list(csv.DictReader(open(trace)))
    for k in kernels:
        if k[5] is None:
            continue
        ds = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if k[0] in r["Kernel_Name"]]
        if k[5] < len(ds):
            avg_ns[label[id(k)]] = float(ds[k[5]])

MAX_CLOCK_GHZ = 2.4  # MI355X peak engine clock: a derived clock above it means a wrong duration

per = {label[id(k)]: collections.defaultdict(list) for k in kernels}
meta = {}
for d in sorted(os.listdir(args.src)):
    f = os.path.join(args.src, d, "run_counter_collection.csv")
    if not d.startswith("pmc") or not os.path.exists(f):
        continue
    for k in kernels:
        by_dispatch = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if k[0] not in r["Kernel_Name"]:
                continue
            by_dispatch[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
            by_dispatch[r["Dispatch_Id"]]["_dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            meta[label[id(k)]] = {x: r[x] for x in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                            "Scratch_Size", "VGPR_Count", "SGPR_Count")}
        disp = [by_dispatch[d] for d in sorted(by_dispatch, key=int)]
        if k[5] is not None:
            disp = disp[k[5]:k[5] + 1]
        for vals in disp:
            for c, v in vals.items():
                per[label[id(k)]][c].append(v)

out = {}
for k in kernels:
    _, inst, R, n, bpr, _ = k
    name = label[id(k)]
    avg = {c: sum(v) / len(v) for c, v in per[name].items()}
    ns = avg_ns.get(name)  # kernel-trace duration only (None: no rates)
    W = (n + 63) // 64
    inst_rounds = inst * R
    o = {"dispatch": meta.get(name), "kernel_trace_avg_ns": avg_ns.get(name),
         "workload": {"instances": inst, "rounds": R, "n": n, "waves_per_instance": W,
                      "process_rounds": inst * R * n},
         "pmc_per_launch": {c: v for c, v in avg.items() if not c.startswith("_")}}
    if ns and "GRBM_GUI_ACTIVE" in avg and avg["GRBM_GUI_ACTIVE"] / 8 / ns > MAX_CLOCK_GHZ * 1.02:
        o["clock_error"] = (f"GRBM_GUI_ACTIVE / 8 / trace duration = {avg['GRBM_GUI_ACTIVE'] / 8 / ns:.2f} GHz "
                            f"> {MAX_CLOCK_GHZ} GHz: the duration does not belong to these counters; no rates")
        ns = None
    if ns and "GRBM_GUI_ACTIVE" in avg:
        cyc = avg["GRBM_GUI_ACTIVE"] / 8
        o["clock_GHz"] = cyc / ns
        o["issue_utilization"] = {
            "valu_of_1per2cyc_per_SIMD": avg.get("SQ_INSTS_VALU", 0) / (CUS * 4 * cyc / 2),
            "salu_of_1per_cyc_per_CU": avg.get("SQ_INSTS_SALU", 0) / (CUS * cyc),
            "lds_of_1per_cyc_per_CU": avg.get("SQ_INSTS_LDS", 0) / (CUS * cyc),
        }
        if "SQ_LDS_IDX_ACTIVE" in avg:
            # SQ_LDS_IDX_ACTIVE: LDS-array cycles summed over CUs (unit not calibrated on gfx950)
            o["issue_utilization"]["lds_array_busy_uncalibrated"] = avg["SQ_LDS_IDX_ACTIVE"] / (CUS * cyc)
    if "SQ_INSTS_VALU" in avg:
        o["per_instance_round"] = {c: avg[c] / inst_rounds for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS")
                                   if c in avg}
        o["per_instance_round_per_wave"] = {c: v / W for c, v in o["per_instance_round"].items()}
    if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_LDS_IDX_ACTIVE"):
        o["lds_bank_conflict_share"] = avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"]
    if "SQ_WAIT_ANY" in avg and "SQ_WAIT_INST_ANY" in avg and "SQ_ACTIVE_INST_ANY" in avg:
        tot = avg["SQ_WAIT_ANY"] + avg["SQ_WAIT_INST_ANY"] + avg["SQ_ACTIVE_INST_ANY"]
        o["wave_cycle_split"] = {
            "issuing (ACTIVE_INST_ANY)": avg["SQ_ACTIVE_INST_ANY"] / tot,
            "issue_stalled (WAIT_INST_ANY)": avg["SQ_WAIT_INST_ANY"] / tot,
            "of_which_lds_issue_stall (WAIT_INST_LDS)": avg.get("SQ_WAIT_INST_LDS", 0) / tot,
            "parked_waitcnt_or_barrier (WAIT_ANY)": avg["SQ_WAIT_ANY"] / tot,
        }
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg and ns:
        fetch = avg["FETCH_SIZE"] * 1024 * 2
        write = avg["WRITE_SIZE"] * 1024
        o["hbm"] = {"fetch_bytes_corrected": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
                    "traffic_GBps": (fetch + write) / ns}
        if bpr:
            alg = inst * R * n * bpr
            # SURVEY §8d's streamed-state bytes: bookkeeping (state stays on chip), never a rate
            o["hbm"].update({"algorithmic_bytes": alg, "traffic_over_algorithmic": (fetch + write) / alg})
    out[name] = o

json.dump(out, open(os.path.join(args.dst, "pmc_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
