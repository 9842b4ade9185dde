#!/usr/bin/env python3
"""Benchmark: checked process-rounds/s of OTR n=64 with every Spec check per round.

Workload (BASELINE.json configs[1]): OTR n=64, 1e7 instances x
20 rounds per GPU, seeded HO schedules (benign loss 1/8, good rounds 1/4),
initial values uniform in {1..V}; after every round the 3 invariants and the
Agreement/Validity/Integrity/Irrevocability properties (+ Termination round)
are evaluated. A step = one psg_run_batch over the GPU's instance shard with
its initial values already resident in HBM.

Multi-GPU: one process per GPU; rank r owns global instance ids [r*I, (r+1)*I)
(weak scaling); the per-batch int64 counters are all-reduced with RCCL
(torch.distributed backend "nccl"). `--gpus N` under torchrun uses the ranks it
was given; `--gpus N` (N > 1) started directly launches N ranks itself, as a
child `torch.distributed.run` started before anything touches the GPU.
`--device-list 0,1,...` instead runs ONE process whose psg context spans the
listed devices (psg_config.devices, one host thread per device — the JVM's route,
psync/runtime/Runtime.scala:43-57), I instances per device. Timing: barrier +
torch.cuda.synchronize() on both sides of exactly K steps, max over ranks.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# torch first: libpsg.so then binds to the HIP runtime torch loaded (one runtime per process)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from round_amd import dist as rdist  # noqa: E402
from round_amd import psync  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
CUS = 256  # MI355X compute units (8 XCDs x 32)
SPEC_CLOCK_GHZ = 2.4  # MI355X peak engine clock (MI355X_MICROARCH.md)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--instances", type=int, default=10_000_000, help="instances per GPU")
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--V", type=int, default=64, help="value-domain size of the headline line")
    ap.add_argument("--variants", default="2,4", help="other V values reported beside the headline")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--device-list", default="",
                    help="one process, one psg context over these HIP devices (e.g. 0,1,2,3)")
    ap.add_argument("--dry-run", action="store_true",
                    help="set up the ranks (gloo) and print the plan without touching a GPU")
    return ap.parse_args(argv)


def plan(args, env):
    """How this invocation runs: ("ranks", world) under torchrun (WORLD_SIZE set),
    ("launch", N) when --gpus N > 1 was asked without one (start N ranks as a child),
    ("device-list", devices) for a single multi-device context, else ("single", 1)."""
    if args.device_list:
        devs = [int(x) for x in args.device_list.split(",") if x.strip()]
        if not devs:
            raise SystemExit("--device-list needs at least one device")
        if "WORLD_SIZE" in env and int(env["WORLD_SIZE"]) > 1:
            raise SystemExit("--device-list runs one process; do not combine it with torchrun ranks")
        return "device-list", devs
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if args.gpus not in (1, world):
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting the {world} ranks",
                  file=sys.stderr)
        return "ranks", world
    if args.gpus > 1:
        return "launch", args.gpus
    return "single", 1


def launch_cmd(argv, nproc, port, script=None):
    """The child torchrun command line for `launch` mode (rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr", "127.0.0.1", f"--master-port={port}",
            os.path.abspath(script or __file__)] + list(argv)


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def visible_gpus(env=None):
    """GPUs the ranks can see, counted WITHOUT the HIP runtime (hipGetDeviceCount would
    initialise HSA in this parent and keep a KFD context open for the whole run): the
    *_VISIBLE_DEVICES list when one is set, else the KFD topology nodes that have SIMDs.
    None when neither is readable (the ranks then report a missing device themselves)."""
    env = os.environ if env is None else env
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if env.get(var, "").strip():
            return len([d for d in env[var].split(",") if d.strip()])
    nodes = "/sys/class/kfd/kfd/topology/nodes"
    try:
        count = 0
        for node in os.listdir(nodes):
            with open(os.path.join(nodes, node, "properties")) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            count += int(props.get("simd_count", "0")) > 0
        return count
    except OSError:
        return None


def launch_ranks(argv, nproc, dry_run, script=None):
    """Start `nproc` ranks of `script` (default: this file) as a child process and return its
    exit code. Nothing in this process touches the GPU: the device count comes from
    visible_gpus(), not from HIP."""
    if not dry_run:
        have = visible_gpus()
        if have is not None and have < nproc:
            raise SystemExit(f"bench.py: --gpus {nproc} needs {nproc} visible GPUs, {have} found "
                             "(--device-list runs several contexts in one process instead)")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(launch_cmd(argv, nproc, _free_port(), script), env=env)


def lib_sha256():
    import hashlib
    with open(os.path.join(ROOT, "round_amd", "libpsg.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_profile(args):
    """The newest committed PMC summary of otr_kernel<1> on this exact workload
    (profiles/*/pmc_summary.json, scripts/summarize_profile.py): HBM bytes per launch and
    instructions per instance-round, with whether it was taken on this very libpsg.so."""
    import glob
    try:
        sha = lib_sha256()
    except OSError:
        sha = None
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_summary.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        w = d.get("workload", {})
        if ("otr_kernel<1" in d.get("kernel", "") and "hbm" in d and "per_instance_round" in d
                and w.get("n") == args.n and w.get("rounds") == args.rounds
                and w.get("instances_per_gpu") == args.instances and w.get("value_range") == args.V):
            # a profile of this very build wins over any other; else the last in name order
            if best is None or best[2] is False or d.get("lib_sha256") == sha:
                best = (os.path.relpath(f, ROOT), d, sha is not None and d.get("lib_sha256") == sha)
    return best


def _cpu_quota():
    """CPUs granted by the cgroup (cpu.max), None when unlimited or unknown."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def _time_oracle(oracle, cfg, threads, target_s):
    cal = 100 * threads
    t0 = time.perf_counter()
    oracle.run(cfg, 0, cal, threads=threads)
    dt = time.perf_counter() - t0
    count = max(cal, int(cal * target_s / max(dt, 1e-3)))
    t0 = time.perf_counter()
    s, _, _ = oracle.run(cfg, 0, count, threads=threads)
    dt = time.perf_counter() - t0
    return s.process_rounds / dt, count, dt


def host_cores():
    """CPUs this process may really use: its affinity set, capped by the cgroup quota
    (a 256-CPU affinity set under a 16-CPU quota is 16 cores)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = _cpu_quota()
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    return cores, aff, quota


def cpu_baseline(cfg, target_s):
    """Time the oracle (C++ restatement of the reference's rounds + Spec, test
    infrastructure; not the JVM reference, which cannot run here) on the host: one
    thread per usable core (affinity capped by the cgroup quota), and one thread alone.
    SURVEY §8d / BASELINE.md §2 ask for both rates."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    cores, aff, quota = host_cores()
    v_all, n_all, t_all = _time_oracle(oracle, cfg, cores, target_s * 2 / 3)
    v_one, n_one, t_one = _time_oracle(oracle, cfg, 1, target_s / 3)
    return {
        "value": v_all,
        "unit": "process-rounds/s",
        "cores": cores,
        "threads": cores,
        "kind": "port",
        "sample": f"{n_all} instances of the same workload (ids 0..{n_all - 1}), oracle/psg_oracle.cpp, "
                  f"{cores} threads, {t_all:.1f} s",
        "single_core": {"value": v_one, "cores": 1, "threads": 1,
                        "sample": f"{n_one} instances (ids 0..{n_one - 1}), 1 thread, {t_one:.1f} s"},
        "affinity_cpus": aff,
        "cgroup_cpu_quota": quota,
        "note": "port = the build's C++ restatement of the reference (oracle/), not the JVM reference "
                "(no JVM in the image; parity with the JVM is unpinned, DESIGN §7); cores = "
                "min(affinity CPUs, cgroup quota)",
    }


def run_variant(rank, world, args, V, steps, warmup, devices=None):
    """One timed series. Under ranks: this rank's shard on its LOCAL_RANK device. With a
    device list: one context over `devices`, I instances per device."""
    dev = int(os.environ.get("LOCAL_RANK", 0))
    per = args.instances
    alg = psync.OTR()
    sched = psync.HOSchedule(drop_log2=3, good_round=0.25)
    if devices:
        begin, count = 0, per * len(devices)
        gr = psync.GpuRound(alg, args.n, rounds=args.rounds, seed=args.seed, schedule=sched, value_range=V,
                            devices=devices, batch_capacity=count)
    else:
        (begin, count) = rdist.shard(rank, world, per)
        gr = psync.GpuRound(alg, args.n, rounds=args.rounds, seed=args.seed, schedule=sched, value_range=V,
                            device=dev, batch_capacity=count)
    gr.load_inputs(begin, count)  # inputs resident in HBM before timing
    for _ in range(warmup):
        gr.run(begin, count)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kns = 0
    last = None
    for _ in range(steps):
        last = gr.run(begin, count)
        kns += last.summary.kernel_ns
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    # node-level result: all-reduce (sum) the int64 counters over RCCL; max of the clocks
    cuda = f"cuda:{dev}"
    total = rdist.allreduce_summary(last.summary, device=cuda)
    dt_max = rdist.allreduce_max(dt, device=cuda)
    my_kernel_s = kns / max(steps, 1) / 1e9
    per_rank = rdist.allgather_float(my_kernel_s, rank, world, device=cuda)
    cfg = gr.cfg
    gr.close()
    return {"summary": total, "dt": dt_max, "kernel_s": max(per_rank), "per_rank_kernel_s": per_rank, "cfg": cfg}


def parallelism_label(mode, world, devices, instances):
    """What ran, stated truthfully: RCCL is named only when a process group exists (torchrun
    ranks, world size 1 included); a directly started single process has no collective."""
    if mode == "device-list":
        return f"one context over devices {devices} (psg_config.devices), {instances} instances each, no collective"
    if mode == "ranks":
        return f"instance-sharded x{world} ranks (RCCL all-reduce of counters)"
    return "single process, no collective"


def dry_run(mode, world, rank, args):
    """--dry-run: the ranks exist and can all-reduce (gloo), nothing touches a GPU."""
    if mode == "ranks":
        dist.init_process_group("gloo")
        t = torch.ones(1)
        dist.all_reduce(t)
        seen = int(t.item())
        dist.destroy_process_group()
    else:
        seen = 1
    if rank == 0:
        print(json.dumps({"dry_run": True, "mode": mode, "world": world, "ranks_seen": seen,
                          "n_gpus": world if mode != "device-list" else len(args.device_list.split(","))}),
              flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    mode, what = plan(args, os.environ)
    if mode == "launch":  # N ranks as a child torchrun, before any GPU call here
        sys.exit(launch_ranks(argv, what, args.dry_run))
    world = what if mode == "ranks" else 1
    devices = what if mode == "device-list" else None
    rank = int(os.environ.get("RANK", "0"))
    if args.dry_run:
        return dry_run(mode, world, rank, args)
    dev = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(dev)
    launched = mode == "ranks"  # torchrun: always go through RCCL, even at world size 1
    if launched:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
    n_gpus = len(devices) if devices else world
    head = run_variant(rank, world, args, args.V, args.steps, args.warmup, devices)
    variants = {}
    for v in [int(x) for x in args.variants.split(",") if x]:
        r = run_variant(rank, world, args, v, max(1, args.steps // 2), 1, devices)
        pr = r["summary"].process_rounds * max(1, args.steps // 2)
        variants[f"V={v}"] = {"value": pr / r["dt"], "kernel_ms": r["kernel_s"] * 1e3,
                              "violations": psync.BatchResult(psync.OTR(), args.rounds, r["summary"]).violations()}
    if rank == 0:
        s = head["summary"]
        steps = args.steps
        pr_per_step = s.process_rounds  # all ranks / devices, one step
        value = pr_per_step * steps / head["dt"]
        per_launch_pr = args.instances * args.n * args.rounds  # one GPU's launch
        inst_rounds = args.instances * args.rounds
        # physical HBM bytes of one launch: the initial values read once (int32 per
        # process), the results written once (decide value int32 + decide round u8 per process,
        # a 24-B summary per instance); process state stays on chip for all R rounds
        hbm_bytes = args.instances * (args.n * (4 + 4 + 1) + 24)
        hbm_gbs = hbm_bytes / head["kernel_s"] / 1e9
        par = parallelism_label(mode, world, devices, args.instances)
        out = {
            "metric": "checked process-rounds/sec (node), OTR n=64 w/ invariants; % HBM peak",
            "value": value,
            "unit": "process-rounds/s",
            "n_gpus": n_gpus,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": head["dt"] / steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: seeded Philox4x32-10 HO schedules and initial values",
            "config": {
                "workload": f"OTR n={args.n}, {args.instances} instances/GPU x {args.rounds} rounds, V={args.V}, "
                            "drop 1/8, good-round 1/4; 3 invariants + Agreement/Validity/Integrity/"
                            "Irrevocability + Termination evaluated after every round",
                "alg": "example.OTR",
                "n": args.n,
                "rounds": args.rounds,
                "instances_per_gpu": args.instances,
                "value_range": args.V,
                "parallelism": par,
            },
            "per_gpu_kernel_ms": [x * 1e3 for x in head["per_rank_kernel_s"]] if not devices else None,
            "roofline": {
                # the fused kernel keeps process state on chip (real HBM traffic ~2 % of the
                # algorithmic bytes): its binding resource is instruction issue
                "bound": "issue",
                "achieved": None,
                "peak": None,
                "unit": "G SALU instructions/s",
                "frac": None,
                "traffic": None,
                "kernel": "psg::otr_kernel<1, false, false, psg::NoHook, false>",  # <W, OTR2, explicit schedule, hook, trace>
                "kernel_ms": head["kernel_s"] * 1e3,
                "hbm": {
                    "model": "per launch: init values in (4 B/process) + decide values and rounds out "
                             "(5 B/process) + instance summaries (24 B/instance); state stays in VGPRs",
                    "bytes_per_launch": hbm_bytes, "achieved": hbm_gbs, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": hbm_gbs / HBM_PEAK_GBS},
            },
            "checks": {
                "violations": psync.BatchResult(psync.OTR(), args.rounds, s).violations(),
                "termination_hist": [s.term_hist[i] for i in range(args.rounds + 2)],
                "decided_processes": s.decided_processes,
                # counted = n*R per instance; active = rounds a process took a step in;
                # check-only = instance-rounds after every process halted (Spec evaluated only)
                "process_rounds_counted": s.process_rounds,
                "process_rounds_active": s.active_process_rounds,
                "instance_rounds_live": s.live_instance_rounds,
                "instance_rounds_check_only": s.instances * args.rounds - s.live_instance_rounds,
                # the same wall time over the process-rounds in which a process took a step
                "active_rate": s.active_process_rounds * steps / head["dt"],
                "active_rate_unit": "active process-rounds/s",
            },
            "variants": variants,
        }
        prof = pmc_profile(args)
        if prof is not None:
            src, d, same = prof
            rl = out["roofline"]
            # live rate of this run: the profile's instructions per instance-round (a property of
            # the code, valid only for the libpsg.so it was taken on) x the launch's
            # instance-rounds / this run's kernel time; peak: one instruction per CU per cycle
            # (SALU) / per SIMD per 2 cycles (VALU, wave64 on a 32-lane SIMD) at the 2.4 GHz
            # spec clock (the profile's measured clock is reported beside it, labelled)
            ipr = d["per_instance_round"]
            clk = SPEC_CLOCK_GHZ
            salu = ipr["SQ_INSTS_SALU"] * inst_rounds / head["kernel_s"] / 1e9
            valu = ipr["SQ_INSTS_VALU"] * inst_rounds / head["kernel_s"] / 1e9
            pk_s, pk_v = CUS * clk, CUS * 4 * clk / 2
            pipe = "SALU" if salu / pk_s >= valu / pk_v else "VALU"
            rl["profile"] = src
            rl["profile_matches_build"] = same
            rl["profile_issue_utilization"] = d.get("issue_utilization")
            if same:
                rl.update({"pipe": pipe, "achieved": salu if pipe == "SALU" else valu,
                           "peak": pk_s if pipe == "SALU" else pk_v, "unit": f"G {pipe} instructions/s"})
                rl["frac"] = rl["achieved"] / rl["peak"]
                mclk = d.get("clock_GHz")
                if mclk:
                    rl["measured_clock"] = {"clock_GHz": mclk, "peak": rl["peak"] * mclk / clk,
                                            "frac": rl["achieved"] / (rl["peak"] * mclk / clk),
                                            "note": "the same rate against the profile's measured clock"}
                rl["valu"] = {"achieved": valu, "peak": pk_v, "frac": valu / pk_v, "unit": "G VALU instructions/s"}
                rl["salu"] = {"achieved": salu, "peak": pk_s, "frac": salu / pk_s, "unit": "G SALU instructions/s"}
                rl["insts_per_instance_round"] = ipr
                rl["traffic"] = d["hbm"]["traffic_bytes"] / head["kernel_s"] / 1e9
                rl["traffic_unit"] = "GB/s"
                rl["traffic_bytes_per_launch"] = d["hbm"]["traffic_bytes"]
                rl["traffic_source"] = src + " (PMC FETCH_SIZE*2 + WRITE_SIZE per launch)"
                rl["hbm"]["pmc_over_model"] = d["hbm"]["traffic_bytes"] / hbm_bytes
            else:
                # counters of another build say nothing about this one's rates
                rl["stale_profile"] = "profile taken on a different libpsg.so: achieved / frac / traffic " \
                                      "left null; profile_issue_utilization is that build's own figure"
        if not args.no_cpu_baseline and n_gpus == 1:  # the host baseline is an N = 1 figure
            out["cpu_baseline"] = cpu_baseline(head["cfg"], args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if launched:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
