#!/usr/bin/env python3
"""Throughput of the other BASELINE.json configuration rows (the headline is bench.py).

  C3  LastVoting n=64, 1e8 instances over 8 GPUs (1.25e7 per GPU), 20 rounds, crash-stop
  C4  FloodMin n=256 crash-stop sweep f in {0,1,2,4,...,64}, R = f+2; KSetAgreement n=256, k=2, R=16,
      the same sweep over f
  C5  BenOr n=128, 64 rounds, |HO(p)| > n/2; termination-round histogram all-reduced
  W2  second-wave algorithms: OTR2, ShortLastVoting, KSetEarlyStopping, EpsilonConsensus

One process per GPU (torchrun), weak scaling, RCCL all-reduce of the summaries.
Prints one JSON line per configuration (rank 0). Algorithmic bytes per
process-round per SURVEY §8d: OTR 24, LV 42, FloodMin 8, KSet 70, BenOr 11 (W2 rows below).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (first: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402  (plan / launch_ranks / dry_run: the same launch logic as the headline)
from round_amd import abi  # noqa: E402
from round_amd import dist as rdist  # noqa: E402
from round_amd import psync  # noqa: E402

H = psync.HOSchedule
HBM_PEAK_GBS = 8000.0


def configs(scale):
    s = scale
    out = [("C3_lastvoting_n64", psync.LastVoting(), 64, int(12_500_000 * s), {}, 42)]
    for f in (0, 1, 2, 4, 8, 16, 32, 64):
        out.append((f"C4_floodmin_n256_f{f}", psync.FloodMin(f), 256, int(1_000_000 * s), {}, 8))
    for f in (0, 1, 2, 4, 8, 16, 32, 64):  # the same crash-stop sweep for KSet, R = 16
        out.append((f"C4_kset_n256_k2_f{f}", psync.KSetAgreement(2), 256, int(200_000 * s),
                    dict(schedule=H(drop_log2=0, good_round=0.0, crash_fmax=f)), 70))
    out.append(("C5_benor_n128", psync.BenOr(), 128, int(1_000_000 * s), {}, 11))
    # second-wave algorithms (not BASELINE configurations). B_alg by the
    # §8d recipe: (state read + written) + init. OTR2 = OTR; SLV (x, ts, vote, decision 4 B
    # + commit, decided 1 B) x 2 + 4; KSetEarlyStopping (est, lastNb, decision 4 B + canDecide,
    # decided 1 B) x 2 + 4; Epsilon n=64 (x, decision 8 B + maxR 4 B + halted-set 8 B +
    # decided 1 B) x 2 + init 8.
    out.append(("W2_otr2_n64", psync.OTR2(), 64, int(10_000_000 * s), dict(value_range=64), 24))
    out.append(("W2_slv_n64", psync.ShortLastVoting(), 64, int(12_500_000 * s), {}, 40))
    out.append(("W2_kset_es_n256_t64_k2", psync.KSetEarlyStopping(64, 2), 256, int(1_000_000 * s), {}, 32))
    out.append(("W2_epsilon_n64_f5", psync.EpsilonConsensus(5, 1e-6), 64, int(1_000_000 * s), {}, 66))
    # generic Spec programs: the reference Specs compiled from the Formula
    # DSL and interpreted on the device over the traced states (psg_run_batch_spec)
    from round_amd import formula
    out.append(("G1_otr_n64_specprog", psync.OTR(), 64, int(1_000_000 * s), dict(value_range=64), 24,
                lambda: formula.compile_spec(formula.otr_spec(), abi.PSG_ALG_OTR)))
    out.append(("G1_lv_n64_specprog", psync.LastVoting(), 64, int(250_000 * s), {}, 42,
                lambda: formula.compile_spec(formula.lv_spec(), abi.PSG_ALG_LAST_VOTING)))
    # the same Specs lowered to native wave code (formula.compile_native)
    out.append(("G1_otr_n64_native", psync.OTR(), 64, int(10_000_000 * s), dict(value_range=64), 24,
                lambda: formula.compile_native(formula.otr_spec(), abi.PSG_ALG_OTR)))
    out.append(("G1_lv_n64_native", psync.LastVoting(), 64, int(2_500_000 * s), {}, 42,
                lambda: formula.compile_native(formula.lv_spec(), abi.PSG_ALG_LAST_VOTING)))
    # ... and fused into the round kernel (one launch, Spec evaluated from registers, no trace)
    out.append(("G1_otr_n64_fused", psync.OTR(), 64, int(10_000_000 * s), dict(value_range=64), 24,
                lambda: formula.compile_native(formula.otr_spec(), abi.PSG_ALG_OTR, fused=True, n=64)))
    out.append(("G1_lv_n64_fused", psync.LastVoting(), 64, int(12_500_000 * s), {}, 42,
                lambda: formula.compile_native(formula.lv_spec(), abi.PSG_ALG_LAST_VOTING, fused=True, n=64)))
    # ... and the same Specs given as Formula text, lowered by the library itself
    # (psg_spec_compile_native: the JVM plugin's route, GpuSpec.compile(native = true))
    from round_amd import lib
    out.append(("G1_otr_n64_fused_text", psync.OTR(), 64, int(10_000_000 * s), dict(value_range=64), 24,
                lambda: lib.spec_compile_native(formula.to_text(formula.otr_spec()), abi.PSG_ALG_OTR, True, 64)))
    out.append(("G1_lv_n64_fused_text", psync.LastVoting(), 64, int(12_500_000 * s), {}, 42,
                lambda: lib.spec_compile_native(formula.to_text(formula.lv_spec()), abi.PSG_ALG_LAST_VOTING, True, 64)))
    return out


def parse(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); > 1 without torchrun starts them as a child torchrun")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=float, default=1.0, help="multiply the per-GPU instance counts")
    ap.add_argument("--only", default="", help="comma-separated name prefixes")
    ap.add_argument("--out", default="")
    ap.add_argument("--dry-run", action="store_true",
                    help="set up the ranks (gloo) and print the plan without touching a GPU")
    args = ap.parse_args(argv)
    args.device_list = ""  # bench.plan's field: ranks only here
    return args


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    # --gpus N really runs N ranks (bench.py's plan / launch logic), e.g. C3's
    # 1e8 LastVoting instances over 8 GPUs and C5's all-reduced histogram from one command
    mode, what = bench.plan(args, os.environ)
    if mode == "device-list":
        raise SystemExit("bench_configs.py runs ranks (--gpus N / torchrun), not device lists")
    if mode == "launch":
        sys.exit(bench.launch_ranks(argv, what, args.dry_run, script=__file__))
    if args.dry_run:
        return bench.dry_run(mode, what if mode == "ranks" else 1, int(os.environ.get("RANK", "0")), args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(dev)
    launched = "WORLD_SIZE" in os.environ  # torchrun: always go through RCCL, even at world size 1
    if launched:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
    results = []
    for row in configs(args.scale):
        name, alg, n, I, kw, balg = row[:6]
        spec = row[6]() if len(row) > 6 else None
        if args.only and not any(name.startswith(p) for p in args.only.split(",")):
            continue
        g = psync.GpuRound(alg, n, seed=7, device=dev, batch_capacity=I, **kw)
        begin, _ = rdist.shard(rank, world, I)
        g.load_inputs(begin, I)
        step = (lambda: g.run(begin, I)) if spec is None else (lambda: g.run_spec(begin, I, spec))
        for _ in range(args.warmup):
            step()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kns = 0
        last = None
        for _ in range(args.steps):
            last = step()
            kns += last.summary.kernel_ns
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = rdist.allreduce_max(time.perf_counter() - t0, device=f"cuda:{dev}")
        kern = rdist.allreduce_max(kns / args.steps / 1e9, device=f"cuda:{dev}")
        tot = rdist.allreduce_summary(last.summary, device=f"cuda:{dev}")
        R = g.cfg.rounds
        split = None
        names = alg.check_names
        if spec is None and "SafetyPredicate" in names:
            # a violation counts as a finding only while the Spec's safety predicate
            # still held on the effective HO sets (first_fail[target] < first_fail[SafetyPredicate],
            # as the adversary search scores it); the rest follow a predicate break. One extra,
            # untimed launch with the per-instance summaries.
            _, pi = g._ctx.run_batch_np(begin, I)
            ff = pi["first_fail"].astype(np.int64)
            sp = ff[:, names.index("SafetyPredicate")]
            cnt = []
            for k in alg.violation_slots:
                if names[k] == "SafetyPredicate":
                    continue
                bad = ff[:, k] != 255
                cnt += [int((bad & (ff[:, k] < sp)).sum()), int((bad & (ff[:, k] >= sp)).sum())]
            cnt.append(int((sp != 255).sum()))
            t = torch.tensor(cnt, dtype=torch.int64, device=f"cuda:{dev}")
            if world > 1:
                dist.all_reduce(t)
            cnt = t.cpu().tolist()
            split = {"instances_with_predicate_break": cnt[-1]}
            j = 0
            for k in alg.violation_slots:
                if names[k] == "SafetyPredicate":
                    continue
                split[names[k]] = {"under_predicate": cnt[j], "after_predicate_break": cnt[j + 1]}
                j += 2
        g.close()
        if rank == 0:
            vb = 8 if alg.real else 4  # Double values for EpsilonConsensus
            hbm_bytes = I * (n * (vb + vb + 1) + 24)
            th = [tot.term_hist[i] for i in range(R + 2)]
            done = sum(th[:-1])
            rec = {
                "config": name, "class": alg.class_name, "n": n, "rounds": R, "instances_per_gpu": I,
                "n_gpus": world,
                "value": tot.process_rounds * args.steps / dt, "unit": "checked process-rounds/s",
                "kernel_ms": kern * 1e3,
                # physical HBM bytes of one launch: initial values in, decide values /
                # rounds and instance summaries out; state stays on chip for all R rounds
                "hbm": {"bytes_per_launch": hbm_bytes, "achieved": hbm_bytes / kern / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": hbm_bytes / kern / 1e9 / HBM_PEAK_GBS},
                # SURVEY §8d's state bytes per process-round as if streamed every round (bookkeeping)
                "alg_bytes_per_process_round": balg,
                "process_rounds_active": tot.active_process_rounds,
                "instance_rounds_live": tot.live_instance_rounds,
                "violations": psync.BatchResult(alg, R, tot).violations(),
                "fail_count": psync.BatchResult(alg, R, tot).as_dict()["fail_count"],
                "spec": ("built-in" if spec is None else
                         "native lowered Formula (psg_run_batch_spec)" if spec.module_path else
                         "Formula bytecode interpreter (psg_run_batch_spec)"),
                "terminated_fraction": done / max(1, tot.instances),
                "mean_termination_round": (sum(i * c for i, c in enumerate(th[:-1])) / done) if done else None,
                "term_hist": th,
            }
            if split is not None:
                rec["violations_split"] = split
            results.append(rec)
            print(json.dumps(rec), flush=True)
    if rank == 0 and args.out:
        with open(args.out, "w") as f:
            json.dump(results, f, indent=1)
    if launched:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
