#!/usr/bin/env python3
"""Batched trust-region SQP benchmark (BASELINE.json metric).

A "step" is one sco::BasicTrustRegionSQP::optimize of every problem in the
per-GPU batch, run by one fused HIP launch from inputs already resident in
HBM.  The default workload is BASELINE.json configs[2] (config C): 7-DoF PR2
arm, 30 waypoints, JointVel + 29 CartPose costs + the LVS-discrete collision
cost against a 10-primitive scene, 1024 problems per GPU.  `value` is SQP
(outer) iterations per second summed over all problems of all ranks
(SURVEY.md §8d).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 1024]
    python bench.py --config HB --batch 256     (host-loop workload, see main_hostloop)
    python bench.py --config HA                 (config B + JointAcc cost: the fused kernel's
                                                 waypoint-pair solve)

Batches in flight: the runtime keeps `--inflight` (default 3) batch contexts,
each with its own HIP stream, and submits step k to context k mod inflight,
so the next batch's problems fill the CUs that the current batch's last
(longest) problems leave idle.  Every step still solves a full batch of
`--batch` problems from its own HBM-resident inputs; `batch_latency_ms` is one
batch alone (no overlap), measured before the timed region.

Multi-GPU: one process per GPU (torchrun); every rank solves its own
contiguous shard of problem seeds (weak scaling, no data-path collective); a
gloo barrier brackets the timed region and the max elapsed time over ranks is
reported.

Extra JSON objects:
  roofline      algorithmic HBM bytes of sqp_kernel (SURVEY.md §8d B_iter
                model, counters read back from the device) / its HIP-event
                duration, against the 8 TB/s HBM3E peak; beside it the same
                bytes over the timed region (achieved_per_step_gbs), the
                PMC-measured traffic rate (measured_gbs) and what actually
                limits the kernel (limiter).
  cpu_baseline  the oracle's CPU restatement (oracle/, "port") on a bounded
                sample of the same problems, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "trajopt-1_amd"))

import numpy as np  # noqa: E402

from trajopt_amd import abi, problems, sharding  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md


def workload_name(wl, config, batch):
    terms = f"JointVel + {wl.desc.n_cart} CartPose ABS costs"
    if wl.desc.n_jdt:
        terms += " + JointAcc cost (joint_costs_unit; waypoint-pair solve)"
    if wl.desc.coll_enabled:
        ev = {0: "LVS-discrete", 1: "LVS-continuous", 2: "discrete"}[wl.desc.coll_continuous]
        terms += f" + {ev} collision cost ({wl.desc.n_prims}-primitive scene)"
    robot = "14-DoF PR2 dual arm" if wl.n_dof == 14 else f"{wl.n_dof}-DoF PR2 arm"
    return (f"config {config}: {robot} x {wl.n_steps} waypoints, {terms}, batch {batch} per GPU "
            "(BasicTrustRegionSQP + OSQP-semantics ADMM/polish)")


def algorithmic_bytes(wl, results):
    """B_iter = fixed + k * per_admm + s * 16 nnz(L) per problem
    per SQP iteration; summed over the batch it needs only the per-problem
    totals of SQP iterations, ADMM iterations and KKT solves."""
    N, D = wl.n_steps, wl.n_dof
    nx = N * D
    R = 6 * wl.desc.n_cart
    n = nx + 2 * R
    m = R + D * wl.desc.n_fixed + n
    nnz_a = R * (D + 2) + D * wl.desc.n_fixed + n
    nnz_p = nx + (N - 1) * D
    nnz_l = N * D * (D + 1) // 2 + (N - 1) * D * D  # block-tridiagonal Cholesky factor
    if wl.desc.n_jdt:
        # JointAccEqCost: P couples t and t + 2; the factor is block-tridiagonal over
        # waypoint pairs (N / 2 blocks of 2 D)
        nnz_p += (N - 2) * D
        G, sD = N // 2, 2 * D
        nnz_l = G * sD * (sD + 1) // 2 + (G - 1) * sD * sD
    fixed = 2 * 8 * nx + 8 * R * (1 + D) + 96 * wl.desc.n_cart + 2 * 8 * (n + 2 * m + R * (D + 2))
    per_admm = 2 * 12 * nnz_a + 24 * nnz_p + 8 * (3 * n + 7 * m)
    refine = wl.desc.osqp.polish_refine_iter
    # config C (§8d): per contact row 8*(1 + 14) when built and 2*12*16 per
    # ADMM iteration; 10 primitives x 16 doubles read per sub-state pass
    row_b, admm_b, sub_b = 8 * (1 + 2 * D), 2 * 12 * (2 * D + 2), 8 * 16 * wl.desc.n_prims
    total = 0
    for r in results:
        kkt_solves = r.n_admm_iters + r.n_qp_solves * (1 + refine)
        total += fixed * r.n_sqp_iters + per_admm * r.n_admm_iters + 16 * nnz_l * kkt_solves
        total += row_b * r.n_contact_rows + admm_b * r.n_hinge_admm + sub_b * r.n_substates
    return total, {"fixed": fixed, "per_admm": per_admm, "nnz_L": nnz_l, "per_contact_row": row_b,
                   "per_contact_admm": admm_b, "per_substate": sub_b}


def measured_traffic(workload_name, batch):
    """HBM bytes per sqp_kernel launch from the newest committed PMC summary
    (profiles/*_pmc_hbm.json, tools/collect_profiles.sh) for this workload."""
    best = None
    for p in sorted((ROOT / "profiles").glob("*_pmc_hbm.json")):
        try:
            d = json.loads(p.read_text())
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload_name and d.get("batch_per_gpu") == batch:
            best = (p.name, d)
    if best is None:
        return None, None
    return best[1]["hbm_bytes_per_launch"], best[0]


def host_cpus():
    """(CPUs this process may use, host nproc, CPU model, cgroup CPU quota).
    The usable count is the scheduler affinity capped by the cgroup quota
    (cpu.max), so a container that sees the whole machine but is limited to a
    share of it reports the share."""
    nproc = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = nproc
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
            usable = max(1, min(usable, int(quota)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for ln in Path("/proc/cpuinfo").read_text().splitlines():
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return usable, nproc, model, quota


def cpu_baseline(config, n_problems, threads):
    """The oracle (CPU restatement of the reference path) timed on a bounded
    sample of the same problems: its -O3 FMA build for the host's ISA level
    (oracle/Makefile liboracle_fast_*), one problem per thread on every CPU the
    process may use, plus the one-thread latency of one problem."""
    sys.path.insert(0, str(ROOT))
    from oracle import oracle  # checker / baseline only

    usable, nproc, model, quota = host_cpus()
    threads = usable if threads <= 0 else threads
    n = n_problems if n_problems > 0 else min(1024, max(128, 2 * threads))
    wl = problems.make_workload(config, n)
    t0 = time.perf_counter()
    _, res = oracle.solve(wl, n_threads=threads, variant="fast")
    dt = time.perf_counter() - t0
    iters = sum(r.n_sqp_iters for r in res)
    one = problems.make_workload(config, 1)
    t1 = time.perf_counter()
    _, r1 = oracle.solve(one, n_threads=1, variant="fast")
    lat = time.perf_counter() - t1
    return {
        "value": iters / dt,
        "unit": "SQP iters/s",
        "cores": threads,
        "kind": "port",
        "sample": f"first {n} problems of the same workload (seeds 20261015+b), {iters} SQP iterations in "
                  f"{dt:.1f} s, one problem per thread on {threads} threads",
        "build": oracle.variant_path("fast").name + " (g++ -O3 -ffp-contract=fast, x86-64-v3/v4 by host ISA)",
        "host_nproc": nproc,
        "host_cpu_model": model,
        "cgroup_cpu_quota": quota,
        "single_problem_latency_s": lat,
        "single_problem_sqp_iters": r1[0].n_sqp_iters,
        "single_thread_sqp_iters_per_s": r1[0].n_sqp_iters / lat,
    }


def latency_model(config):
    """The newest committed critical-path model of the kernel (profiles/*_latency_<config>.json,
    tools/latency_model.py): cycles per ADMM iteration on the serial path against the measured."""
    best = None
    for p in sorted((ROOT / "profiles").glob(f"*_latency_{config}.json")):
        try:
            best = json.loads(p.read_text()) | {"source": p.name}
        except (OSError, ValueError):
            continue
    return best


def pmc_evidence(config):
    """The newest committed counter summary of sqp_kernel (profiles/*_pmc_<config>.json,
    tools/pmc_latency.sh): where the wave cycles go."""
    best = None
    for p in sorted((ROOT / "profiles").glob(f"*_pmc_{config}.json")):
        try:
            d = json.loads(p.read_text())
        except (OSError, ValueError):
            continue
        if "wave_cycle_split" in d:
            best = {"source": p.name, "wave_cycle_split": d["wave_cycle_split"],
                    "lds_bank_conflict_share": d.get("lds_bank_conflict_share"),
                    "measured_hbm_gbs": d.get("measured_hbm_gbs")}
    return best


HOSTLOOP_BASE = "B"  # bench --config HB: config B's problems + JointAcc and JointJerk costs


def hostloop_workload_name(wl, batch):
    return (f"config HB: {wl.n_dof}-DoF PR2 arm x {wl.n_steps} waypoints, JointVel + {wl.desc.n_cart} CartPose "
            f"ABS costs (config {HOSTLOOP_BASE}) + JointAcc + JointJerk costs (joint_costs_unit), batch {batch} per GPU "
            "(host BasicTrustRegionSQP loops, GpuModel QPs batched one launch per round)")


def hostloop_oracle_workload(texts):
    """The lowered JSON problems as one oracle Workload (every problem of a
    config HB batch lowers to the same description; the targets and initial
    trajectories differ)."""
    from trajopt_amd import host
    from trajopt_amd.problems import Workload

    low = [host.lower_json(t) for t in texts]
    desc = low[0][0]
    return Workload("HB", desc, np.stack([v[1] for v in low]), np.stack([v[2] for v in low]),
                    np.zeros((len(texts), 0, 16)), np.stack([v[1] for v in low]), None)


def main_hostloop(args, world, rank, local_rank, json_out):
    """bench.py --config HB: problems the fused kernel does not lower, solved by
    the C++ host loops (one per problem, all at once) whose QP rounds go to the
    device as one qp_csc launch per pattern (sco::GpuQPBatcher).  A step is one
    prepared batch (thost_batch_create: parse, lower, device set-up, outside the
    timed region) solved to convergence; each step solves fresh copies of the
    same problems.  roofline: the QP solver's algorithmic bytes
    (GpuQPBatcher::bytes) over the wall time inside its launches."""
    import torch
    import torch.distributed as dist

    from trajopt_amd import host

    abi.load_hip()
    if world > 1:
        dist.init_process_group("gloo")
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    wl = sharding.rank_workload(HOSTLOOP_BASE, args.batch, rank)
    texts = [host.hostloop_workload_json(wl, b) for b in range(args.batch)]
    batches = [host.PreparedBatch(texts, device=device) for _ in range(args.warmup + args.steps)]
    if not batches[0].stats()["host_loops"]:
        raise SystemExit("config HB lowered onto the fused kernel: it must run the host loops")
    res0 = None
    for k in range(args.warmup):
        _, res0 = batches[k].solve()
    barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = [batches[args.warmup + k].solve() for k in range(args.steps)]
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    res_last = outs[-1][1]
    for _, r in outs[:-1] + ([(None, res0)] if res0 is not None else []):
        if any(a.n_sqp_iters != b.n_sqp_iters or a.n_admm_iters != b.n_admm_iters for a, b in zip(r, res_last)):
            raise SystemExit("non-deterministic SQP counters between steps")
    st = [batches[args.warmup + k].stats() for k in range(args.steps)]
    iters_local = sum(r.n_sqp_iters for r in res_last)
    elapsed, iters_total = sharding.reduce_step_stats(elapsed, iters_local, world)
    if rank == 0:
        qp_bytes = float(np.mean([s["qp_bytes"] for s in st]))
        qp_s = float(np.mean([s["qp_seconds"] for s in st]))
        launches = float(np.mean([s["qp_launches"] for s in st]))
        achieved = qp_bytes / qp_s / 1e9
        out = {
            "metric": "SQP iters/sec + achieved HBM GB/s, 7-DoF x 30-wpt host-loop batch (JointAcc/Jerk, not lowered)",
            "value": iters_total * args.steps / elapsed,
            "unit": "SQP iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (config {HOSTLOOP_BASE} seeds 20261015+b written as TrajOptRequest JSON, + JointAcc + JointJerk)",
            "config": {
                "workload": hostloop_workload_name(wl, args.batch),
                "batch_per_gpu": args.batch,
                "global_batch": args.batch * world,
                "sqp_iters_per_step": iters_total,
                "qp_solves_per_step_rank0": sum(r.n_qp_solves for r in res_last),
                "admm_iters_per_step_rank0": sum(r.n_admm_iters for r in res_last),
                "qp_launches_per_step": launches,
                "parallelism": f"shard{world} (independent problems, no collective)",
            },
            "roofline": {
                # the host loops' QP rounds: one qp_csc_group_kernel launch per
                # round of the batch (a workgroup per QP, sparse LDL^T KKT + ADMM);
                # `achieved` is ALGORITHMIC bytes (the GpuQPBatcher model, which
                # leaves out the factor of a pattern staged in LDS) over the wall
                # time inside the rounds (staging, H2D, launch, D2H) -- not
                # measured HBM traffic
                "bound": "hbm",
                "limiter": "latency",
                "kernel": "thip::qp_csc_group_kernel",
                "achieved_kind": "algorithmic bytes / round wall time",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": None,
                "qp_launch_share_of_step": qp_s / (elapsed / args.steps),
                "algorithmic_bytes_per_step": qp_bytes,
                "qp_seconds_per_step": qp_s,
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu:
            sys.path.insert(0, str(ROOT))
            from oracle import oracle  # checker / baseline only

            usable, nproc, model, _ = host_cpus()
            threads = usable if args.cpu_threads <= 0 else args.cpu_threads
            n = min(args.batch, args.cpu_problems if args.cpu_problems > 0 else max(128, 4 * threads))
            owl = hostloop_oracle_workload(texts[:n])
            t1 = time.perf_counter()
            _, ores = oracle.solve(owl, n_threads=threads, variant="fast")
            dt = time.perf_counter() - t1
            it = sum(r.n_sqp_iters for r in ores)
            out["cpu_baseline"] = {
                "value": it / dt, "unit": "SQP iters/s", "cores": threads, "kind": "port",
                "sample": f"first {n} problems of the same batch, {it} SQP iterations in {dt:.1f} s, one problem "
                          f"per thread on {threads} threads",
                "host_nproc": nproc, "host_cpu_model": model,
            }
        print(json.dumps(out), file=json_out, flush=True)
    for b in batches:
        b.close()
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1024, help="problems per GPU")
    ap.add_argument("--config", default="C")
    ap.add_argument("--inflight", type=int, default=3, help="batch contexts (streams) in flight")
    ap.add_argument("--cpu-problems", type=int, default=0, help="0: max(128, 2 x threads), at most 1024")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every CPU this process may use")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--diag-util", action="store_true",
                    help="diagnostic: per-problem cycle/wall counters over the timed steps (phase timers on; "
                         "~1 %% slower) -> CU utilisation and shader clock on stderr")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")

    # stdout carries only the JSON line: anything the runtime or gloo prints
    # there (gloo's "Rank r is connected to n peer ranks" banner at N > 1) goes
    # to stderr, and the line is written to the saved descriptor
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    if args.config == "HB":
        return main_hostloop(args, world, rank, local_rank, json_out)

    import torch
    import torch.distributed as dist

    abi.load_hip()  # after torch: one HIP runtime per process (see abi.load_hip)

    if world > 1:
        dist.init_process_group("gloo")  # barrier + max-time only; the data path has no collective

    from trajopt_amd.runtime import BatchTrustRegionSQP

    wl = sharding.rank_workload(args.config, args.batch, rank)
    # one GPU per rank; ranks beyond the visible GPUs share them (a rehearsal of the N > 1
    # path on a smaller box -- the weak-scaling numbers are only meaningful with one GPU each)
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    # one torch stream per batch context, so that torch events bracket each launch on its own stream
    streams = [torch.cuda.Stream() for _ in range(max(1, args.inflight))]
    solvers = [BatchTrustRegionSQP(wl, device=device, stream=st.cuda_stream) for st in streams]
    for s in solvers:
        s.upload()
    solver = solvers[0]
    # the fused kernel that runs this workload's QPs: the main build, or the
    # generic-step build for QPs outside the register-resident segment's domain
    fused_kernel = "thip::sqp_kernel_gen" if solver.layout()["gen"] else "thip::sqp_kernel"

    for _ in range(args.warmup):
        for s in solvers:
            s.run()
    res = solver.download()[1] if args.warmup > 0 else None
    # one batch alone (no other batch in flight): the per-batch latency.  Every
    # context's warmup launches must have drained first, else this launch shares
    # the CUs with their tails
    for s in solvers:
        s.sync()
    torch.cuda.synchronize()
    solver.run()
    solver.sync()
    batch_latency_ms = solver.kernel_ms()

    def barrier():
        if world > 1:
            dist.barrier()

    if args.diag_util:
        for s in solvers:
            s.enable_profile(True)  # zeroed counters, accumulated over the timed launches
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    events = []
    for k in range(args.steps):
        st = streams[k % len(streams)]
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record(st)
        solvers[k % len(solvers)].run()  # asynchronous: each context's stream queues its steps
        ev[1].record(st)
        events.append(ev)
    for s in solvers:
        s.sync()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    # every timed launch, bracketed on its own stream (stage + sqp_kernel + gather; the
    # sqp_kernel share of a launch is > 97 % in profiles/*_kernel_stats.csv)
    kernel_ms = [a.elapsed_time(b) for a, b in events]
    if args.diag_util:
        pf = np.concatenate([s.get_profile() for s in solvers]).astype(np.float64)
        n_cu = torch.cuda.get_device_properties(device).multi_processor_count
        busy = pf[:, 14].sum() * 1e-8  # problem wall time, 10 ns units (s_memrealtime)
        print(f"diag-util: {n_cu} CUs busy {100 * busy / (n_cu * elapsed):.1f} % of {elapsed:.2f} s; "
              f"shader clock {pf[:, 13].sum() / pf[:, 14].sum() * 100:.0f} MHz; mean problem "
              f"{busy / (len(solvers) and args.steps * wl.batch) * 1e3:.1f} ms", file=sys.stderr)
    x_last, res_last = solver.download()
    for s in solvers[1:min(len(solvers), args.steps)]:  # the contexts that ran a timed step
        _, r2 = s.download()
        if any(a.n_sqp_iters != b.n_sqp_iters or a.n_admm_iters != b.n_admm_iters for a, b in zip(r2, res_last)):
            raise SystemExit("batch contexts disagree on the same problems")

    # every step solves the same problems: the counters must repeat exactly
    same = res is None or all(a.n_sqp_iters == b.n_sqp_iters and a.n_admm_iters == b.n_admm_iters
                              for a, b in zip(res, res_last))
    if not same:
        raise SystemExit("non-deterministic SQP counters between steps")
    iters_local = sum(r.n_sqp_iters for r in res_last)
    bytes_local, model = algorithmic_bytes(wl, res_last)
    kms = float(np.mean(kernel_ms))

    elapsed, iters_total = sharding.reduce_step_stats(elapsed, iters_local, world)

    if rank == 0:
        value = iters_total * args.steps / elapsed
        achieved = bytes_local / (kms * 1e-3) / 1e9
        # the same bytes over the whole timed region (all batches in flight
        # together), and the PMC-measured HBM traffic over the launch duration
        aggregate = bytes_local * args.steps / elapsed / 1e9  # rank 0's GPU
        wname = workload_name(wl, args.config, args.batch)
        traffic, traffic_src = measured_traffic(wname, args.batch)
        out = {
            "metric": "SQP iters/sec + achieved HBM GB/s, 7-DoF x 30-wpt x 1024-batch",
            "value": value,
            "unit": "SQP iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (splitmix64 seeds 20261015+b, PR2 %s; SURVEY.md §8d)"
                    % ("both arms" if wl.n_dof == 14 else "right arm"),
            "config": {
                "workload": wname,
                "batch_per_gpu": args.batch,
                "global_batch": args.batch * world,
                "sqp_iters_per_step": iters_total,
                "qp_solves_per_step_rank0": sum(r.n_qp_solves for r in res_last),
                "admm_iters_per_step_rank0": sum(r.n_admm_iters for r in res_last),
                "parallelism": f"shard{world} (independent problems, no collective)",
                "batches_in_flight": len(solvers),
                "batch_latency_ms": batch_latency_ms,
            },
            "roofline": {
                # what limits the kernel: the serial block-tridiagonal KKT chains and
                # barriers of every ADMM iteration (one 256-thread problem per CU; wave
                # cycles mostly parked on s_waitcnt / barriers, see `pmc`).  `achieved` /
                # `frac` are the SURVEY.md 8d streaming-byte model against HBM peak, as
                # the metric asks; the working set is LDS/register resident, so the
                # measured HBM traffic (`traffic`, `measured_gbs`) is far below it.
                "bound": "hbm",
                "limiter": "latency",
                "kernel": fused_kernel,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "measured_gbs": (traffic / (kms * 1e-3) / 1e9) if traffic else None,
                "achieved_per_step_gbs": aggregate,
                "latency": latency_model(args.config),
                "pmc": pmc_evidence(args.config),
                "kernel_ms": kms,
                "algorithmic_bytes_per_launch": bytes_local,
                "model": model,
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_problems, args.cpu_threads)
        print(json.dumps(out), file=json_out, flush=True)

    for s in solvers:
        s.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
