"""Latency roofline of sqp_kernel's ADMM iteration (run on the GPU box).

    python tools/latency_model.py r03 C 1024

The kernel is latency-bound (profiles/*_pmc_C.json: most wave cycles parked on
s_waitcnt / barriers; measured HBM traffic ~1 % of peak).  Its serial floor
per ADMM iteration in the register-resident segment is
    chain depth x chain-step latency + phase edges x LDS hand-off latency
with
  chain depth   the twisted block solve's forward and backward half-chains,
                run concurrently on two waves: 2 x ceil((N - 1) / 2) dependent
                block steps (N waypoints);
  chain step    one 7x7 block step (fma + 3-level DPP/permlane reduction),
                measured by tools/micro/chain2 (V1 octet);
  phase edges   the segment's barriers per ADMM iteration (5), each an LDS
                write -> barrier -> dependent read + fp64 add, measured by
                tools/micro/barrier (lds_handoff).
Against it: the measured cycles per ADMM iteration of the whole kernel and of
the segment (thip_debug_profile, as tools/phase_profile.py).  Writes
profiles/<round>_latency_<config>.json (bench.py quotes it in roofline.latency).
"""
import json
import math
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "trajopt-1_amd"))

SEG_BARRIERS = 5


def micro(name):
    exe = REPO / "tools" / "micro" / name
    if not exe.exists():
        subprocess.run(["make", "-C", str(exe.parent), name], check=True, capture_output=True)
    return subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=60).stdout


def main(rnd, cfg, batch):
    out = micro("chain2")
    step = float(re.search(r"V1 octet ([0-9.]+)", out).group(1))
    add = float(re.search(r"add ([0-9.]+)", out.split("dependent fp64:")[1]).group(1))
    out = micro("barrier")
    bar = float(re.search(r"barrier ([0-9.]+)", out).group(1))
    hand = float(re.search(r"lds_handoff ([0-9.]+)", out).group(1))

    import numpy as np

    from trajopt_amd import problems
    from trajopt_amd.runtime import BatchTrustRegionSQP

    wl = problems.make_workload(cfg, batch)
    s = BatchTrustRegionSQP(wl)
    s.upload()
    s.run()
    s.download()
    s.enable_profile(True)
    s.run()
    _, res = s.download()
    pf = s.get_profile().astype(np.float64)
    s.close()
    admm = float(sum(r.n_admm_iters for r in res))
    names = BatchTrustRegionSQP.PROFILE_SLOTS
    per = {names[k]: pf[:, k].sum() / admm for k in range(len(names))
           if not names[k].startswith(("unused", "n_")) and k != 14}
    N = wl.n_steps
    depth = 2 * math.ceil((N - 1) / 2)
    floor = depth * step + SEG_BARRIERS * hand
    measured = per["sqp_total"]
    chains = per["fwd_chain"] + per["bwd_chain"]
    d = {
        "kernel": "thip::sqp_kernel", "config": cfg, "batch": batch, "n_steps": N,
        "chain_depth_steps": depth, "chain_step_cycles": step, "fp64_add_latency_cycles": add,
        "barrier_cycles": bar, "lds_handoff_cycles": hand, "segment_barriers_per_admm_iter": SEG_BARRIERS,
        "critical_path_cycles_per_admm_iter": floor,
        "measured_cycles_per_admm_iter": measured,
        "frac": floor / measured,
        "measured_chain_cycles_per_admm_iter": chains,
        "chain_floor_cycles_per_admm_iter": depth * step,
        "chain_frac": depth * step / chains if chains else None,
        "phases_cycles_per_admm_iter": {k: v for k, v in per.items() if v > 0},
        "note": ("serial floor = chain depth x measured chain-step latency + segment barriers x measured LDS "
                 "hand-off; measured = thip_debug_profile cycles of sqp_kernel per ADMM iteration (all phases, "
                 "amortised), one lone batch"),
    }
    (REPO / "profiles" / f"{rnd}_latency_{cfg}.json").write_text(json.dumps(d, indent=1) + "\n")
    (REPO / "gpurun_out" / f"{rnd}_latency_{cfg}.json").write_text(json.dumps(d, indent=1) + "\n")
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:] + ["r03", "C", "1024"][len(sys.argv) - 1:]
    main(a[0], a[1], int(a[2]))
