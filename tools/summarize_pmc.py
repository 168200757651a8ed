"""Summarise tools/pmc_latency.sh's rocprofv3 --pmc passes into profiles/<round>_pmc_<config>.json.

    python tools/summarize_pmc.py r03 C 1024

For sqp_kernel (one lone launch per pass) it reports every counter's per-launch
total and the ratios that say what limits the kernel:
  - wave-cycle split (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY of
    SQ_WAVE_CYCLES: parked on s_waitcnt/barrier, issue-stalled, issuing);
  - VALU issue share of wave cycles, LDS bank-conflict share of LDS cycles;
  - waves per SIMD (one 256-thread workgroup per CU = 1 wave per SIMD);
  - HBM bytes (FETCH_SIZE + WRITE_SIZE) against the kernel's duration.
SQ_*_CYCLES counters count quad-cycles (MI355X_MICROARCH.md, cycle constants).
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
PROF = REPO / "profiles"


def read_pass(d):
    vals = defaultdict(list)
    for p in Path(d).rglob("*counter_collection.csv"):
        with open(p) as f:
            for row in csv.DictReader(f):
                if "sqp_kernel" in row["Kernel_Name"]:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def kernel_ns(d):
    for p in Path(d).rglob("*kernel_trace.csv"):
        with open(p) as f:
            ds = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(f)
                  if "sqp_kernel" in r["Kernel_Name"]]
        if ds:
            return sum(ds) / len(ds)
    return None


def main(rnd, cfg, batch):
    base = REPO / "gpurun_out" / f"pmc_{cfg}"
    c, n = {}, {}
    for sub in sorted(base.iterdir()):
        if sub.is_dir():
            v, k = read_pass(sub)
            c.update(v)
            n.update(k)
    wc = c.get("SQ_WAVE_CYCLES")
    out = {"kernel": "thip::sqp_kernel", "config": cfg, "batch": int(batch), "counters_per_launch": c,
           "launches_per_pass": n}
    if wc:
        out["wave_cycle_split"] = {
            "parked_waitcnt_or_barrier": c.get("SQ_WAIT_ANY", 0) / wc,
            "issue_stalled": c.get("SQ_WAIT_INST_ANY", 0) / wc,
            "issuing": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            "valu_issue": c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
            "lds_issue": c.get("SQ_ACTIVE_INST_LDS", 0) / wc,
            "vmem_issue": c.get("SQ_ACTIVE_INST_VMEM", 0) / wc,
            "salu_issue": c.get("SQ_ACTIVE_INST_SCA", 0) / wc,
            "lds_issue_stall": c.get("SQ_WAIT_INST_LDS", 0) / wc,
        }
    if c.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_share"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
    if c.get("SQ_WAVES") and c.get("SQ_BUSY_CYCLES"):
        # average resident waves = wave-cycles / busy cycles (both quad-cycle units, per SE sum)
        out["avg_waves_resident_per_busy_cycle"] = wc / c["SQ_BUSY_CYCLES"] if wc else None
    if c.get("SQ_INSTS_VALU") and c.get("SQ_INSTS_WAVE") is not None:
        out["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / max(1.0, c.get("SQ_WAVES", 1.0))
    fs, ws = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
    if fs is not None and ws is not None:
        out["hbm_bytes_per_launch"] = (fs + ws) * 1024.0
        out["hbm_bytes_per_launch_fetch_x2"] = (2 * fs + ws) * 1024.0
    ns = None
    for sub in sorted(base.iterdir()):
        if sub.is_dir():
            ns = ns or kernel_ns(sub)
    out["kernel_ns_lone_launch"] = ns
    if ns and fs is not None and ws is not None:
        out["measured_hbm_gbs"] = (fs + ws) * 1024.0 / ns
    out["note"] = ("one lone launch per pass (bench.py --steps 1 --warmup 0 --inflight 1); SQ cycle counters in "
                   "quad-cycles; FETCH_SIZE uncorrected (x2 bound for 16 B/lane streaming reads on gfx950)")
    PROF.mkdir(exist_ok=True)
    (PROF / f"{rnd}_pmc_{cfg}.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*(sys.argv[1:4] if len(sys.argv) > 3 else ["r03", "C", 1024]))
