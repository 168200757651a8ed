"""Summarise the rocprofv3 CSV outputs of tools/collect_profiles.sh into profiles/.

    python tools/summarize_profiles.py r01

Writes
  profiles/<round>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<round>_pmc_hbm.json       FETCH_SIZE / WRITE_SIZE of sqp_kernel per launch (separate passes)
  profiles/<round>_bench.json         the bench line of the same round
bench.py reads the newest profiles/*_pmc_hbm.json matching its workload to fill roofline.traffic.
"""
import csv
import json
import shutil
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
OUT = REPO / "gpurun_out"
PROF = REPO / "profiles"


def counter(path, name):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if "sqp_kernel" in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {name} rows for sqp_kernel in {path}")
    return sum(vals) / len(vals), len(vals)


def main(rnd):
    PROF.mkdir(exist_ok=True)
    shutil.copy(OUT / "prof_kt" / "kt_kernel_stats.csv", PROF / f"{rnd}_kernel_stats.csv")
    bench = json.loads((OUT / "bench.json").read_text().strip().splitlines()[-1])
    (PROF / f"{rnd}_bench.json").write_text(json.dumps(bench, indent=1) + "\n")
    fetch_kb, nf = counter(OUT / "prof_fetch" / "f_counter_collection.csv", "FETCH_SIZE")
    write_kb, nw = counter(OUT / "prof_write" / "w_counter_collection.csv", "WRITE_SIZE")
    pmc = {
        "kernel": "thip::sqp_kernel",
        "workload": bench["config"]["workload"],
        "batch_per_gpu": bench["config"]["batch_per_gpu"],
        "fetch_size_kb_per_launch": fetch_kb,
        "write_size_kb_per_launch": write_kb,
        "launches": [nf, nw],
        "hbm_bytes_per_launch": (fetch_kb + write_kb) * 1024.0,
        "hbm_bytes_per_launch_fetch_x2": (2 * fetch_kb + write_kb) * 1024.0,
        "note": ("rocprofv3 FETCH_SIZE/WRITE_SIZE (KB) from separate --pmc passes (MI355X_MICROARCH.md: TCC slots); "
                 "FETCH_SIZE under-reports 16 B/lane streaming reads by 2x on gfx950, other widths uncalibrated: "
                 "hbm_bytes_per_launch is uncorrected, *_fetch_x2 applies the 2x bound"),
    }
    (PROF / f"{rnd}_pmc_hbm.json").write_text(json.dumps(pmc, indent=1) + "\n")
    print(json.dumps(pmc))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
