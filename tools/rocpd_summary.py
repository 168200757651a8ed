"""Summarise a rocprofv3 rocpd database (--kernel-trace --stats) as text.

    python tools/rocpd_summary.py gpurun_out/prof1/run_results.db > profiles/<name>.txt
"""
import sqlite3
import sys


def main(path):
    db = sqlite3.connect(path)
    print(f"# rocprofv3 kernel-trace summary of {path}")
    print("# durations in microseconds (rocpd top_kernels view: ns / 1e3)")
    print(f"{'kernel':<80} {'calls':>6} {'total_us':>14} {'avg_us':>14} {'pct':>7}")
    for name, calls, total, avg, pct in db.execute(
        "select name, total_calls, total_duration, average, percentage from top_kernels"
    ):
        print(f"{name[:80]:<80} {calls:>6} {total / 1e3:>14.1f} {avg / 1e3:>14.1f} {pct:>7.3f}")
    print()
    print("# per-dispatch resources")
    seen = set()
    for row in db.execute(
        "select name, grid_x, workgroup_x, lds_size, static_lds_size, scratch_size, vgpr_count, "
        "accum_vgpr_count, sgpr_count, duration from kernels order by start"
    ):
        if row[0] in seen:
            continue
        seen.add(row[0])
        name, gx, wx, lds, slds, scr, vgpr, agpr, sgpr, dur = row
        print(f"{name[:60]:<60} grid {gx} wg {wx} lds {lds} (static {slds}) scratch {scr} "
              f"vgpr {vgpr} agpr {agpr} sgpr {sgpr}")
    print()
    print("# sqp_kernel dispatch durations (us)")
    for (dur,) in db.execute("select duration from kernels where name like '%sqp_kernel%' order by start"):
        print(f"{dur / 1e3:.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
