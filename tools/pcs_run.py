"""One SQP batch for PC sampling (diagnostic): python tools/pcs_run.py C 256"""
import sys

sys.path.insert(0, "trajopt-1_amd")
from trajopt_amd import problems
from trajopt_amd.runtime import BatchTrustRegionSQP

cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
s = BatchTrustRegionSQP(problems.make_workload(cfg, B))
s.upload()
s.run()
s.download()
print(f"config {cfg} batch {B}: kernel {s.kernel_ms():.1f} ms")
