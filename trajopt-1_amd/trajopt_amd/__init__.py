"""trajopt_amd — MI355X-native batched SQP trajectory optimizer.

Host-side Python access to the C-ABI HIP library (include/trajopt_hip.h):
`abi` (struct mirror + loader), `problems` (synthetic workloads),
`runtime` (BatchTrustRegionSQP over the C-ABI).
"""
from . import abi, problems, robots  # noqa: F401

__all__ = ["abi", "problems", "robots"]
