"""Test configuration.

Markers: `gpu` tests need an MI355X (run on the GPU box with `-m gpu`); all
other tests run on CPU.  The oracle (oracle/, CPU restatement of the
reference path) is imported here only as the checker.
"""
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
for p in (REPO, REPO / "trajopt-1_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (MI355X, gfx950)")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    d = REPO / "tests" / "golden"

    def load(name):
        return dict(np.load(d / f"{name}.npz"))

    return load


def pytest_sessionfinish(session, exitstatus):
    """Write the parity gate's per-check table (tests/parity.py RECORDS) to
    gpurun_out/parity_table.json (DESIGN.md §5 is regenerated from it)."""
    try:
        import parity
    except ImportError:
        return
    if not parity.RECORDS:
        return
    import json

    out = REPO / "gpurun_out"
    out.mkdir(exist_ok=True)
    strict, total = parity.pooled()
    (out / "parity_table.json").write_text(json.dumps(
        {"records": parity.RECORDS, "pooled_strict": strict, "pooled_total": total}, indent=1) + "\n")
    # the pooled floor over every check of 8 or more problems (tests/parity.py)
    if total and strict < parity.POOLED_MIN * total:
        print(f"\nparity gate: pooled strict {strict}/{total} = {strict / total:.3f} < {parity.POOLED_MIN}")
        session.exitstatus = 1


def pytest_runtest_logreport(report):
    """Each GPU test's wall time as it finishes (THIP_TEST_TIMES=1: the suite's
    time budget is checked from a log that a time limit may cut short)."""
    import os

    if report.when == "call" and os.environ.get("THIP_TEST_TIMES"):
        sys.__stderr__.write(f"[time] {report.nodeid} {report.duration:.1f} s {report.outcome}\n")
        sys.__stderr__.flush()
