"""CPU tests of the parity gate itself (tests/parity.py) with a stand-in oracle
whose reruns scatter around a fixed trajectory: a GPU outcome drawn from the
same scatter is excused by (spread); one biased away from it, or scattered
wider than the cloud, is not."""
from types import SimpleNamespace

import numpy as np
import pytest

import parity
from trajopt_amd import problems


class ScatterOracle:
    """oracle.solve stand-in: every call returns base + sigma * N(0, 1), so the
    reruns are exchangeable draws (the first call is 'the oracle')."""

    def __init__(self, base, sigma, seed):
        self.base, self.sigma = base, sigma
        self.rng = np.random.default_rng(seed)

    def solve(self, wl, n_threads=16, variant="exact"):
        x = self.base[None] + self.sigma * self.rng.standard_normal((wl.batch,) + self.base.shape)
        return x, [SimpleNamespace(status=0, max_cnt_viol=0.0, total_cost=1.0) for _ in range(wl.batch)]

    def set_jitter(self, *a, **k):
        pass

    def set_jitter_coll(self, *a, **k):
        pass


def _gate(gpu_shift, gpu_scale, seed):
    wl = problems.make_workload("A", 1)
    base = np.zeros(wl.init.shape[1:])
    orc = ScatterOracle(base, 1e-3, seed)
    g = np.random.default_rng(1000 + seed)
    x = base[None] + gpu_shift + gpu_scale * 1e-3 * g.standard_normal((1,) + base.shape)
    res = [SimpleNamespace(status=0, max_cnt_viol=0.0, total_cost=1.0)]
    try:
        parity.check_parity(wl, orc, x, res, label="gate-test", min_strict=0.0)
        return True
    except AssertionError:
        return False
    finally:
        parity.RECORDS.pop()


def test_same_distribution_is_excused():
    """A draw from the cloud's own distribution passes nearly always (it sticks
    out further than all n + 1 cloud points with probability 1 / (n + 2))."""
    ok = sum(_gate(0.0, 1.0, s) for s in range(20))
    assert ok >= 18, ok


@pytest.mark.parametrize("shift,scale", [(3e-3, 1.0), (0.0, 3.0)])
def test_biased_or_wider_is_refused(shift, scale):
    """A GPU outcome offset by 3 sigma in every coordinate, or scattered three
    times wider than the reruns, is refused."""
    ok = sum(_gate(shift, scale, s) for s in range(10))
    assert ok == 0, ok
