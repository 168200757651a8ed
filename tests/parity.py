"""The parity gate (BASELINE.json north_star): the HIP path against the oracle.

Bar, per problem: identical OptStatus, identical constraint-satisfied flag
(max violation < cnt_tolerance) and the converged trajectory within 1e-5
absolute of the oracle's.

A problem that misses the bar passes only with a proof, on THAT problem, that
the reference algorithm itself does not determine its outcome at double
precision.  The proof reruns the oracle on the problem under rounding-level
changes that leave the mathematics untouched:
  * the oracle's second build (oracle/Makefile `liboracle_fast_*`: the same
    sources at -O3 with FMA contraction): the same algorithm, another rounding;
  * rounding jitter (oracle/src/jitter.hpp), re-drawing the noise that the
    GPU's different operation order puts into the quantities the algorithm
    thresholds: +-3e-10 on every forward-difference CartPose Jacobian entry,
    a relative 5e-15 on every KKT solve, 1e-9 on every returned QP solution
    and +-1e-12 on every linearised contact expression (collision gradient
    coefficients and constant: FK and Jacobian products in the GPU's
    contraction order); each amplitude is checked against the measured
    GPU-vs-oracle gap of its quantity (test_gpu.py
    test_jitter_amplitudes_match_measured_gaps);
  * the initial trajectory perturbed by 1e-13, then 1e-12 (interior
    waypoints, seeded normal noise).
The rerun "cloud" is grown lazily, only for the problems that miss the bar,
and the problem is excused iff
  (reach)   some rerun reaches the GPU's outcome: same status, same flag and
            a trajectory within 1e-5 of the GPU's; or
  (spread)  the GPU has the oracle's status and flag, the reruns' trajectories
            spread beyond 1e-5 from the oracle's own, and the GPU's trajectory
            lies inside that cloud: its distance to the oracle is at most the
            cloud's own largest distance to the oracle, it lies outside the
            cloud's envelope (the coordinate-wise range of the oracle and its
            reruns) by no more than 1e-5 -- or, once the cloud holds at least
            49 reruns, by no more than the cloud's own scatter: the largest
            amount by which one cloud point lies outside the envelope of the
            others (a draw from the same rounding distribution sticks out
            further than all n + 1 cloud points with probability 1 / (n + 2),
            at most 1/51) -- and its total cost lies within the reruns' cost
            range (+-2 %).
A status or flag mismatch needs (reach).  "Some QP was unpolished" is no
longer an excuse by itself.

Every check is recorded (label, batch, strict, reached, spread, and each
excused problem with its distance to the oracle and to the nearest rerun) and
tests/conftest.py writes the table to gpurun_out/parity_table.json at the end
of the session.

Floors on the strict fraction (problems that meet the bar with no excuse):
  * a check of 32 or more problems: min_strict (default 85 %);
  * a check of 8 to 31 problems: MIN_STRICT_SMALL (60 %);
  * pooled over every check of 8 or more problems: POOLED_MIN (93 %), enforced
    by tests/conftest.py at the end of the session (the run fails below it).

The gate is frozen (round 5): its rules, jitter amplitudes, schedule and floors
are those of the end of round 4 plus the floors above, and a red run is not
answered by widening them -- the failing problem's trace is compared with the
oracle's (tools/trace_compare.py, tools/hostloop_trace.py) and the cause fixed
or recorded.
"""
from __future__ import annotations

import numpy as np

TOL_X = 1e-5
COST_RTOL = 0.02
# reruns before the envelope test is calibrated by the cloud's own scatter (below
# that, the GPU must lie within 1e-5 of the envelope)
LOO_MIN_CLOUD = 49
# strict-fraction floors (module docstring)
MIN_STRICT_SMALL = 0.60
POOLED_MIN = 0.93
POOLED_MIN_BATCH = 8

# (build, input perturbation amplitude, rounding jitter on, seed)
# FD Jacobian (absolute), KKT solve, QP solution (relative), contact expressions (absolute)
JITTER = (3e-10, 5e-15, 1e-9, 1e-12)
SCHEDULE = ([("fast", 0.0, False, 0)]
            + [("exact", 0.0, True, s) for s in range(1, 9)]
            + [("exact", 1e-13, False, s) for s in range(1, 5)]
            + [("fast", 0.0, True, s) for s in range(1, 5)]
            + [("exact", 1e-12, False, s) for s in range(1, 5)]
            + [("exact", 1e-13, True, s) for s in range(9, 13)]
            + [("exact", 0.0, True, s) for s in range(13, 21)]
            + [("fast", 1e-13, True, s) for s in range(21, 25)]
            + [("exact", 1e-12, True, s) for s in range(25, 33)]
            + [("fast", 1e-12, True, s) for s in range(33, 37)]
            # runs 50-97: only problems the first 49 leave unexplained get here (the
            # cloud grows lazily); a GPU outcome drawn from the same rounding
            # distribution falls outside the envelope of n reruns in a given
            # coordinate with probability 2/(n+2), so a chaotic problem can need more
            # than 49 (4 of C-1024's 14 misses did in round 4)
            + [("exact", 0.0, True, s) for s in range(37, 61)]
            + [("fast", 0.0, True, s) for s in range(61, 73)]
            + [("exact", 1e-13, True, s) for s in range(73, 85)])

RECORDS: list[dict] = []


def progress(msg):
    """Progress line for long checks (pytest -s on the GPU box: a silent
    minute reads as a hang there)."""
    import sys
    import time

    print(f"[parity {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def oracle_solve(wl, oracle_mod, threads=16, chunk=256, variant="exact"):
    """oracle.solve over wl in chunks, with a progress line per chunk."""
    if wl.batch <= chunk:
        return oracle_mod.solve(wl, n_threads=threads, variant=variant)
    xs, rs = [], []
    for lo in range(0, wl.batch, chunk):
        hi = min(wl.batch, lo + chunk)
        x, r = oracle_mod.solve(subset(wl, np.arange(lo, hi)), n_threads=threads, variant=variant)
        xs.append(x)
        rs.extend(r)
        progress(f"oracle {variant}: problems {lo}-{hi - 1} of {wl.batch}")
    return np.concatenate(xs), rs


def subset(wl, idx):
    """The workload restricted to problems idx (same descriptor)."""
    from trajopt_amd.problems import Workload

    idx = np.asarray(idx, dtype=int)
    return Workload(wl.name, wl.desc, wl.init[idx].copy(), wl.targets[idx].copy(), wl.scene[idx].copy(),
                    wl.q_ref[idx].copy(), None if wl.jpos_targets is None else wl.jpos_targets[idx].copy())


def perturbed(wl, amp, seed):
    if amp == 0.0:
        return wl
    wp = subset(wl, np.arange(wl.batch))
    rng = np.random.default_rng(seed)
    wp.init[:, 1:] += rng.normal(0.0, amp, wp.init[:, 1:].shape)
    return wp


class Cloud:
    """Oracle reruns (SCHEDULE) of the problems that missed the bar."""

    def __init__(self, wl, idx, oracle_mod, threads=16, solver=None):
        self.wl, self.idx, self.oracle_mod, self.threads = wl, list(idx), oracle_mod, threads
        self.solver = solver
        self.members = {b: [] for b in self.idx}  # b -> [(x, status, flag, cost)]
        self.k = 0

    def grow(self, pending):
        """Run the next schedule entry on the pending problems; False when exhausted."""
        if self.k >= len(SCHEDULE) or not pending:
            return False
        build, amp, jit, seed = SCHEDULE[self.k]
        self.k += 1
        sub = perturbed(subset(self.wl, pending), amp, seed)
        if jit:
            self.oracle_mod.set_jitter(*JITTER[:3], seed=seed, variant=build)
            self.oracle_mod.set_jitter_coll(JITTER[3], variant=build)
        try:
            if self.solver is not None:
                x, res = self.solver(sub, build)
            else:
                x, res = oracle_solve(sub, self.oracle_mod, self.threads, variant=build)
        finally:
            if jit:
                self.oracle_mod.set_jitter(0.0, 0.0, 0.0, seed=0, variant=build)
                self.oracle_mod.set_jitter_coll(0.0, variant=build)
        progress(f"cloud run {self.k}/{len(SCHEDULE)} ({build}, input {amp:g}, jitter {jit}, seed {seed}) "
                 f"on {len(pending)} problems")
        tol = self.wl.desc.sqp.cnt_tolerance
        for j, b in enumerate(pending):
            self.members[b].append((x[j], res[j].status, res[j].max_cnt_viol < tol, res[j].total_cost))
        return True


def check_parity(wl, oracle_mod, x, res, label="", min_strict=0.85, oracle=None, threads=16, solver=None):
    """Assert the bar for every problem of wl (see the module docstring).
    oracle: precomputed (x_oracle, results) of the same workload, else solved here.
    solver: solver(workload, build) -> (x, results), the oracle entry point for
    problems oracle.solve does not cover (a caller's cost next to the lowered
    terms); it serves the reference solve and every cloud rerun (the jitter is
    set on the oracle library around it as for oracle.solve).
    Returns the record added to RECORDS."""
    if oracle is not None:
        xo, ro = oracle
    elif solver is not None:
        xo, ro = solver(wl, "exact")
    else:
        xo, ro = oracle_solve(wl, oracle_mod, threads)
    tol = wl.desc.sqp.cnt_tolerance
    B = wl.batch
    dx = np.abs(np.asarray(x) - xo).reshape(B, -1).max(1)
    miss = []
    for b in range(B):
        fg, fo = res[b].max_cnt_viol < tol, ro[b].max_cnt_viol < tol
        if res[b].status != ro[b].status or fg != fo or dx[b] > TOL_X:
            miss.append(b)
    reached, spread, unexplained = [], [], []
    if miss:
        cloud = Cloud(wl, miss, oracle_mod, threads, solver)
        pending = list(miss)
        while pending:
            still = []
            for b in pending:
                fg, fo = res[b].max_cnt_viol < tol, ro[b].max_cnt_viol < tol
                same_outcome = res[b].status == ro[b].status and fg == fo
                mem = cloud.members[b]
                if any(st == res[b].status and fl == fg and np.abs(xm - x[b]).max() <= TOL_X
                       for xm, st, fl, _ in mem):
                    reached.append(b)
                    continue
                if same_outcome and mem:
                    sp = max(np.abs(xm - xo[b]).max() for xm, _, _, _ in mem)
                    costs = [ro[b].total_cost] + [c for _, _, _, c in mem]
                    lo, hi = min(costs), max(costs)
                    cg = res[b].total_cost
                    exc, loo = _excess(x[b], xo[b], mem), _loo_excess(xo[b], mem)
                    inside = exc <= TOL_X or (len(mem) >= LOO_MIN_CLOUD and exc <= loo)
                    if (sp > TOL_X and dx[b] <= sp and inside
                            and lo - COST_RTOL * max(1.0, abs(lo)) <= cg <= hi + COST_RTOL * max(1.0, abs(hi))):
                        spread.append(b)
                        continue
                still.append(b)
            pending = still
            if pending and not cloud.grow(pending):
                unexplained = pending
                break
    strict = B - len(miss)
    excused = []
    for kind, lst in (("reach", reached), ("spread", spread)):
        for b in lst:
            near = min(np.abs(xm - x[b]).max() for xm, _, _, _ in cloud.members[b])
            e = {"problem": int(b), "kind": kind, "dx_oracle": float(dx[b]), "dx_nearest_rerun": float(near),
                 "status": int(res[b].status), "oracle_status": int(ro[b].status), "cloud": len(cloud.members[b])}
            if kind == "spread":
                e["envelope_excess"] = _excess(x[b], xo[b], cloud.members[b])
                e["cloud_loo_excess"] = _loo_excess(xo[b], cloud.members[b])
            excused.append(e)
    rec = {"label": label, "batch": B, "strict": strict, "reached": len(reached), "spread": len(spread),
           "excused": excused,
           "status_mismatch": int(sum(res[b].status != ro[b].status for b in range(B))),
           "median_dx": float(np.median(dx)) if B else 0.0,
           "max_dx_strict": float(max([dx[b] for b in range(B) if b not in miss], default=0.0)),
           "cloud_runs": 0 if not miss else cloud.k, "unexplained": [int(b) for b in unexplained],
           "min_strict": min_strict}
    RECORDS.append(rec)
    msgs = []
    for b in unexplained:
        fg, fo = res[b].max_cnt_viol < tol, ro[b].max_cnt_viol < tol
        mem = cloud.members[b]
        msgs.append(f"problem {b}: status {res[b].status} vs {ro[b].status}, flag {fg} vs {fo}, "
                    f"|dx| {dx[b]:.2e}, cost {res[b].total_cost:.6g} vs {ro[b].total_cost:.6g}; "
                    f"{len(mem)} oracle reruns reach {sorted({(st, fl) for _, st, fl, _ in mem})}, "
                    f"spread {max([np.abs(xm - xo[b]).max() for xm, _, _, _ in mem], default=0):.1e}, "
                    f"envelope excess {_excess(x[b], xo[b], mem):.1e} (cloud's own {_loo_excess(xo[b], mem):.1e})")
    assert not unexplained, f"{label}: {len(unexplained)} problems miss the bar without proof:\n" + "\n".join(msgs)
    if B >= 32:
        assert strict >= min_strict * B, f"{label}: only {strict}/{B} problems meet the bar strictly"
    elif B >= POOLED_MIN_BATCH and min_strict > 0:
        assert strict >= MIN_STRICT_SMALL * B, f"{label}: only {strict}/{B} problems meet the bar strictly"
    return rec


def _excess(xg, xo, mem):
    """How far the GPU's trajectory lies outside the cloud's coordinate-wise
    envelope (0 inside)."""
    cx = np.stack([xo] + [xm for xm, _, _, _ in mem])
    return float(max(0.0, (cx.min(0) - xg).max(), (xg - cx.max(0)).max()))


def _loo_excess(xo, mem):
    """The cloud's own scatter about its envelope: the largest amount by which one
    point of the cloud (the oracle or a rerun) lies outside the envelope of all
    the others.  For a GPU outcome drawn from the same rounding distribution,
    the chance that it sticks out further than every one of the n + 1 cloud
    points does is 1 / (n + 2)."""
    cx = np.stack([xo] + [xm for xm, _, _, _ in mem])
    if len(cx) < 2:
        return 0.0
    order = np.sort(cx, axis=0)
    lo1, lo2, hi1, hi2 = order[0], order[1], order[-1], order[-2]
    worst = 0.0
    for p in cx:
        lo = np.where(p == lo1, lo2, lo1)  # the others' minimum (ties leave lo1)
        hi = np.where(p == hi1, hi2, hi1)
        worst = max(worst, float((lo - p).max()), float((p - hi).max()))
    return worst


def pooled(records=None):
    """Pooled (strict, total) over the recorded checks of POOLED_MIN_BATCH or
    more problems that carry a fraction bound."""
    rs = RECORDS if records is None else records
    rs = [r for r in rs if r["min_strict"] > 0 and r["batch"] >= POOLED_MIN_BATCH]
    return sum(r["strict"] for r in rs), sum(r["batch"] for r in rs)
