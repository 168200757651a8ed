"""Dispatch simulation of bench.py's pipeline, diagnostic.

Replays per-problem durations (tools/phase_profile.py writes them to
gpurun_out/pp_<cfg>_<B>_wall.npy, 10 ns units) through a model of the GPU:
`cus` compute units holding one workgroup (one problem) each; `inflight` batch
contexts, each a stream whose launches run one after the other; the workgroups
of every running launch are dispatched in index order, oldest launch first,
whenever a CU is free.  Prints the time per step for K steps submitted
round-robin, against the bound total work / cus.

    python tools/dispatch_sim.py gpurun_out/pp_C_1024_wall.npy [steps] [cus]
"""
import heapq
import sys

import numpy as np


def simulate(dur, steps, inflight, cus=256, order=None):
    """Wall time of `steps` launches of the batch `dur` on `inflight` streams."""
    B = len(dur)
    order = np.arange(B) if order is None else order
    free = [0.0] * cus  # heap of CU free times
    heapq.heapify(free)
    stream_ready = [0.0] * inflight  # when each stream's previous launch ended
    launches = []  # (start time, next wg, step, end time so far)
    pending = list(range(steps))
    t_end = 0.0
    # event-driven: launches become dispatchable when their stream is ready; workgroups
    # go to the earliest free CU among the oldest dispatchable launch's next workgroup
    running = []  # [ready_time, step, next_idx, finish_max]
    for k in range(min(inflight, steps)):
        running.append([0.0, k, 0, 0.0])
    next_step = len(running)
    while running:
        # the launch whose next workgroup can start earliest (oldest first on ties)
        t_cu = free[0]
        cand = min(running, key=lambda r: (max(r[0], t_cu), r[1]))
        start = max(cand[0], heapq.heappop(free))
        wg = order[cand[2]]
        fin = start + dur[wg]
        heapq.heappush(free, fin)
        cand[2] += 1
        cand[3] = max(cand[3], fin)
        if cand[2] == B:
            running.remove(cand)
            t_end = max(t_end, cand[3])
            if next_step < steps:
                running.append([cand[3], next_step, 0, 0.0])  # same stream: after this launch's last problem
                next_step += 1
    return t_end


def simulate_xcd(dur, steps, inflight, cus=256, xcds=8):
    """The same with the grid dealt round-robin over `xcds` dies (workgroup i runs
    on die i % xcds, cus / xcds CUs each): the slowest die ends the run."""
    return max(simulate(dur[x::xcds], steps, inflight, cus // xcds) for x in range(xcds))


def main():
    dur = np.load(sys.argv[1]).astype(np.float64) * 1e-8  # seconds
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    cus = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    bound = dur.sum() / cus
    print(f"{len(dur)} problems: mean {dur.mean() * 1e3:.1f} ms, max {dur.max() * 1e3:.1f} ms; "
          f"work / {cus} CUs = {bound * 1e3:.0f} ms per batch")
    for inflight in (1, 2, 3, 4, 6, 8, steps):
        t = simulate(dur, steps, inflight, cus)
        tx = simulate_xcd(dur, steps, inflight, cus)
        print(f"  {inflight:2d} in flight: {t / steps * 1e3:7.0f} ms/step ({bound * steps / t * 100:5.1f} % of the bound); "
              f"grid dealt over 8 XCDs: {tx / steps * 1e3:7.0f} ms/step ({bound * steps / tx * 100:5.1f} %)")


if __name__ == "__main__":
    main()
