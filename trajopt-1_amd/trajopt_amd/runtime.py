"""BatchTrustRegionSQP over the C-ABI (the batched tier of SURVEY.md §8b).

Lowers a Workload (one shared thip_problem_desc + per-problem arrays) onto one
HIP device and runs sco::BasicTrustRegionSQP::optimize for every problem in
one fused launch.  No CPU fallback: every method raises if the HIP library or
the device call fails.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class HipError(RuntimeError):
    pass


class BatchTrustRegionSQP:
    def __init__(self, workload, device: int = 0, stream=None):
        self.lib = abi.load_hip()
        self.wl = workload
        self.batch = workload.batch
        self.ctx = C.c_void_p()
        rc = self.lib.thip_create(device, C.byref(workload.desc), self.batch, C.byref(self.ctx))
        if rc != 0:
            raise HipError(f"thip_create: {self.lib.thip_last_error(None).decode()}")
        if stream is not None:
            self._check(self.lib.thip_set_stream(self.ctx, C.c_void_p(stream)), "thip_set_stream")
        self.uploaded = False

    def _check(self, rc, what):
        if rc != 0:
            raise HipError(f"{what}: {self.lib.thip_last_error(self.ctx).decode()}")

    def upload(self):
        wl = self.wl
        self._init = np.ascontiguousarray(wl.init, dtype=np.float64)
        self._tgt = np.ascontiguousarray(wl.targets, dtype=np.float64) if wl.targets.size else None
        self._scene = np.ascontiguousarray(wl.scene, dtype=np.float64) if wl.scene.size else None
        self._check(
            self.lib.thip_upload(self.ctx, _dp(self._init), _dp(self._tgt) if self._tgt is not None else None,
                                 _dp(self._scene) if self._scene is not None else None),
            "thip_upload",
        )
        jt = getattr(wl, "jpos_targets", None)
        if jt is not None:
            self._jpt = np.ascontiguousarray(jt, dtype=np.float64)
            self._check(self.lib.thip_upload_joint_targets(self.ctx, _dp(self._jpt)), "thip_upload_joint_targets")
        self.uploaded = True

    def run(self):
        if not self.uploaded:
            self.upload()
        self._check(self.lib.thip_sqp_run(self.ctx), "thip_sqp_run")

    def sync(self):
        self._check(self.lib.thip_synchronize(self.ctx), "thip_synchronize")

    def kernel_ms(self) -> float:
        return float(self.lib.thip_last_kernel_ms(self.ctx))

    def download(self):
        x = np.zeros((self.batch, self.wl.n_steps, self.wl.n_dof))
        res = (abi.Result * self.batch)()
        self._check(self.lib.thip_download(self.ctx, _dp(x), res), "thip_download")
        return x, list(res)

    def optimize(self):
        self.run()
        return self.download()

    def linearize(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        D = self.wl.n_dof
        n_cart = self.wl.desc.n_cart
        err = np.zeros((self.batch, n_cart, 6))
        jac = np.zeros((self.batch, n_cart, 6, D))
        if not self.uploaded:
            self.upload()
        self._check(self.lib.thip_linearize(self.ctx, _dp(x), _dp(err), _dp(jac)), "thip_linearize")
        return err, jac

    def fwd_kin(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        n_links = self.wl.desc.chain.n_links
        poses = np.zeros((self.batch, self.wl.n_steps, n_links, 12))
        self._check(self.lib.thip_fwd_kin(self.ctx, _dp(x), _dp(poses)), "thip_fwd_kin")
        return poses

    def collision_rows(self, x, cap=4096):
        """Linearised collision rows at trajectories x [B, N, D] (list of
        [n, 8 + 2 D + 1] arrays, one per problem; see thip_collision_rows)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        if not self.uploaded:
            self.upload()
        W = 8 + 2 * self.wl.n_dof + 1
        rec = np.zeros((self.batch, cap, W))
        cnt = (C.c_int * self.batch)()
        self._check(self.lib.thip_collision_rows(self.ctx, _dp(x), _dp(rec), cap, cnt), "thip_collision_rows")
        out = []
        for b in range(self.batch):
            if cnt[b] < 0:
                raise HipError(f"problem {b}: contact overflow")
            out.append(rec[b, : min(cnt[b], cap)])
        return out

    def enable_trace(self, capacity=512):
        self._trace_cap = capacity
        self._check(self.lib.thip_debug_trace(self.ctx, capacity), "thip_debug_trace")

    def get_trace(self):
        rec = np.zeros((self.batch, self._trace_cap, abi.TRACE_W))
        cnt = (C.c_int * self.batch)()
        self._check(self.lib.thip_debug_get_trace(self.ctx, _dp(rec), cnt), "thip_debug_get_trace")
        return [rec[b, : cnt[b]] for b in range(self.batch)]

    PROFILE_SLOTS = ["admm_step", "residuals", "termination", "factor", "polish", "linearize", "evaluate",
                     "build_and_scale", "solve_rhs_diag", "fwd_chain", "bwd_chain", "aux_backsub", "qp_solve",
                     "sqp_total", "sqp_wall_ticks", "seg_B_rhs_linv", "fwd_wave0_own",
                     "seg_hinge_gather", "seg_hinge_E", "coll_count_pass", "coll_rank_pass", "coll_rows", "coll_fk_substates",
                     "gen_rhs_mr", "gen_rhs_cols", "gen_rhs_linv", "gen_dvalue_middle",
                     "n_primal_inf_full", "n_dual_inf_full", "n_factor", "gen_pre", "gen_updates",
                     "factor_blocks", "factor_twisted", "bwd_wave0_own", "gen_dvalue", "gen_middle_wait", "unused37", "unused38",
                     "unused39"]

    def layout(self):
        """The solve layout this context chose (thip_debug_solve_layout): branches, dofs
        per block, wide, segment possible, generic-step build, threads, waypoints per solve
        block (2 with JointAccEqCost terms), solve blocks per branch."""
        out = (C.c_int * 8)()
        self._check(self.lib.thip_debug_solve_layout(self.ctx, out, 8), "thip_debug_solve_layout")
        return dict(zip(("nbr", "block_dofs", "wide", "seg_ok", "gen", "threads", "grp", "blocks"), list(out)))

    def enable_profile(self, on=True):
        self._check(self.lib.thip_debug_profile(self.ctx, 1 if on else 0), "thip_debug_profile")

    def get_profile(self):
        out = np.zeros((self.batch, 40), dtype=np.int64)
        self._check(self.lib.thip_debug_get_profile(self.ctx, out.ctypes.data_as(C.POINTER(C.c_longlong))),
                    "thip_debug_get_profile")
        return out

    def close(self):
        if self.ctx:
            self.lib.thip_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TermEvaluator:
    """thip_eval_*: the CartPose and collision terms of a workload's problems
    evaluated on the device (what the host SQP loop calls for problems the
    fused kernel does not lower)."""

    def __init__(self, workload, device: int = 0):
        self.lib = abi.load_hip()
        self.wl = workload
        self.ev = C.c_void_p()
        rc = self.lib.thip_eval_create(device, C.byref(workload.desc), workload.batch, C.byref(self.ev))
        if rc != 0:
            raise HipError(f"thip_eval_create: {self.lib.thip_eval_last_error(None).decode()}")
        self._tgt = np.ascontiguousarray(workload.targets, dtype=np.float64) if workload.targets.size else None
        self._scene = np.ascontiguousarray(workload.scene, dtype=np.float64) if workload.scene.size else None
        self._check(self.lib.thip_eval_upload(self.ev, None if self._tgt is None else _dp(self._tgt),
                                              None if self._scene is None else _dp(self._scene)), "thip_eval_upload")

    def _check(self, rc, what):
        if rc != 0:
            raise HipError(f"{what}: {self.lib.thip_eval_last_error(self.ev).decode()}")

    def cart_pose(self, term, q, jac=True):
        """q [B, D] -> err [B, 6], jac [B, 6, D] (or None)."""
        B, D = self.wl.batch, self.wl.n_dof
        q = np.ascontiguousarray(q, dtype=np.float64).reshape(B, D)
        err = np.zeros((B, 6))
        J = np.zeros((B, 6, D)) if jac else None
        self._check(self.lib.thip_eval_cart_pose(self.ev, term, _dp(q), _dp(err), None if J is None else _dp(J)),
                    "thip_eval_cart_pose")
        return err, J

    def collision(self, term, x, cap=4096):
        """x [B, N, D] -> list of record arrays [n_b, 8 + 2 D + 1]."""
        B, D = self.wl.batch, self.wl.n_dof
        W = 8 + 2 * D + 1
        x = np.ascontiguousarray(x, dtype=np.float64)
        cnt = (C.c_int * B)()
        out = np.zeros((B, cap, W))
        self._check(self.lib.thip_eval_collision(self.ev, term, _dp(x), _dp(out), cap, cnt), "thip_eval_collision")
        if max(cnt) > cap:
            return self.collision(term, x, cap=max(cnt))
        return [out[b, : cnt[b]].copy() for b in range(B)]

    def close(self):
        if self.ev:
            self.lib.thip_eval_destroy(self.ev)
            self.ev = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
