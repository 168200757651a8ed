"""ctypes binding of the C++ host front door (include/trajopt_host.h).

The front door parses problems in the reference's JSON format
(ProblemConstructionInfo::fromJson, trajopt/src/problem_description.cpp:276-312)
on the built-in environment of the reference's test robots (the PR2 groups, or
spherebot's "manipulator") and lowers them with the
TermInfo::hatch restatements; `solve_json_batch` runs them through the C++
BatchTrustRegionSQP on the HIP path.  `workload_to_json` writes a synthetic
workload problem in that format (used by the tests to drive the front door).
"""
from __future__ import annotations

import ctypes as C
import json
import math

import numpy as np

from . import abi

HOST_LIB = abi.LIB_DIR / "libtrajopt_host.so"
_host = None


class HostError(RuntimeError):
    pass


def load_host():
    global _host
    if _host is None:
        abi.load_hip()  # one HIP runtime: torch first, then libtrajopt_hip.so
        if not HOST_LIB.exists():
            raise RuntimeError(f"{HOST_LIB} is missing: run __graft_entry__.build()")
        L = C.CDLL(str(HOST_LIB))
        dp = C.POINTER(C.c_double)
        L.thost_lower_json.argtypes = [C.c_char_p, dp, C.c_int, C.POINTER(abi.ProblemDesc), dp, dp, dp, dp,
                                       C.c_char_p, C.c_int]
        L.thost_lower_json.restype = C.c_int
        L.thost_solve_json_batch.argtypes = [C.POINTER(C.c_char_p), C.c_int, dp, C.c_int, C.c_int, dp,
                                             C.POINTER(abi.Result), C.c_char_p, C.c_int]
        L.thost_solve_json_batch.restype = C.c_int
        L.thost_solve_json_batch_multi.argtypes = [C.POINTER(C.c_char_p), C.c_int, dp, C.c_int, C.POINTER(C.c_int),
                                                   C.c_int, dp, C.POINTER(abi.Result), C.c_char_p, C.c_int]
        L.thost_solve_json_batch_multi.restype = C.c_int
        L.thost_solve_json_stream.argtypes = [C.POINTER(C.c_char_p), C.c_int, C.c_int, dp, C.c_int,
                                              C.POINTER(C.c_int), C.c_int, C.c_int, dp, C.POINTER(abi.Result),
                                              C.c_char_p, C.c_int]
        L.thost_solve_json_stream.restype = C.c_int
        L.thost_last_batch_qp_stats.argtypes = [C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]
        L.thost_last_batch_qp_stats.restype = None
        L.thost_set_host_loop_workers.argtypes = [C.c_int]
        L.thost_set_host_loop_workers.restype = None
        L.thost_batch_create.argtypes = [C.POINTER(C.c_char_p), C.c_int, dp, C.c_int, C.c_int, C.POINTER(C.c_void_p),
                                         C.c_char_p, C.c_int]
        L.thost_batch_create.restype = C.c_int
        L.thost_batch_solve.argtypes = [C.c_void_p, dp, C.POINTER(abi.Result), C.c_char_p, C.c_int]
        L.thost_batch_solve.restype = C.c_int
        L.thost_batch_stats.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_longlong),
                                        C.POINTER(C.c_longlong), dp, dp]
        L.thost_batch_stats.restype = C.c_int
        L.thost_batch_qp_shape.argtypes = [C.c_void_p, C.POINTER(C.c_longlong)]
        L.thost_batch_qp_shape.restype = C.c_int
        L.thost_batch_destroy.argtypes = [C.c_void_p]
        L.thost_batch_destroy.restype = None
        L.thost_solve_json.argtypes = [C.c_char_p, dp, C.c_int, C.c_int, dp, C.POINTER(abi.Result),
                                       C.POINTER(C.c_int), C.c_char_p, C.c_int]
        L.thost_solve_json.restype = C.c_int
        _host = L
    return _host


def _dp(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def lower_json(text: str, scene=None, with_scene=False):
    """-> (desc, init [N, D], cart_targets [n_cart, 12], jpos_targets [n_jpos, D])
    (+ the scene [n_prims, 16] the collision terms see, with_scene=True: the
    built-in environment's primitives, then `scene`)."""
    L = load_host()
    sc = None if scene is None or len(scene) == 0 else np.ascontiguousarray(scene, dtype=np.float64)
    n_prims = 0 if sc is None else sc.shape[0]
    desc = abi.ProblemDesc()
    init = np.zeros((abi.EVAL_MAX_STEPS, abi.MAX_DOF))
    tgt = np.zeros((abi.MAX_CART, 12))
    jpt = np.zeros((abi.MAX_JPOS, abi.MAX_DOF))
    sco = np.zeros((abi.EVAL_MAX_PRIMS, 16))
    err = C.create_string_buffer(4096)
    rc = L.thost_lower_json(text.encode(), _dp(sc), n_prims, C.byref(desc), _dp(init), _dp(tgt), _dp(jpt), _dp(sco),
                            err, 4096)
    if rc != 0:
        raise HostError(err.value.decode())
    N, D = desc.n_steps, desc.chain.n_dof
    init = init.reshape(-1)[: N * D].reshape(N, D)
    tgt = tgt.reshape(-1)[: desc.n_cart * 12].reshape(desc.n_cart, 12)
    jpt = jpt.reshape(-1)[: desc.n_jpos * D].reshape(desc.n_jpos, D)
    if with_scene:
        has_coll = desc.coll_enabled or desc.n_coll_extra > 0
        return desc, init, tgt, jpt, sco[: desc.n_prims if has_coll else 0].copy()
    return desc, init, tgt, jpt


def solve_json_batch(texts, scenes=None, device=0, devices=None):
    """-> (x [B, N, D], list of abi.Result) through trajopt::BatchTrustRegionSQP, or
    trajopt::MultiDeviceBatchSQP over `devices` (a list of HIP device ids)."""
    L = load_host()
    B = len(texts)
    desc, _, _, _ = lower_json(texts[0], None if scenes is None else scenes[0])
    N, D = desc.n_steps, desc.chain.n_dof + (1 if desc.use_time else 0)  # (+ the dt column)
    sc = None if scenes is None else np.ascontiguousarray(scenes, dtype=np.float64)
    n_prims = 0 if sc is None else sc.shape[1]
    arr = (C.c_char_p * B)(*[t.encode() for t in texts])
    x = np.zeros((B, N, D))
    res = (abi.Result * B)()
    err = C.create_string_buffer(4096)
    devs = [device] if devices is None else list(devices)
    dv = (C.c_int * max(1, len(devs)))(*devs)
    rc = L.thost_solve_json_batch_multi(arr, B, _dp(sc), n_prims, dv, len(devs), _dp(x), res, err, 4096)
    if rc != 0:
        raise HostError(err.value.decode())
    return x, list(res)


def last_batch_qp_stats():
    """(QP launches, QPs) of this thread's last solve_json_batch: a batch of
    problems the fused kernel does not lower runs their host loops with every
    QP round batched into one launch per pattern."""
    L = load_host()
    a, b = C.c_longlong(0), C.c_longlong(0)
    L.thost_last_batch_qp_stats(C.byref(a), C.byref(b))
    return a.value, b.value


def set_host_loop_workers(n):
    """Worker threads of host-loop batches (process-wide; n <= 0: the default, 64)."""
    load_host().thost_set_host_loop_workers(int(n))


def solve_json_stream(batches, scenes=None, devices=(0,), inflight=2):
    """A stream of batches (lists of JSON texts of one structure and size)
    through trajopt::MultiDeviceBatchSQP::optimizeStream with `inflight` batches
    in flight per device entry -> (x [n_batches, B, N, D], results [n_batches][B])."""
    L = load_host()
    J, B = len(batches), len(batches[0])
    desc, _, _, _ = lower_json(batches[0][0], None if scenes is None else scenes[0][0])
    N, D = desc.n_steps, desc.chain.n_dof
    sc = None if scenes is None else np.ascontiguousarray(scenes, dtype=np.float64).reshape(J * B, -1, 16)
    n_prims = 0 if sc is None else sc.shape[1]
    arr = (C.c_char_p * (J * B))(*[t.encode() for bt in batches for t in bt])
    x = np.zeros((J * B, N, D))
    res = (abi.Result * (J * B))()
    err = C.create_string_buffer(4096)
    dv = (C.c_int * len(devices))(*devices)
    rc = L.thost_solve_json_stream(arr, J, B, _dp(sc), n_prims, dv, len(devices), inflight, _dp(x), res, err, 4096)
    if rc != 0:
        raise HostError(err.value.decode())
    res = list(res)
    return x.reshape(J, B, N, D), [res[j * B:(j + 1) * B] for j in range(J)]


class PreparedBatch:
    """A batch parsed, lowered and set up on its device ahead of the solve
    (thost_batch_create): `solve()` then runs only the optimisation, which is
    what bench.py times.  A host-loop batch solves once (its models keep their
    warm starts)."""

    def __init__(self, texts, scenes=None, device=0):
        L = load_host()
        self._L = L
        self.B = len(texts)
        desc, _, _, _ = lower_json(texts[0], None if scenes is None else scenes[0])
        self.shape = (self.B, desc.n_steps, desc.chain.n_dof + (1 if desc.use_time else 0))
        sc = None if scenes is None else np.ascontiguousarray(scenes, dtype=np.float64)
        n_prims = 0 if sc is None else sc.shape[1]
        arr = (C.c_char_p * self.B)(*[t.encode() for t in texts])
        h = C.c_void_p()
        err = C.create_string_buffer(4096)
        if L.thost_batch_create(arr, self.B, _dp(sc), n_prims, device, C.byref(h), err, 4096) != 0:
            raise HostError(err.value.decode())
        self._h = h

    def solve(self):
        """-> (x [B, N, D], list of abi.Result)."""
        x = np.zeros(self.shape)
        res = (abi.Result * self.B)()
        err = C.create_string_buffer(4096)
        if self._L.thost_batch_solve(self._h, _dp(x), res, err, 4096) != 0:
            raise HostError(err.value.decode())
        return x, list(res)

    def stats(self):
        """{host_loops, qp_launches, qps, qp_bytes, qp_seconds} (thost_batch_stats)."""
        hl, la, q = C.c_int(0), C.c_longlong(0), C.c_longlong(0)
        by, sec = np.zeros(1), np.zeros(1)
        self._L.thost_batch_stats(self._h, C.byref(hl), C.byref(la), C.byref(q), _dp(by), _dp(sec))
        return {"host_loops": bool(hl.value), "qp_launches": la.value, "qps": q.value,
                "qp_bytes": float(by[0]), "qp_seconds": float(sec[0])}

    def qp_shape(self):
        """{admm_iters, N, nnz_L, levels, widest_level} (thost_batch_qp_shape)."""
        out = (C.c_longlong * 7)()
        self._L.thost_batch_qp_shape(self._h, out)
        return dict(zip(("admm_iters", "N", "nnz_L", "levels", "widest_level", "lds_factor", "lds_bytes"), list(out)))

    def close(self):
        if self._h:
            self._L.thost_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def solve_json(text: str, scene=None, device=0):
    """-> (x [N, D], abi.Result, native) through trajopt::BasicTrustRegionSQP:
    native is True when the problem ran the fused kernel as a batch of one,
    False when it ran the host SQP loop with the GpuModel's QPs."""
    L = load_host()
    desc, _, _, _ = lower_json(text, scene)
    N, D = desc.n_steps, desc.chain.n_dof + (1 if desc.use_time else 0)  # (+ the dt column)
    sc = None if scene is None or len(scene) == 0 else np.ascontiguousarray(scene, dtype=np.float64)
    n_prims = 0 if sc is None else sc.shape[0]
    x = np.zeros((N, D))
    res = abi.Result()
    native = C.c_int(-1)
    err = C.create_string_buffer(4096)
    rc = L.thost_solve_json(text.encode(), _dp(sc), n_prims, device, _dp(x), C.byref(res), C.byref(native), err, 4096)
    if rc != 0:
        raise HostError(err.value.decode())
    return x, res, bool(native.value)


def _quat_wxyz(R):
    """Unit quaternion (w, x, y, z) of a rotation matrix (Shepperd)."""
    R = np.asarray(R, dtype=float)
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0:
        s = math.sqrt(tr + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    q = np.array(q)
    return (q / np.linalg.norm(q)).tolist()


def workload_to_json(wl, b: int) -> str:
    """Problem b of a synthetic workload (configs A, B, C, E, J) in the
    reference's TrajOptRequest JSON format: given_traj init, joint_vel cost,
    cart_pose terms with target_frame torso_lift_link and the target as
    target_frame_offset, joint_pos terms, and the collision term (evaluator
    LVS_DISCRETE, LVS_CONTINUOUS or DISCRETE).  Config E's 14-DoF chain is the
    both_arms group, its tool frames links 11 (left) and 22 (right)."""
    d = wl.desc
    N, D = wl.n_steps, wl.n_dof
    dual = d.chain.n_dof == 14 and d.chain.n_links == 23
    manip = "both_arms" if dual else "right_arm"
    tool_name = {11: "l_gripper_tool_frame", 22: "r_gripper_tool_frame"} if dual else {11: "r_gripper_tool_frame"}
    costs, cnts = [], []
    if d.jv_enabled:
        costs.append({"type": "joint_vel", "params": {
            "coeffs": [d.jv_coeffs[j] for j in range(D)], "targets": [d.jv_targets[j] for j in range(D)],
            "first_step": d.jv_first_step, "last_step": d.jv_last_step}})
    for k in range(d.n_cart):
        T = np.asarray(wl.targets[b, k]).reshape(3, 4)
        term = {"type": "cart_pose", "params": {
            "timestep": d.cart_step[k], "source_frame": tool_name[d.cart_source_link[k]],
            "target_frame": "torso_lift_link",
            "pos_coeffs": [d.cart_pos_coeffs[k][i] for i in range(3)],
            "rot_coeffs": [d.cart_rot_coeffs[k][i] for i in range(3)],
            "target_frame_offset_xyz": T[:, 3].tolist(), "target_frame_offset_wxyz": _quat_wxyz(T[:, :3])}}
        (cnts if d.cart_is_cnt[k] else costs).append(term)
    jt = wl.jpos_targets
    for k in range(d.n_jpos):
        tg = jt[b, k] if jt is not None else [d.jpos_targets[k][j] for j in range(D)]
        term = {"type": "joint_pos", "params": {
            "coeffs": [d.jpos_coeffs[k][j] for j in range(D)], "targets": [float(v) for v in tg],
            "first_step": d.jpos_first_step[k], "last_step": d.jpos_last_step[k]}}
        (cnts if d.jpos_is_cnt[k] else costs).append(term)
    if d.coll_enabled:
        term = {"type": "collision", "params": {
            "coeffs": d.coll_coeff, "dist_pen": d.coll_margin,
            "evaluator_type": {0: 2, 1: 4, 2: 1}[d.coll_continuous],
            "first_step": d.coll_first_step, "last_step": d.coll_last_step if d.coll_last_step >= 0 else N - 1,
            "fixed_steps": [d.coll_fixed_steps[i] for i in range(d.coll_n_fixed)],
            "longest_valid_segment_length": d.coll_lvs}}
        (cnts if d.coll_is_cnt else costs).append(term)
    doc = {
        "basic_info": {"n_steps": N, "manip": manip,
                       "fixed_timesteps": [d.fixed_steps[i] for i in range(d.n_fixed)]},
        "costs": costs,
        "constraints": cnts,
        "init_info": {"type": "given_traj", "data": np.asarray(wl.init[b]).tolist()},
    }
    return json.dumps(doc)


def hostloop_workload_json(wl, b: int, acc_coeff: float = 1.0, jerk_coeff: float = 0.5) -> str:
    """Problem b of `wl` with joint_costs_unit's JointAcc and JointJerk costs
    added (every step, zero targets; trajopt/test/joint_costs_unit.cpp): the
    fused kernel lowers neither, so the problem runs the host SQP loop with its
    QPs batched on the device (bench.py --config HB)."""
    doc = json.loads(workload_to_json(wl, b))
    D = wl.n_dof
    doc["costs"].append({"type": "joint_acc", "params": {"coeffs": [acc_coeff] * D, "targets": [0.0] * D}})
    doc["costs"].append({"type": "joint_jerk", "params": {"coeffs": [jerk_coeff] * D, "targets": [0.0] * D}})
    return json.dumps(doc)
