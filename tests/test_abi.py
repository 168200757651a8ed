"""C-ABI checks that need no GPU: the HIP library loads, exports every entry
point include/trajopt_hip.h declares, agrees on struct layouts and defaults,
and validates descriptors before touching a device."""
import ctypes as C
import subprocess

import numpy as np
import pytest

from trajopt_amd import abi, problems


@pytest.fixture(scope="module")
def lib():
    if not abi.HIP_LIB.exists():
        import __graft_entry__

        __graft_entry__.build()
    return abi.load_hip()


def test_exports_every_declared_symbol(lib):
    declared = abi.exported_symbols()
    assert len(declared) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", str(abi.HIP_LIB)], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    for s in declared:
        assert hasattr(lib, s)


def test_host_library_exports_every_declared_symbol(lib):
    import re

    from trajopt_amd import host

    hdr = (abi.PKG_DIR.parent / "include" / "trajopt_host.h").read_text()
    declared = sorted(set(re.findall(r"\b(thost_[a-z_]+)\s*\(", hdr)))
    assert len(declared) >= 2
    out = subprocess.run(["nm", "-D", "--defined-only", str(host.HOST_LIB)], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    assert not [s for s in declared if s not in exported]


def test_struct_layout_and_build_info(lib):
    assert lib.thip_sizeof_desc() == C.sizeof(abi.ProblemDesc)
    info = lib.thip_build_info().decode()
    assert "gfx950" in info


def test_defaults_match_reference_values(lib):
    """optimizers.hpp:92-135 and osqp_interface.cpp:78-90 (+ OSQP 1.0 defaults)."""
    p = abi.SqpParams()
    lib.thip_default_sqp_params(C.byref(p))
    q = abi.default_sqp_params()
    for name, _ in abi.SqpParams._fields_:
        assert getattr(p, name) == getattr(q, name), name
    s = abi.OsqpSettings()
    lib.thip_default_osqp_settings(C.byref(s))
    t = abi.default_osqp_settings()
    for name, _ in abi.OsqpSettings._fields_:
        assert getattr(s, name) == getattr(t, name), name
    assert s.eps_abs == 1e-4 and s.eps_rel == 1e-6 and s.max_iter == 8192 and s.polish_refine_iter == 3


def _with_collision(d, evaluator):
    c = problems.make_workload("C", 1).desc
    for name, _ in abi.ProblemDesc._fields_:
        if name.startswith("coll_") or name in ("n_spheres", "sphere_link", "sphere_center", "sphere_radius", "n_prims"):
            setattr(d, name, getattr(c, name))
    d.coll_first_step, d.coll_last_step = 0, -1
    d.coll_continuous = evaluator


def _create(lib, desc, batch=4):
    ctx = C.c_void_p()
    rc = lib.thip_create(0, C.byref(desc), batch, C.byref(ctx))
    return rc, ctx


@pytest.mark.parametrize(
    "mutate, needle",
    [
        (lambda d: setattr(d, "n_steps", 1), "n_steps"),
        (lambda d: setattr(d, "n_steps", 65), "n_steps"),
        (lambda d: setattr(d.osqp, "max_iter", 0), "OSQP"),
        (lambda d: setattr(d, "coll_enabled", 1), "n_spheres"),
        (lambda d: setattr(d, "n_cart", 65), "cart"),
        (lambda d: setattr(d, "n_jpos", 9), "n_jpos"),
        (lambda d: (setattr(d, "n_jpos", 1), d.jpos_upper_tols[0].__setitem__(2, float("inf"))), "finite"),
        (lambda d: (setattr(d, "n_jpos", 1), d.jpos_coeffs[0].__setitem__(0, float("nan"))), "finite"),
        (lambda d: (d.cart_has_tol.__setitem__(0, 1), d.cart_lower_tol[0].__setitem__(3, 0.3)),
         "Inverted tolerance band"),
        (lambda d: setattr(d, "n_jvx", 5), "n_jvx"),
        (lambda d: setattr(d, "n_jvx", 1), "tolerance forms"),
        (lambda d: _with_collision(d, 3), "coll_continuous"),
    ],
)
def test_create_rejects_invalid_descriptors(lib, mutate, needle):
    wl = problems.make_workload("A", 1)
    d = wl.desc
    mutate(d)
    rc, ctx = _create(lib, d)
    assert rc == -1
    assert not ctx
    msg = lib.thip_last_error(None).decode()
    assert needle.lower() in msg.lower(), msg


def test_create_rejects_bad_batch(lib):
    wl = problems.make_workload("A", 1)
    rc, _ = _create(lib, wl.desc, batch=0)
    assert rc == -1


def test_calls_on_null_context_fail_cleanly(lib):
    assert lib.thip_sqp_run(None) == -1
    assert lib.thip_upload(None, None, None, None) == -1
    assert lib.thip_upload_joint_targets(None, None) == -1
    assert lib.thip_download(None, None, None) == -1
    assert lib.thip_last_kernel_ms(None) < 0
    lib.thip_destroy(None)


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    """No CPU fallback: a missing HIP library is an error."""
    monkeypatch.setattr(abi, "HIP_LIB", tmp_path / "missing.so")
    monkeypatch.setattr(abi, "_hip", None)
    with pytest.raises(RuntimeError, match="missing"):
        abi.load_hip()


def test_jdt_fused_domain(lib):
    """thip_jdt_fused (trajopt_hip.h): the fused kernel takes JointAccEqCost terms on an
    even number of waypoints with 2 n_dof <= 16; every other joint-derivative form (a
    constraint, tolerances, JointJerk, an odd horizon) is the generic path's."""
    def fused(wl):
        return lib.thip_jdt_fused(C.byref(wl.desc))

    assert fused(problems.make_workload("B", 1)) == 1  # no jdt terms
    assert fused(problems.with_joint_acc(problems.make_workload("B", 1))) == 1
    assert fused(problems.make_workload("HA", 1)) == 1
    assert fused(problems.with_joint_acc(problems.make_workload("B", 1, n_steps=29))) == 0
    wl = problems.with_joint_acc(problems.make_workload("B", 1))
    wl.desc.jdt_is_cnt[0] = 1
    assert fused(wl) == 0
    wl = problems.with_joint_acc(problems.make_workload("B", 1))
    wl.desc.jdt_upper_tols[0][3] = 0.1
    assert fused(wl) == 0
    wl = problems.with_joint_acc(problems.make_workload("B", 1))
    wl.desc.jdt_order[0] = 3
    assert fused(wl) == 0
    assert fused(problems.with_joint_acc(problems.make_workload("E", 1))) == 0  # 2 x 14 dofs > 16
