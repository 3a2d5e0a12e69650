"""Node preflight against synthetic sysroots."""
from __future__ import annotations

import os

from gpupool.agent import preflight


def _root(tmp_path, kfd=True, module=True, render=True, rocm="7.2.0", kernel="6.18.54-ant.1",
          dkms=None):
    r = tmp_path / "root"
    (r / "dev" / "dri").mkdir(parents=True)
    (r / "proc" / "sys" / "kernel").mkdir(parents=True)
    (r / "proc" / "sys" / "kernel" / "osrelease").write_text(kernel + "\n")
    if kfd:
        (r / "dev" / "kfd").write_text("")
    if render:
        (r / "dev" / "dri" / "renderD128").write_text("")
    if module:
        (r / "sys" / "module" / "amdgpu").mkdir(parents=True)
        if dkms:
            (r / "sys" / "module" / "amdgpu" / "version").write_text(dkms + "\n")
    if rocm:
        (r / "opt" / "rocm" / ".info").mkdir(parents=True)
        (r / "opt" / "rocm" / ".info" / "version").write_text(rocm)
    return str(r) + os.sep


SNAP = {"devices": [{"asic": {"gfx": "gfx950"}}] * 2}


def test_all_good(tmp_path):
    out = preflight.check(SNAP, sysroot=_root(tmp_path))
    assert out["ready"], out


def test_missing_kfd_and_old_rocm(tmp_path):
    out = preflight.check(SNAP, sysroot=_root(tmp_path, kfd=False, rocm="6.4.1"))
    assert not out["ready"]
    assert not out["checks"]["kfd"]["ok"] and not out["checks"]["rocmVersion"]["ok"]


def test_wrong_arch_and_fake(tmp_path):
    out = preflight.check({"devices": [{"asic": {"gfx": "gfx942"}}]}, sysroot=_root(tmp_path))
    assert not out["checks"]["gfx950"]["ok"]
    assert preflight.check(SNAP, fake=True)["ready"]


def test_this_image_rocm_version():
    v = preflight.rocm_version()
    assert v is None or preflight._ver_tuple(v) >= (7, 0)


# ---- the host amdgpu driver against the image's ROCm user space
FACTS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fixtures",
                     "real_mi355x", "driver_facts.json")


def test_host_driver_present_and_compatible(tmp_path):
    import json
    facts = json.load(open(FACTS))  # the GPU box: in-tree amdgpu of Linux 6.18, ROCm 7.2.0
    out = preflight.check(SNAP, sysroot=_root(tmp_path, kernel=facts["kernelRelease"],
                                              rocm=facts["rocmVersion"]))
    hd = out["checks"]["hostDriver"]
    assert out["ready"] and hd["ok"], out
    assert "in-tree (Linux 6.18.54-ant.1)" in hd["detail"] and "ROCm 7.2.0" in hd["detail"]
    assert hd["driver"] == {"loaded": True, "kind": "in-tree", "version": None,
                            "kernel": facts["kernelRelease"]}
    r2 = tmp_path / "dkms"
    r2.mkdir()
    out = preflight.check(SNAP, sysroot=_root(r2, dkms="6.16.6", rocm="7.2.0"))
    assert out["checks"]["hostDriver"]["ok"], out["checks"]["hostDriver"]
    assert "6.16.6 (DKMS)" in out["checks"]["hostDriver"]["detail"]


def test_host_driver_missing(tmp_path):
    out = preflight.check(SNAP, sysroot=_root(tmp_path, module=False))
    assert not out["ready"]
    assert not out["checks"]["hostDriver"]["ok"]
    assert "not loaded" in out["checks"]["hostDriver"]["detail"]


def test_host_driver_too_old_for_the_images_rocm(tmp_path):
    # the ROCm 6.4 DKMS driver under ROCm 7.2 user space (needs 7.1's or 7.2's)
    out = preflight.check(SNAP, sysroot=_root(tmp_path, dkms="6.12.12", rocm="7.2.0"))
    hd = out["checks"]["hostDriver"]
    assert not out["ready"] and not hd["ok"] and "too old, needs >= 6.16" in hd["detail"], hd
    # an in-tree amdgpu of a kernel that predates gfx950
    r2 = tmp_path / "old"
    r2.mkdir()
    out = preflight.check(SNAP, sysroot=_root(r2, kernel="6.8.0-45-generic"))
    assert not out["checks"]["hostDriver"]["ok"]
    assert "gfx950 needs Linux >= 6.14" in out["checks"]["hostDriver"]["detail"]
    # ROCm 7.0 user space accepts the driver of the release before it too (6.4's 6.12 no: gfx950
    # arrived with 7.0's driver)
    r3 = tmp_path / "r70"
    r3.mkdir()
    assert not preflight.check(SNAP, sysroot=_root(r3, dkms="6.12.12", rocm="7.0.2"))["ready"]
    r4 = tmp_path / "r71"
    r4.mkdir()
    assert preflight.check(SNAP, sysroot=_root(r4, dkms="6.14.14", rocm="7.1.0"))["ready"]
