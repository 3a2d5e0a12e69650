"""Node preflight against synthetic sysroots."""
from __future__ import annotations

import os

from gpupool.agent import preflight


def _root(tmp_path, kfd=True, module=True, render=True, rocm="7.2.0"):
    r = tmp_path / "root"
    (r / "dev" / "dri").mkdir(parents=True)
    if kfd:
        (r / "dev" / "kfd").write_text("")
    if render:
        (r / "dev" / "dri" / "renderD128").write_text("")
    if module:
        (r / "sys" / "module" / "amdgpu").mkdir(parents=True)
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
