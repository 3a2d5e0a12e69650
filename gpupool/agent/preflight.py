"""Node preflight: the ROCm analogue of "NVIDIA driver + container toolkit installed"
(GPU调度平台搭建.md:115-126), checked instead of assumed, reported as Node condition ``ROCmReady``.

Checks: amdgpu kernel module loaded, /dev/kfd and /dev/dri/renderD* present, ROCm >= 7.0 in
/opt/rocm, every enumerated GPU is gfx950 (MI355X). Read-only: never loads modules or changes
device settings (the GPU box is non-root).
"""
from __future__ import annotations

import glob
import os
import re


def rocm_version(root: str = "/opt/rocm") -> str | None:
    for p in (os.path.join(root, ".info", "version"), os.path.join(root, ".info", "version-dev")):
        try:
            with open(p) as f:
                return f.read().strip()
        except OSError:
            continue
    m = re.search(r"rocm-(\d+\.\d+(\.\d+)?)", os.path.realpath(root))
    return m.group(1) if m else None


def _ver_tuple(v: str) -> tuple[int, ...]:
    return tuple(int(x) for x in re.findall(r"\d+", v)[:3])


def check(snapshot: dict | None, fake: bool = False, sysroot: str = "/") -> dict:
    """Returns {"ready": bool, "checks": {name: {"ok": bool, "detail": str}}}."""
    checks: dict[str, dict] = {}

    def add(name, ok, detail):
        checks[name] = {"ok": bool(ok), "detail": detail}

    if fake:
        add("backend", True, "fake backend: host device checks skipped")
    else:
        mod = os.path.exists(os.path.join(sysroot, "sys/module/amdgpu"))
        add("amdgpuModule", mod, "amdgpu loaded" if mod else "amdgpu kernel module not loaded")
        kfd = os.path.exists(os.path.join(sysroot, "dev/kfd"))
        add("kfd", kfd, "/dev/kfd present" if kfd else "/dev/kfd missing")
        render = sorted(glob.glob(os.path.join(sysroot, "dev/dri/renderD*")))
        add("renderNodes", bool(render), ", ".join(os.path.basename(r) for r in render) or
            "no /dev/dri/renderD* nodes")
        ver = rocm_version(os.path.join(sysroot, "opt/rocm"))
        add("rocmVersion", ver is not None and _ver_tuple(ver) >= (7, 0),
            f"ROCm {ver}" if ver else "ROCm not found under /opt/rocm")
    devs = (snapshot or {}).get("devices", [])
    gfx = sorted({(d.get("asic") or {}).get("gfx", "?") for d in devs})
    add("gfx950", bool(devs) and gfx == ["gfx950"],
        f"{len(devs)} GPU(s): {','.join(gfx) or 'none'}")
    return {"ready": all(c["ok"] for c in checks.values()), "checks": checks}
