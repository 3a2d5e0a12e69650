"""Node preflight: the ROCm analogue of "NVIDIA driver + container toolkit installed"
(GPU调度平台搭建.md:115-126), checked instead of assumed, reported as Node condition ``ROCmReady``.

Checks: amdgpu kernel module loaded, the HOST's amdgpu driver able to serve this image's ROCm user
space on gfx950 (the reference's driver step is about the node's kernel driver, not a container's
libraries: GPU调度平台搭建.md:115-126), /dev/kfd and /dev/dri/renderD* present, ROCm >= 7.0 in
/opt/rocm, every enumerated GPU is gfx950 (MI355X). Read-only: never loads modules or changes
device settings (the GPU box is non-root).

The driver is read through the host's /sys (the DaemonSet's hostPath) and kernel release:
  * an out-of-tree (DKMS) amdgpu reports ``/sys/module/amdgpu/version`` ("6.14.14"): AMD ships one
    driver series with each ROCm release, and ROCm user space is supported on the driver of its own
    release and of the release before it (``AMDGPU_DKMS_FOR_ROCM``);
  * the kernel's in-tree amdgpu has no version file: the kernel release decides; gfx950 (GC 9.5.0)
    needs ``MIN_KERNEL_GFX950``.
The table is AMD's published pairing as far as it can be reproduced without network access (parity
unpinned beyond the pairing measured on the GPU box: in-tree amdgpu of Linux 6.18 with ROCm 7.2
user space, tests/fixtures/real_mi355x/driver_facts.json).
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


# ROCm user-space release -> the amdgpu (DKMS) driver series shipped with it
AMDGPU_DKMS_FOR_ROCM = {(6, 2): (6, 8), (6, 3): (6, 10), (6, 4): (6, 12), (7, 0): (6, 14),
                        (7, 1): (6, 16), (7, 2): (6, 16)}
GFX950_MIN_DKMS = (6, 14)      # MI355X support arrived with the ROCm 7.0 driver
MIN_KERNEL_GFX950 = (6, 14)    # in-tree amdgpu with GC 9.5.0 (gfx950)


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def host_driver(sysroot: str = "/") -> dict:
    """The node's amdgpu driver: {loaded, kind: dkms|in-tree, version, kernel}."""
    loaded = os.path.isdir(os.path.join(sysroot, "sys/module/amdgpu"))
    ver = _read(os.path.join(sysroot, "sys/module/amdgpu/version"))
    kernel = _read(os.path.join(sysroot, "proc/sys/kernel/osrelease"))
    return {"loaded": loaded, "kind": "dkms" if ver else "in-tree", "version": ver,
            "kernel": kernel}


def driver_compatible(drv: dict, rocm: str | None) -> tuple[bool, str]:
    """Can the host driver ``drv`` serve ROCm user space ``rocm`` on gfx950? (ok, detail)"""
    if not drv.get("loaded"):
        return False, "host amdgpu driver not loaded (no /sys/module/amdgpu)"
    user = f"ROCm {rocm} user space" if rocm else "ROCm user space (version unknown)"
    if drv.get("kind") == "dkms":
        have = _ver_tuple(drv["version"])[:2]
        rv = _ver_tuple(rocm or "")[:2]
        known = sorted(AMDGPU_DKMS_FOR_ROCM)
        # the driver of this ROCm release or of the one before it (nearest known release at or
        # below a ROCm newer than the table)
        at = max((k for k in known if k <= rv), default=None) if rv else None
        need = GFX950_MIN_DKMS
        if at is not None:
            i = known.index(at)
            need = max(need, AMDGPU_DKMS_FOR_ROCM[known[max(0, i - 1)]])
        ok = have >= need
        return ok, (f"host amdgpu {drv['version']} (DKMS) with {user}: "
                    + ("ok" if ok else f"too old, needs >= {need[0]}.{need[1]}"))
    k = _ver_tuple(drv.get("kernel") or "")[:2]
    ok = bool(k) and k >= MIN_KERNEL_GFX950
    return ok, (f"host amdgpu in-tree (Linux {drv.get('kernel') or '?'}) with {user}: "
                + ("ok" if ok else f"gfx950 needs Linux >= {MIN_KERNEL_GFX950[0]}."
                                   f"{MIN_KERNEL_GFX950[1]}"))


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
        drv = host_driver(sysroot)
        ok, detail = driver_compatible(drv, ver)
        add("hostDriver", ok, detail)
        checks["hostDriver"]["driver"] = drv
    devs = (snapshot or {}).get("devices", [])
    gfx = sorted({(d.get("asic") or {}).get("gfx", "?") for d in devs})
    add("gfx950", bool(devs) and gfx == ["gfx950"],
        f"{len(devs)} GPU(s): {','.join(gfx) or 'none'}")
    return {"ready": all(c["ok"] for c in checks.values()), "checks": checks}
