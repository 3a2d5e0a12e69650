"""GPU box diagnostic: how do amdsmi's GPU process pids relate to this container's /proc? Holds
2 GiB on GPU 0, then prints its own pid/NSpid, the amdsmi process list and the amdgpu DRM
fdinfo of its own file descriptors."""
import json
import os
import sys
import time

import torch

x = torch.ones(2 << 30, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
out = {"pid": os.getpid()}
out["status"] = [l for l in open("/proc/self/status").read().splitlines() if l.startswith(("NSpid", "NStgid"))]
out["cgroup"] = open("/proc/self/cgroup").read()[-400:]
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from gpupool.ops import devlib  # noqa: E402
snap = devlib.DeviceLib("amdsmi", node="d").snapshot()
out["amdsmi_processes"] = [d.get("processes") for d in snap["devices"]]
fdinfo = {}
for fd in os.listdir("/proc/self/fd"):
    try:
        target = os.readlink(f"/proc/self/fd/{fd}")
        info = open(f"/proc/self/fdinfo/{fd}").read()
    except OSError:
        continue
    if "drm" in info or "kfd" in target or "dri" in target:
        fdinfo[fd] = {"target": target, "info": info[-1200:]}
out["fdinfo"] = fdinfo
try:
    out["kfd_proc"] = {p: os.listdir(f"/sys/class/kfd/kfd/proc/{p}") for p in os.listdir("/sys/class/kfd/kfd/proc")}
except OSError as e:
    out["kfd_proc"] = repr(e)
print(json.dumps(out, indent=1))
