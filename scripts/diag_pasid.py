"""GPU box diagnostic for per-pod accounting: two child processes hold 2 and 6 GiB; print the
amdsmi process list, each KFD proc entry's pasid file, and the local render-node fdinfo pasids."""
import json
import os
import subprocess
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", ".")
sys.path.insert(0, ROOT)
HOLD = ("import torch, time, sys\n"
        "x = torch.ones(int(sys.argv[1]), dtype=torch.uint8, device='cuda'); torch.cuda.synchronize()\n"
        "print('ready', flush=True); time.sleep(30)\n")
kids = [subprocess.Popen([sys.executable, "-c", HOLD, str(n << 30)], stdout=subprocess.PIPE, text=True)
        for n in (2, 6)]
for k in kids:
    k.stdout.readline()
out = {"kids": [k.pid for k in kids]}
from gpupool.ops import devlib  # noqa: E402
from gpupool.agent.agent import _scan_pasids  # noqa: E402
snap = devlib.DeviceLib("amdsmi", node="d").snapshot()
out["amdsmi"] = [d.get("processes") for d in snap["devices"]]
kfd = {}
for p in os.listdir("/sys/class/kfd/kfd/proc"):
    try:
        kfd[p] = open(f"/sys/class/kfd/kfd/proc/{p}/pasid").read().strip()
    except OSError as e:
        kfd[p] = repr(e)
out["kfd_pasid"] = kfd
out["local_scan"] = _scan_pasids()
for k in kids:
    fds = {}
    for fd in os.listdir(f"/proc/{k.pid}/fd"):
        try:
            t = os.readlink(f"/proc/{k.pid}/fd/{fd}")
        except OSError:
            continue
        if "dri" in t or "kfd" in t:
            info = open(f"/proc/{k.pid}/fdinfo/{fd}").read()
            fds[fd] = [t] + [l for l in info.splitlines() if l.startswith(("pasid", "drm-client", "drm-memory-vram", "drm-pdev"))]
    out[f"kid_{k.pid}"] = fds
print(json.dumps(out, indent=1))
for k in kids:
    k.kill()
