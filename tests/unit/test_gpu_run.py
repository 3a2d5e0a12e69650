"""scripts/gpu_run.py: every GPU-box scenario still runs against this tree (its scripts exist,
compile and answer --help without a GPU), so a measurement launcher cannot rot silently."""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_every_scenario_dry_runs():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "gpu_run.py"), "--dry-run",
                        "all"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    steps = [ln for ln in r.stdout.splitlines() if ln.startswith("[")]
    assert len(steps) >= 15 and all(ln.endswith("ok") for ln in steps), r.stdout
    # every maintained script is reachable from a scenario (or is a CPU tool)
    cpu_tools = {"gen_manifests.py", "gen_fake_fixture.py", "run_local.py", "scale_bench.py",
                 "claim_rpc_bench.py", "gpu_run.py"}
    used = {os.path.basename(w) for ln in steps for w in ln.split() if w.endswith(".py")}
    for f in os.listdir(os.path.join(ROOT, "scripts")):
        if f.endswith(".py"):
            assert f in used or f in cpu_tools, f"scripts/{f} is run by no scenario"
    assert not [f for f in os.listdir(os.path.join(ROOT, "scripts")) if f.endswith(".sh")]


def test_unknown_scenario_is_refused():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "gpu_run.py"), "nope"],
                       capture_output=True, text=True, timeout=60, cwd=ROOT)
    assert r.returncode == 2 and "unknown scenario" in r.stderr
