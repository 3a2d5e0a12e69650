"""Daemons started by the test harness exit once the process that started them is gone
(``GPUPOOL_EXIT_WITH_PARENT``, gpupool/utils/parent_watch.py and the manager's main): a test runner
killed at a timeout skips its teardown, and its apiserver-sim, kubelets, agents and manager used to
run on for hours."""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MANAGER = os.path.join(ROOT, "build", "native", "gpupool-manager")

PARENT = r"""
import os, subprocess, sys, time
env = dict(os.environ, GPUPOOL_EXIT_WITH_PARENT=str(os.getpid()), PYTHONPATH=sys.argv[1])
p = subprocess.Popen(sys.argv[2:], env=env, start_new_session=True, cwd=sys.argv[1],
                     stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
print(p.pid, flush=True)
time.sleep(120)
"""


def alive(pid: int) -> bool:
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except FileNotFoundError:
        return False


def orphan_exits(argv: list[str], within: float) -> float:
    parent = subprocess.Popen([sys.executable, "-c", PARENT, ROOT, *argv], stdout=subprocess.PIPE,
                              text=True)
    child = int(parent.stdout.readline())
    try:
        time.sleep(1.0)
        assert alive(child), "the daemon did not start"
        t0 = time.monotonic()
        parent.send_signal(signal.SIGKILL)  # no teardown
        parent.wait(5)
        while alive(child) and time.monotonic() - t0 < within:
            time.sleep(0.1)
        return time.monotonic() - t0 if not alive(child) else -1.0
    finally:
        if alive(child):
            os.kill(child, signal.SIGKILL)


def test_an_orphaned_apiserver_sim_exits(tmp_path):
    dt = orphan_exits([sys.executable, "-m", "gpupool.apiserver_sim", "--port", "0", "--port-file",
                       str(tmp_path / "port"), "--crd-dir", os.path.join(ROOT, "config", "crd")], 10)
    assert 0 <= dt < 5, dt


@pytest.mark.skipif(not os.path.exists(MANAGER), reason="native manager not built")
def test_an_orphaned_manager_exits(tmp_path):
    dt = orphan_exits([MANAGER, "--apiserver", "http://127.0.0.1:9", "--port-file",
                       str(tmp_path / "mport")], 30)
    # SIGTERM to itself, then the normal shutdown: informer backoffs are interruptible (it took
    # 15 s with the apiserver unreachable before they were)
    assert 0 <= dt < 6, dt
