"""Exit when the process that started this one is gone (``GPUPOOL_EXIT_WITH_PARENT=<pid>``).

The test harness (gpupool/testing/cluster.py) starts the apiserver-sim, fake kubelets, agents and
the manager in their own sessions so it can signal each group; a test runner killed at a timeout
never runs its teardown, and those daemons then ran on for hours. With the variable set, the
daemon polls its parent pid and exits once it was re-parented. The variable is removed from the
environment first, so the daemon's own children (probe helpers, pods) never inherit the check.
Unset in production (a DaemonSet's process has no such parent)."""
from __future__ import annotations

import os
import threading
import time

ENV = "GPUPOOL_EXIT_WITH_PARENT"


def start(poll_s: float = 1.0) -> bool:
    raw = os.environ.pop(ENV, None)
    if not raw:
        return False
    try:
        parent = int(raw)
    except ValueError:
        return False

    def watch() -> None:
        while True:
            if os.getppid() != parent:
                os._exit(0)
            time.sleep(poll_s)
    threading.Thread(target=watch, daemon=True, name="parent-watch").start()
    return True
