"""Long-running daemons must not leak: the node agent and the manager go through many claim /
release cycles (pool 0 -> N -> 0) and their thread count, open descriptors and resident memory
are sampled from /proc. A leak of one thread, socket or stream per claim, or of the claim path's
per-call state, shows as growth proportional to the cycle count."""
from __future__ import annotations

import os
import time

import pytest

from gpupool.kube import MI355XPOOLS

from .helpers import mi_pool, wait_ready

pytestmark = pytest.mark.slow


def _proc(pid: int) -> dict:
    out = {"fds": len(os.listdir(f"/proc/{pid}/fd"))}
    with open(f"/proc/{pid}/status") as f:
        for line in f:
            if line.startswith("Threads:"):
                out["threads"] = int(line.split()[1])
            elif line.startswith("VmRSS:"):
                out["rss_kib"] = int(line.split()[1])
    return out


def test_claim_release_cycles_do_not_leak(cluster_factory):
    c = cluster_factory()
    k = c.client
    agent = c.procs["agent-mi355x-node-0"].pid
    manager = c.procs["manager"].pid
    k.create(MI355XPOOLS, mi_pool("p", 0), "default")
    wait_ready(k, "p", 0)
    samples = []
    for cycle in range(60):
        for r in (8, 3, 0):
            k.patch(MI355XPOOLS, "p", {"spec": {"replicas": r}}, "default")
            wait_ready(k, "p", r)
        if cycle in (15, 59):
            time.sleep(1.0)  # let per-claim threads and streams wind down before sampling
            samples.append({"agent": _proc(agent), "manager": _proc(manager)})
    (a0, a1) = samples[0]["agent"], samples[1]["agent"]
    (m0, m1) = samples[0]["manager"], samples[1]["manager"]
    print("agent", a0, "->", a1, "manager", m0, "->", m1)
    for before, after, who in ((a0, a1, "agent"), (m0, m1, "manager")):
        assert after["threads"] - before["threads"] <= 3, (who, before, after)
        assert after["fds"] - before["fds"] <= 4, (who, before, after)
        # 44 cycles x 2 claims: a leak of even 100 KiB per claim would show as ~9 MiB
        assert after["rss_kib"] - before["rss_kib"] < 8 * 1024, (who, before, after)
