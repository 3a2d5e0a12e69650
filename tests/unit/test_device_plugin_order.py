"""The device plugin's ListAndWatch lists are numbered in the order they were built
(gpupool/agent/deviceplugin/server.py ``notify``): two claims on one agent notifying at once must
never leave the newest version carrying the older list — the GPUs of the claim whose state the
older list predates would never count as advertised (found by scripts/scale_bench.py at 128 nodes:
pools stuck at 0/2 ready with their GPUs claimed and healthy)."""
from __future__ import annotations

import random
import threading
import time

from gpupool.agent.deviceplugin.server import DevicePluginServer


class StubAgent:
    def __init__(self):
        self.claimed = {"g0"}
        self.a_built = threading.Event()
        self.b_in = threading.Event()

    def plugin_devices(self, resource):
        snap = sorted(self.claimed)
        if threading.current_thread().name == "claim-a":
            self.a_built.set()        # claim A has its list ...
            self.b_in.wait(0.5)       # ... and is descheduled while claim B notifies
        return [{"uuid": u, "advertisable": True} for u in snap]

    def mark_advertised(self, resource, healthy):
        pass


def test_the_newest_version_carries_the_newest_list(tmp_path):
    agent = StubAgent()
    dp = DevicePluginServer(agent, "amd.com/gpu", str(tmp_path))

    def claim_b():
        agent.a_built.wait(5)
        agent.claimed.add("g1")       # claim B committed its GPU after A built A's list
        agent.b_in.set()
        dp.notify()

    a = threading.Thread(target=dp.notify, name="claim-a")
    b = threading.Thread(target=claim_b, name="claim-b")
    a.start()
    b.start()
    a.join(5)
    b.join(5)
    ver, resp, healthy = dp._pending
    assert ver == 2
    assert healthy == {"g0", "g1"}, healthy
    assert sorted(d.ID for d in resp.devices) == ["g0", "g1"]


def test_concurrent_notifies_end_on_the_final_state(tmp_path):
    """Eight claims commit a GPU each and notify at once, with the device-list build descheduled
    at random points: whatever the interleaving, the newest version lists every GPU."""
    class Racy(StubAgent):
        def __init__(self, rng):
            super().__init__()
            self.claimed = set()
            self.rng = rng
            self.mu = threading.Lock()

        def plugin_devices(self, resource):
            with self.mu:
                snap = sorted(self.claimed)
            time.sleep(self.rng.random() * 0.002)  # descheduled after reading the state
            return [{"uuid": u, "advertisable": True} for u in snap]

    for seed in range(20):
        rng = random.Random(seed)
        agent = Racy(rng)
        dp = DevicePluginServer(agent, "amd.com/gpu", str(tmp_path))

        def claim(i):
            time.sleep(rng.random() * 0.001)
            with agent.mu:
                agent.claimed.add(f"g{i}")
            dp.notify()
        ts = [threading.Thread(target=claim, args=(i,)) for i in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(5)
        ver, _, healthy = dp._pending
        assert ver == 8 and healthy == {f"g{i}" for i in range(8)}, (seed, healthy)
