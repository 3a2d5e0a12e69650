"""The device plugin's ListAndWatch lists are numbered in the order they were built
(gpupool/agent/deviceplugin/server.py ``notify``): two claims on one agent notifying at once must
never leave the newest version carrying the older list — the GPUs of the claim whose state the
older list predates would never count as advertised (found by scripts/scale_bench.py at 128 nodes:
pools stuck at 0/2 ready with their GPUs claimed and healthy)."""
from __future__ import annotations

import threading

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
