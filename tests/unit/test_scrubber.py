"""HBM scrubber coordination with claims, on a stand-in agent (no GPU): the sweep buffer is mapped
and unmapped only while no claim-time probe runs (gpupool/agent/scrubber.py ``_probes_quiet``;
a probe beside the free measured 23.8 ms on MI355X, profiles/r4o_bench_gpu1_real.json)."""
from __future__ import annotations

import threading
import time
from types import SimpleNamespace

from gpupool.agent.scrubber import HbmScrubber

UUID = "gpu-0"


class FakeHip:
    def __init__(self):
        self.calls: list[tuple[str, float]] = []

    def sweep_alloc(self, ordinal, reserve):
        self.calls.append(("alloc", time.monotonic()))
        return 0

    def sweep_release(self, ordinal):
        self.calls.append(("release", time.monotonic()))
        return 0

    def hbm_sweep(self, ordinal, offset, nbytes, reserve, keep=True):
        return {"passed": True, "offset": offset, "bytes": nbytes, "span": 8 * nbytes,
                "badBits": 0, "GBps": 6000.0, "ms": 0.1}


def fake_agent():
    hip = FakeHip()
    ledger = SimpleNamespace(sweep_state=lambda: {}, quarantined=lambda: {},
                             commit_sweep=lambda snap: None)
    from gpupool.agent.prober import Prober
    prober = Prober("simulated")
    prober.mode = "inproc"  # the real inproc code path, over the stub library
    prober._hip, prober.ordinals = hip, {"gpu-hip-0": 0}
    prober.warm_arena = lambda dev: None
    return SimpleNamespace(ledger=ledger, prober=prober, lock=threading.RLock(), records={},
                           maintenance={}, by_uuid={UUID: {"uuid": UUID, "hipUUID": "GPU-HIP-0"}},
                           verdicts={UUID: {"healthy": True}}, _pods_by_device=lambda: {}), hip


def test_sweep_buffer_free_waits_for_a_running_claim_probe():
    agent, hip = fake_agent()
    s = HbmScrubber(agent, window_bytes=1 << 20, windows_per_pass=4)
    # a claim of another GPU is probing: the allocation waits for it
    agent.records["gpu-1"] = {"state": "Probing"}
    done = threading.Event()
    t = threading.Thread(target=lambda: (s.scrub_device(UUID), done.set()))
    t.start()
    time.sleep(0.1)
    assert not hip.calls  # not allocated beside the probe
    t_probe_end = time.monotonic()
    with agent.lock:
        agent.records["gpu-1"]["state"] = "Claimed"
    assert done.wait(5)
    kinds = [k for k, _ in hip.calls]
    assert kinds == ["alloc", "release"]
    assert hip.calls[0][1] >= t_probe_end


def test_sweep_buffer_free_after_the_claim_that_interrupted_the_pass():
    """The claim that makes the scrubbed GPU ineligible starts its probe right away; the scrubber
    stops at its next window and frees the buffer only once that probe is done."""
    agent, hip = fake_agent()
    s = HbmScrubber(agent, window_bytes=1 << 20, windows_per_pass=50)
    orig = hip.hbm_sweep

    def window_then_claim(*a, **kw):
        r = orig(*a, **kw)
        if len([c for c in hip.calls if c[0] == "alloc"]) and not agent.records:
            agent.records[UUID] = {"state": "Probing"}  # claimed mid-pass
        return r
    hip.hbm_sweep = window_then_claim
    done = threading.Event()
    threading.Thread(target=lambda: (s.scrub_device(UUID), done.set())).start()
    time.sleep(0.1)
    assert [k for k, _ in hip.calls] == ["alloc"]  # stopped, but the free waits for the probe
    t_probe_end = time.monotonic()
    with agent.lock:
        agent.records[UUID]["state"] = "Claimed"
    assert done.wait(5)
    assert [k for k, _ in hip.calls] == ["alloc", "release"]
    assert hip.calls[1][1] >= t_probe_end
    assert not s._held  # a pod's Allocate (wait_released) may proceed now


def test_probe_wait_is_bounded():
    agent, hip = fake_agent()
    s = HbmScrubber(agent, window_bytes=1 << 20, windows_per_pass=1)
    agent.records["gpu-1"] = {"state": "Probing"}  # a probe that never ends
    t0 = time.monotonic()
    s._probes_quiet(timeout=0.2)
    assert 0.18 < time.monotonic() - t0 < 1.0


def test_no_new_sweep_buffer_while_the_driver_clears_the_last_one():
    agent, hip = fake_agent()
    s = HbmScrubber(agent, window_bytes=1 << 20, windows_per_pass=1)
    s.scrub_device(UUID)
    assert [k for k, _ in hip.calls] == ["alloc", "release"]
    s.scrub_device(UUID)  # within CLEAR_GRACE_S of the free: skipped
    assert [k for k, _ in hip.calls] == ["alloc", "release"]
    s._released_at[UUID] -= s.CLEAR_GRACE_S
    s.scrub_device(UUID)
    assert [k for k, _ in hip.calls] == ["alloc", "release", "alloc", "release"]


def test_no_sweep_buffer_soon_after_a_release_freed_the_gpus_vram():
    """A GPU released by its pool (its pods' VRAM just freed) or seen at agent start is not
    scrubbed until the clear grace has passed since then."""
    agent, hip = fake_agent()
    agent.freed_at = {UUID: time.monotonic()}
    s = HbmScrubber(agent, window_bytes=1 << 20, windows_per_pass=1)
    s.scrub_device(UUID)
    assert hip.calls == []
    agent.freed_at[UUID] -= s.CLEAR_GRACE_S
    s.scrub_device(UUID)
    assert [k for k, _ in hip.calls] == ["alloc", "release"]


def test_agent_notes_vram_freed_by_any_process(tmp_path):
    """A drop of VRAM in use between two samples (a process outside any pool freed memory) marks
    the GPU freed, so the scrubber waits out the driver's clear there too."""
    import json
    import os
    from gpupool.agent.agent import Agent, AgentConfig
    fixture = os.path.join(os.path.dirname(os.path.dirname(__file__)), "fixtures", "node_8x_mi355x.json")
    faults = tmp_path / "faults.json"
    faults.write_text("{}")
    a = Agent(AgentConfig(node="n0", backend="fake", fixture=fixture, state_dir=str(tmp_path / "s"),
                          probe_mode="simulated", probe_sim_ms=0.1, fsync=False, faults=str(faults),
                          scrub_interval_s=0))
    u = next(iter(a.by_uuid))
    a.freed_at[u] = 0.0
    idx = str(a.by_uuid[u]["index"])
    faults.write_text(json.dumps({"devices": {idx: {"memUsedBytes": 200 << 30}}}))
    a.sample()
    assert a.freed_at[u] == 0.0 and a.by_uuid[u]["memUsedBytes"] == 200 << 30
    faults.write_text(json.dumps({"devices": {idx: {"memUsedBytes": 198 << 30}}}))
    a.sample()
    assert a.freed_at[u] == 0.0  # 2 GiB: below the threshold (the probe arena's trim is ~1.2 GiB)
    faults.write_text(json.dumps({"devices": {idx: {"memUsedBytes": 1 << 30}}}))
    a.sample()
    assert a.freed_at[u] > 0.0
