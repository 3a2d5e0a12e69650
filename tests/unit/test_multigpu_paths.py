"""Multi-GPU code paths exercised without 8-GPU hardware (the driver's 8-GPU node runs only the
bench): the in-process prober driven with a stub HIP library standing in for libmi355x_probe.so
(same call signatures), over the 8-GPU fake topology.

* ``probe_many`` over 8 GPUs runs the probes concurrently: wall ~ T, not 8T;
* the xGMI peer ring maps every (src -> dst) copy result to its sender, and an injected failure
  on one link fails exactly that sender;
* a claim of 8 and topology-aware subsets with amdsmi-shaped link weights (direct xGMI 15, a
  PCIe-only pair 40, unknown = far) pick the xGMI-packed, single-NUMA sets.
"""
from __future__ import annotations

import json
import os
import threading
import time

import pytest

from gpupool.agent.prober import Prober
from gpupool.ops import devlib

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "node_8x_mi355x.json")


class StubHip:
    """Stands in for gpupool.ops.probe: run() sleeps ``ms`` (GIL released, like the ctypes call)
    and serialises per ordinal like the library's device mutex; peer() fails on chosen links."""

    def __init__(self, ms: float, bad_links: set[tuple[int, int]] = frozenset()):
        self.ms = ms
        self.bad_links = set(bad_links)
        self.calls: list[tuple[str, int, int]] = []
        self._locks = {i: threading.Lock() for i in range(64)}
        self.active = 0
        self.max_active = 0
        self._mu = threading.Lock()

    def run(self, ordinal: int, **kw):
        with self._locks[ordinal]:
            with self._mu:
                self.active += 1
                self.max_active = max(self.max_active, self.active)
            time.sleep(self.ms / 1e3)
            with self._mu:
                self.active -= 1
            self.calls.append(("run", ordinal, -1))
            return {"passed": True, "device": ordinal, "hbm": {"GBps": 5000.0, "badBits": 0},
                    "mfma": {"tflops": 1200.0}, "ms": self.ms}

    def peer(self, a: int, b: int, nbytes: int):
        self.calls.append(("peer", a, b))
        ok = (a, b) not in self.bad_links
        r = {"src": a, "dst": b, "passed": ok, "badBits": 0 if ok else 7, "GBps": 120.0}
        return r


@pytest.fixture
def devices(native_built):
    return devlib.DeviceLib("fake", fixture=FIXTURE, node="n0").snapshot()["devices"]


def inproc_prober(stub: StubHip, devs: list[dict]) -> Prober:
    p = Prober("simulated")
    p.mode = "inproc"  # the real inproc code path, over the stub library
    p._trim_stop = threading.Event()
    p._hip = stub
    p.ordinals = {d["hipUUID"].lower(): d["index"] for d in devs}
    return p


def test_probe_many_runs_eight_gpus_concurrently(devices):
    stub = StubHip(ms=200)
    p = inproc_prober(stub, devices)
    try:
        t0 = time.perf_counter()
        res = p.probe_many(devices, {"enabled": True})
        wall = time.perf_counter() - t0
    finally:
        p.close()
    assert [r["passed"] for r in res] == [True] * 8
    assert sorted(o for k, o, _ in stub.calls if k == "run") == list(range(8))
    assert stub.max_active == 8
    assert wall < 0.9, wall  # ~T (0.2 s), far below 8T (1.6 s)


def test_same_device_probes_serialise_in_the_stub_like_the_library(devices):
    stub = StubHip(ms=100)
    p = inproc_prober(stub, devices)
    try:
        t0 = time.perf_counter()
        res = p.probe_many([devices[0], devices[0]], {"enabled": True})
        wall = time.perf_counter() - t0
    finally:
        p.close()
    assert all(r["passed"] for r in res) and wall >= 0.19 and stub.max_active == 1


def test_peer_ring_maps_each_link_to_its_sender(devices):
    # link 3 -> 4 corrupts data; every other link is clean
    stub = StubHip(ms=1, bad_links={(3, 4)})
    p = inproc_prober(stub, devices)
    try:
        links = p.peer_ring(devices, {"xgmiBytes": 1 << 20})
    finally:
        p.close()
    assert len(links) == 8
    pairs = sorted((a, b) for k, a, b in stub.calls if k == "peer")
    assert pairs == [(i, (i + 1) % 8) for i in range(8)]
    by_index = {d["uuid"]: d["index"] for d in devices}
    for u, r in links.items():
        i = by_index[u]
        assert r["peer"] == devices[(i + 1) % 8]["uuid"]
        assert r["passed"] is (i != 3), (i, r)


class RingStub(StubHip):
    """A library with mi355x_probe_peer_ring: one call for the whole ring."""

    def __init__(self, *a, broken: bool = False, **kw):
        super().__init__(*a, **kw)
        self.broken = broken

    def peer_ring(self, ords: list[int], nbytes: int):
        self.calls.append(("ring", len(ords), nbytes))
        self.ring_ords = list(ords)
        if self.broken:
            return {"passed": False, "error": "hipMemcpyPeerAsync: invalid argument"}
        links = []
        for i, a in enumerate(ords):
            b = ords[(i + 1) % len(ords)]
            ok = (a, b) not in self.bad_links
            links.append({"src": a, "dst": b, "passed": ok, "badBits": 0 if ok else 3,
                          "GBps": 110.0, "ms": 0.6, "bytes": nbytes})
        return {"bytes": nbytes, "links": links, "passed": all(x["passed"] for x in links)}


def test_peer_ring_runs_as_one_concurrent_library_call(devices):
    """With the ring entry point the prober issues ONE call (all links concurrently in the
    library) and maps link i to its sender; pairwise calls are not made."""
    stub = RingStub(ms=1, bad_links={(5, 6)})
    p = inproc_prober(stub, devices)
    try:
        links = p.peer_ring(devices, {"xgmiBytes": 8 << 20})
    finally:
        p.close()
    assert [c for c in stub.calls if c[0] == "ring"] == [("ring", 8, 8 << 20)]
    assert not [c for c in stub.calls if c[0] == "peer"]
    assert stub.ring_ords == [d["index"] for d in devices]
    by_index = {d["uuid"]: d["index"] for d in devices}
    for u, r in links.items():
        i = by_index[u]
        assert r["peer"] == devices[(i + 1) % 8]["uuid"] and r["passed"] is (i != 5), (i, r)


def test_peer_ring_library_error_fails_every_link(devices):
    stub = RingStub(ms=1, broken=True)
    p = inproc_prober(stub, devices[:4])
    try:
        links = p.peer_ring(devices[:4], {})
    finally:
        p.close()
    assert len(links) == 4
    assert all(not r["passed"] and "invalid argument" in r["error"] for r in links.values())


def test_peer_ring_failure_fails_the_right_gpus_probe(tmp_path, native_built):
    """Through the agent: an injected link failure on GPU 2's outgoing link (overlay
    xgmiPeerFail) fails GPU 2's claim-time probe with XGMIPeerCheckFailed, nothing else."""
    from gpupool.agent.agent import Agent, AgentConfig
    faults = tmp_path / "faults.json"
    faults.write_text(json.dumps({"devices": {"2": {"xgmiPeerFail": True}}}))
    a = Agent(AgentConfig(node="n0", backend="fake", fixture=FIXTURE, state_dir=str(tmp_path / "s"),
                          probe_mode="simulated", probe_sim_ms=1, fsync=False, faults=str(faults),
                          scrub_interval_s=0))
    try:
        r = a.claim({"poolUID": "p1", "pool": "default/p", "count": 4, "resourceName": "amd.com/gpu",
                     "policy": {}, "topologyPolicy": "xgmi-packed",
                     "probe": {"enabled": True, "xgmiPeerCheck": True}})
        assert r["ok"]
        failed = {d["index"]: d["probe"] for d in r["devices"] if not d["probe"]["passed"]}
        assert list(failed) == [2] and "XGMIPeerCheckFailed" in failed[2]["error"]
        assert all("xgmi" in d["probe"] for d in r["devices"])
    finally:
        a.stop()


def amdsmi_weights(n: int = 8, pcie: tuple[int, int] | None = None, unknown: tuple[int, int] | None = None):
    """amdsmi_topo_get_link_weight on an 8x MI355X OAM node: every pair one direct xGMI hop
    (weight 15); optionally one pair reached over PCIe (weight 40) and one pair unreported."""
    w = [[0 if i == j else 15 for j in range(n)] for i in range(n)]
    if pcie:
        a, b = pcie
        w[a][b] = w[b][a] = 40
    if unknown:
        a, b = unknown
        w[a][b] = w[b][a] = None
    return w


def test_select_eight_and_xgmi_packed_subsets(native_built):
    numa = [0, 0, 0, 0, 1, 1, 1, 1]
    assert devlib.select(8, list(range(8)), [], "xgmi-packed", amdsmi_weights(), numa) == list(range(8))
    assert devlib.select(9, list(range(8)), [], "xgmi-packed", amdsmi_weights(), numa) == []
    # 4 of 8: one NUMA node
    assert devlib.select(4, list(range(8)), [], "xgmi-packed", amdsmi_weights(), numa) == [0, 1, 2, 3]
    # GPU 1 reaches GPU 0 only over PCIe: a set of 4 that avoids the slow pair wins
    sel = devlib.select(4, list(range(8)), [], "xgmi-packed", amdsmi_weights(pcie=(0, 1)), numa)
    assert not {0, 1} <= set(sel), sel
    # an unreported link counts as far
    sel = devlib.select(2, [2, 3, 5], [], "xgmi-packed", amdsmi_weights(unknown=(2, 3)), numa)
    assert sel != [2, 3], sel
    # growing an owned set prefers its NUMA node
    assert devlib.select(2, [3, 4, 5, 6], [0, 1, 2], "xgmi-packed", amdsmi_weights(), numa)[0] == 3


def _rccl_check_world2(extra_rank1: list[str]) -> list[tuple[int, dict]]:
    """Two gloo ranks of gpupool.parallel.rccl_check on the CPU (the N>1 bench's comm check)."""
    import json
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, "-m", "gpupool.parallel.rccl_check", "--rank", str(r),
                               "--world", "2", "--master-port", str(port), "--backend", "gloo",
                               "--device", "cpu", "--bytes", str(1 << 20), "--iters", "2",
                               "--warmup", "1"] + (extra_rank1 if r == 1 else []),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=ROOT)
             for r in range(2)]
    out = []
    for p in procs:
        so, se = p.communicate(timeout=120)
        lines = [x for x in so.splitlines() if x.startswith("{")]
        out.append((p.returncode, json.loads(lines[-1]) if lines else {"stderr": se[-1500:]}))
    return out


def test_rccl_check_proves_data_moved_between_ranks():
    """Rank r contributes r + 1: only a real reduction over both ranks yields 3 everywhere."""
    res = _rccl_check_world2([])
    for rc, o in res:
        assert rc == 0 and o["exact"] and o["expected"] == 3 and o["got"] == [3.0, 3.0], o


def test_rccl_check_fails_a_rank_that_skipped_the_reduction():
    """A rank that joins the collective but drops its result keeps its own contribution (2): the
    harness fails it (exit 2) — a local copy cannot pass as a collective."""
    res = _rccl_check_world2(["--inject", "skip-reduce"])
    rc1, o1 = res[1]
    assert rc1 == 2 and o1["exact"] is False and o1["got"] == [2.0, 2.0], o1
