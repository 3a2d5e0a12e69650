"""Agent-side leader fencing (gpupool/agent/fence.py, the agent's ``check_leader`` guard): the newest manager epoch
seen on a mutating RPC is persisted in the ledger and older epochs are refused (409 StaleLeader)
before the handler runs — also after an agent restart. Requests without a token (leader election
off, gpuctl) pass unchecked."""
from __future__ import annotations

import json
import os

import pytest

from gpupool.agent.agent import Agent, AgentConfig

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "node_8x_mi355x.json")


def make_agent(tmp_path) -> Agent:
    return Agent(AgentConfig(node="n0", backend="fake", fixture=FIXTURE, count=2,
                             state_dir=str(tmp_path / "state"), probe_mode="simulated",
                             probe_sim_ms=0, fsync=False, scrub_interval_s=0))


def tok(holder: str, epoch: int, lease: str | None = None) -> dict:
    h = {"x-gpupool-leader": holder, "x-gpupool-leader-epoch": str(epoch)}
    if lease is not None:
        h["x-gpupool-leader-lease"] = lease
    return h


def test_older_epochs_are_refused_and_the_newest_survives_a_restart(tmp_path, native_built):
    a = make_agent(tmp_path)
    assert a.check_leader("POST", "/v1/claims", tok("m-a", 3)) is None
    assert a.check_leader("POST", "/v1/release", tok("m-a", 3)) is None  # same leader again
    assert a.check_leader("POST", "/v1/claims", tok("m-b", 4)) is None   # a successor
    r = a.check_leader("POST", "/v1/claims", tok("m-a", 3))              # the old one resumes
    assert r[0] == 409 and json.loads(r[2])["reason"] == "StaleLeader"
    r = a.check_leader("POST", "/v1/cordon", tok("m-c", 4))  # same epoch, another holder
    assert r[0] == 409
    assert a.stats["stale_leader_refused"] == 2
    # not mutating / no token: never checked
    assert a.check_leader("GET", "/v1/node", tok("m-a", 0)) is None
    assert a.check_leader("POST", "/v1/claims", {}) is None
    a.stop()
    b = make_agent(tmp_path)  # restart: the fence is in the ledger
    assert b.leader_fence["holder"] == "m-b" and b.leader_fence["epoch"] == 4
    assert b.check_leader("POST", "/v1/release", tok("m-a", 3))[0] == 409
    assert b.check_leader("POST", "/v1/release", tok("m-b", 4)) is None
    b.stop()


def test_a_refused_request_never_reaches_its_handler(tmp_path, native_built):
    from gpupool.agent.agent import build_routes
    from gpupool.agent.rpc import RpcServer
    a = make_agent(tmp_path)
    srv = RpcServer(build_routes(a), guard=a.check_leader)
    a.check_leader("POST", "/v1/claims", tok("new", 7))
    out = srv._dispatch("POST", "/v1/claims", tok("old", 6),
                        json.dumps({"poolUID": "p", "count": 1}).encode())
    assert out[0] == 409 and not a.records  # nothing claimed
    out = srv._dispatch("POST", "/v1/claims", tok("new", 7),
                        json.dumps({"poolUID": "p", "count": 1}).encode())
    assert out[0] == 200 and len(a.records) == 1
    srv.close()
    a.stop()


def test_a_recreated_lease_starts_a_new_generation(tmp_path, native_built):
    """leaseTransitions restarts at 0 when the Lease is deleted and created again: its new leader
    must be accepted (or no claim would ever pass again), and a leader of the deleted Lease —
    whatever its epoch — refused."""
    a = make_agent(tmp_path)
    old = "2026-10-18T01:00:00Z uid-old"
    new = "2026-10-18T02:00:00Z uid-new"
    assert a.check_leader("POST", "/v1/claims", tok("m-a", 5, old)) is None
    assert a.check_leader("POST", "/v1/claims", tok("m-b", 0, new)) is None  # recreated Lease
    assert a.leader_fence["leaseUID"] == "uid-new" and a.leader_fence["epoch"] == 0
    r = a.check_leader("POST", "/v1/release", tok("m-a", 5, old))  # the deleted Lease's leader
    assert r[0] == 409 and "newer Lease" in json.loads(r[2])["message"]
    assert a.check_leader("POST", "/v1/release", tok("m-b", 1, new)) is None
    assert a.check_leader("POST", "/v1/release", tok("m-b", 0, new))[0] == 409  # older epoch
    # recreated within the same second: told apart by its uid
    same_sec = "2026-10-18T02:00:00Z uid-newer"
    assert a.check_leader("POST", "/v1/claims", tok("m-c", 0, same_sec)) is None
    a.stop()
    b = make_agent(tmp_path)  # the generation is persisted with the epoch
    assert b.leader_fence["leaseUID"] == "uid-newer"
    assert b.check_leader("POST", "/v1/claims", tok("m-b", 1, new))[0] == 409
    b.stop()


def test_a_fence_from_before_lease_generations_adopts_the_first_generation(tmp_path, native_built):
    """A fence persisted by an agent that predates the Lease-generation header has no generation
    to compare. The first token that carries one is adopted as the generation from then on —
    comparing its creationTimestamp (apiserver clock) with the fence's "at" (the agent's clock)
    refused a recreated Lease for good whenever the node clock ran ahead. From then on
    generations order tokens as usual."""
    a = make_agent(tmp_path)
    assert a.check_leader("POST", "/v1/claims", tok("m-a", 5)) is None  # no generation
    assert "leaseCreated" not in a.leader_fence
    # a Lease "created" before the fence's own timestamp (node clock ahead) is still adopted
    assert a.check_leader("POST", "/v1/claims", tok("m-x", 0, "2000-01-01T00:00:00Z uid-older")) \
        is None
    assert a.leader_fence["leaseUID"] == "uid-older" and a.leader_fence["epoch"] == 0
    assert a.check_leader("POST", "/v1/claims", tok("m-b", 0, "2999-01-01T00:00:00Z uid-new")) is None
    assert a.leader_fence["leaseUID"] == "uid-new" and a.leader_fence["epoch"] == 0
    # the Lease before it, whatever its epoch, is now the older generation
    assert a.check_leader("POST", "/v1/release", tok("m-a", 5, "2000-01-01T00:00:00Z uid-older"))[0] == 409
    a.stop()


def test_fence_unit_without_an_agent():
    """fence.LeaderFence on its own (narrow interface: persisted state, a persist callback)."""
    from gpupool.agent.fence import LeaderFence, StaleLeader
    saved = []
    f = LeaderFence({}, saved.append)
    f.admit("POST", "/v1/claims", tok("m-a", 1))
    assert saved[-1]["holder"] == "m-a" and f.epoch == 1
    f.admit("GET", "/v1/node", tok("m-z", 0))  # reads are never fenced
    f.admit("POST", "/v1/claims", {})          # no token: not checked
    with pytest.raises(StaleLeader) as ei:
        f.admit("POST", "/v1/release", tok("m-b", 0))
    assert ei.value.status == 409 and f.stats["stale_leader_refused"] == 1
    with pytest.raises(StaleLeader) as ei:
        f.admit("POST", "/v1/release", {"x-gpupool-leader-epoch": "x"})
    assert ei.value.status == 400

    def boom(_):
        raise OSError("disk full")
    g = LeaderFence({"holder": "m-a", "epoch": 1}, boom)
    with pytest.raises(OSError):
        g.admit("POST", "/v1/claims", tok("m-b", 2))
    assert g.epoch == 1  # not adopted unless durable
