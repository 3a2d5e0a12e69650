"""Agent endpoints are bound to their node and no reusable credential travels (round-5 weak #2).

A rogue listener stands in for a compromised node that rewrote node B's agent-endpoint
annotation (the admin write here stands in for what the agent's ValidatingAdmissionPolicy now
refuses an agent identity, tests/unit/test_nodereg.py):

* with pod discovery (the deployed configuration) the manager keeps calling node B's agent at
  its Pod's IP: the rogue gets no connection at all, B's pool keeps its GPUs and stays Ready, and
  the ignored annotation is counted;
* with annotation discovery (local setups) the rogue does get requests — carrying no
  Authorization header, only per-request signatures for node B that node A's agent refuses and
  node B's agent accepts once.
"""
from __future__ import annotations

import http.server
import json
import os
import socketserver
import threading
import time

import pytest

from gpupool.kube import MI355XPOOLS, NODES, Client, KubeError
from gpupool.testing.cluster import NodeSpec, _free_port
from tests.integration.helpers import mi_pool, wait_ready

pytestmark = pytest.mark.slow


class Rogue:
    """Records every request (method, path, headers) and answers with a fabricated node view."""

    def __init__(self, host: str, node: str):
        self.seen: list[tuple[str, str, dict]] = []
        rogue = self
        fake = {"node": node, "backend": "fake", "gen": 999, "advertiseRequired": False,
                "devices": [{"uuid": f"ROGUE-{i}", "index": i, "node": node, "healthy": True,
                             "state": "Free"} for i in range(8)], "freeHealthy": 8}

        class H(http.server.BaseHTTPRequestHandler):
            def _any(self):
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n) if n else b""
                rogue.seen.append((self.command, self.path, dict(self.headers), body))
                out = json.dumps(fake if self.path.startswith("/v1/node") else
                                 {"ok": True, "devices": fake["devices"][:1], "gen": 999}).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(out)))
                self.end_headers()
                self.wfile.write(out)

            do_GET = do_POST = _any

            def log_message(self, *a):
                pass

        self.port = _free_port()
        self.srv = socketserver.ThreadingTCPServer((host, self.port), H)
        self.srv.daemon_threads = True
        self.url = f"http://{host}:{self.port}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def close(self):
        self.srv.shutdown()
        self.srv.server_close()


def _nodes():
    return [NodeSpec("node-a", count=4), NodeSpec("node-b", count=4)]


def test_pod_discovery_ignores_a_redirected_annotation(cluster_factory):
    c = cluster_factory(nodes=_nodes(), agent_auth="signature", discovery="pod")
    k = c.client
    k.create(MI355XPOOLS, mi_pool("pb", 2, nodeSelector={"kubernetes.io/hostname": "node-b"}),
             "default")
    before = wait_ready(k, "pb", 2, timeout=60)
    real = {d["uuid"] for d in before["status"]["devices"]}
    rogue = Rogue("127.0.0.99", "node-b")
    try:
        k.patch(NODES, "node-b", {"metadata": {"annotations": {
            "gpupool.amd.com/agent-endpoint": rogue.url}}})
        # a surge rollout's second agent pod on node B, newer but not Ready yet, at another
        # address: the manager stays with the Ready one (else B's claims would fail to connect)
        c.publish_agent_pod("node-b", ip="127.0.0.99", ready=False, name="gpupool-agent-4x7kq")  # sorts first
        # make the manager talk to node B's agent: scale up and down, then a resync
        k.patch(MI355XPOOLS, "pb", {"spec": {"replicas": 3}}, "default")
        wait_ready(k, "pb", 3, timeout=60)
        k.patch(MI355XPOOLS, "pb", {"spec": {"replicas": 2}}, "default")
        o = wait_ready(k, "pb", 2, timeout=60)
        time.sleep(2)
        assert rogue.seen == []
        uuids = {d["uuid"] for d in o["status"]["devices"]}
        assert not any(u.startswith("ROGUE") for u in uuids)
        assert all(d["node"] == "node-b" for d in o["status"]["devices"])
        agent_view = c.agent_request("node-b", "GET", "/v1/node")
        mine = {d["uuid"] for d in agent_view["devices"]
                if d.get("poolUID") == o["metadata"]["uid"]}
        assert mine == uuids and real & uuids
        m = c.manager_metrics()
        assert 'gpupool_agent_endpoint_rejected_total{node="node-b"}' in m
        # the agents saw only signed requests for themselves
        am = c.agent_request("node-b", "GET", "/metrics")
        assert 'gpupool_agent_rpc_auth_total{result="signature"}' in am
        # once the agent's key-exchange key is on its Node, the manager MACs per node (v2)
        assert 'gpupool_agent_rpc_signature_versions_total{version="v2"}' in am
    finally:
        rogue.close()


def test_annotation_mode_rogue_gets_no_reusable_credential(cluster_factory):
    c = cluster_factory(nodes=_nodes(), agent_auth="signature")
    k = c.client
    k.create(MI355XPOOLS, mi_pool("pb", 1, nodeSelector={"kubernetes.io/hostname": "node-b"}),
             "default")
    wait_ready(k, "pb", 1, timeout=60)
    rogue = Rogue("127.0.0.1", "node-b")
    try:
        k.patch(NODES, "node-b", {"metadata": {"annotations": {
            "gpupool.amd.com/agent-endpoint": rogue.url}}})
        deadline = time.monotonic() + 30
        while not rogue.seen and time.monotonic() < deadline:
            k.patch(MI355XPOOLS, "pb", {"metadata": {"labels": {"poke": str(time.time_ns())}}},
                    "default")
            time.sleep(0.5)
        assert rogue.seen, "the manager never called the annotated endpoint"
        for method, path, headers, body in rogue.seen:
            low = {h.lower(): v for h, v in headers.items()}
            assert "authorization" not in low, headers
            assert "node=node-b " in low["x-gpupool-signature"]
        # what the rogue holds is refused by every other agent
        method, path, headers, body = rogue.seen[-1]
        sig = {h.lower(): v for h, v in headers.items()}["x-gpupool-signature"]
        a = Client("unix://" + c.agent_socket("node-a"))
        with pytest.raises(KubeError) as ei:
            a.request(method, path, json.loads(body) if body else None,
                      extra_headers={"X-Gpupool-Signature": sig})
        assert ei.value.code == 401 and ei.value.reason == "WrongNode"
    finally:
        rogue.close()


def test_a_stale_key_exchange_key_falls_back_to_signatures(cluster_factory):
    """The Node names another X25519 key than the agent holds (its state dir was wiped, or an
    admin edit): the agent refuses the MAC before reading the body (StaleAgentKey), the manager
    re-sends that request signed with Ed25519 and keeps doing so for that key — no reconcile
    fails."""
    from gpupool.utils import edsig
    c = cluster_factory(nodes=[NodeSpec("node-k", count=4)], agent_auth="signature")
    k = c.client
    k.create(MI355XPOOLS, mi_pool("pk", 1), "default")
    wait_ready(k, "pk", 1, timeout=60)
    other = edsig.x25519_public(os.urandom(32))
    k.patch(NODES, "node-k", {"metadata": {"annotations": {
        "gpupool.amd.com/agent-kx": edsig._b64u(other)}}})
    time.sleep(0.5)
    for n in (3, 1, 2):
        k.patch(MI355XPOOLS, "pk", {"spec": {"replicas": n}}, "default")
        wait_ready(k, "pk", n, timeout=60)
    am = c.agent_request("node-k", "GET", "/metrics")
    assert 'gpupool_agent_rpc_auth_total{result="rejected_StaleAgentKey"} 1' in am, \
        [ln for ln in am.splitlines() if "rpc_auth" in ln]
    assert 'gpupool_agent_rpc_signature_versions_total{version="v1"}' in am
    mm = c.manager_metrics()
    assert 'gpupool_agent_kx_refused_total{node="node-k"} 1' in mm
    assert 'gpupool_reconcile_total{kind="Mi355xPool",result="error"}' not in mm
