"""The manager's agent-RPC signing key rotated with ``gpuctl keys`` under a running pool, no RPC
refused on the way (gpupool/cli/keys.py). The kubelet's volume sync — Secret and ConfigMap into
the mounted files the manager and the agents re-read — is done by ``_sync`` here."""
from __future__ import annotations

import base64
import time

import pytest

from gpupool.cli import gpuctl, keys
from gpupool.kube import CONFIGMAPS, MI355XPOOLS, SECRETS, Client
from gpupool.testing.cluster import NodeSpec
from gpupool.utils import edsig

from .helpers import mi_pool, wait_ready
from .rotation import _metric, _write

pytestmark = pytest.mark.slow
NS = "gpupool-system"


def _sync(c, k: Client) -> None:
    """What the kubelet does for the mounted Secret and ConfigMap."""
    sec = k.get(SECRETS, keys.SECRET, NS)
    _write(c.signing_key, base64.b64decode(sec["data"]["key"]).decode().strip())
    cm = k.get(CONFIGMAPS, keys.CONFIGMAP, NS)
    _write(c.pubkeys, "".join(cm["data"][f] for f in sorted(cm["data"])).strip())


def _wait(pred, timeout=20.0):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(0.2)
    return pred()


def test_rotation_in_three_steps_without_a_refused_rpc(cluster_factory, capsys):
    c = cluster_factory(nodes=[NodeSpec("ka", count=4), NodeSpec("kb", count=4)],
                        agent_auth="signature")
    k = c.client

    def scale(sizes):  # one pool per node: RPCs to both agents
        for name, n in sizes.items():
            k.patch(MI355XPOOLS, name, {"spec": {"replicas": n}}, "default")
        for name, n in sizes.items():
            wait_ready(k, name, n, timeout=60)
    for name, node in (("kp", "ka"), ("kq", "kb")):
        k.create(MI355XPOOLS, mi_pool(name, 1, nodeSelector={"kubernetes.io/hostname": node}),
                 "default")
    scale({"kp": 2, "kq": 1})
    # what `kubectl create secret/configmap --from-file` made at install time
    priv = open(c.signing_key).read()
    kid0 = edsig.key_id(edsig.public_from_private(edsig.load_private_key(priv)))
    k.create(SECRETS, {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": keys.SECRET},
                       "data": {"key": base64.b64encode(priv.encode()).decode()}}, NS)
    k.create(CONFIGMAPS, {"apiVersion": "v1", "kind": "ConfigMap",
                          "metadata": {"name": keys.CONFIGMAP},
                          "data": {f"{kid0}.pem": open(c.pubkeys).read()}}, NS)
    base = ["--server", c.url]
    assert keys.status(k, NS)["signing"] == kid0

    # 1. publish a new key
    assert gpuctl.main(base + ["keys", "rotate"]) == 0
    kid1 = keys.status(k, NS)["next"]
    assert kid1 and kid1 != kid0
    # out of order: the agents do not trust it until the kubelet synced the ConfigMap
    assert gpuctl.main(base + ["keys", "rotate"]) == 1
    assert "not trusted yet" in capsys.readouterr().err
    _sync(c, k)
    assert _wait(lambda: all(kid1 in a.get("trusted", []) for a in keys.agents(k).values()))

    # 2. the manager signs with it
    assert gpuctl.main(base + ["keys", "rotate"]) == 0
    assert keys.status(k, NS)["signing"] == kid1 and keys.status(k, NS)["next"] is None
    _sync(c, k)
    time.sleep(6.0)  # the manager re-checks its key file every 5 s
    scale({"kp": 4, "kq": 3})
    assert _wait(lambda: all(a["used"].get(kid1) for a in keys.agents(k).values()))

    # 3. drop the old key
    assert gpuctl.main(base + ["keys", "prune"]) == 0
    assert keys.status(k, NS)["published"] == [kid1]
    _sync(c, k)
    assert _wait(lambda: all(a.get("trusted") == [kid1] for a in keys.agents(k).values()))
    scale({"kp": 1, "kq": 2})

    # no agent refused a signed request, no reconcile failed
    for node in ("ka", "kb"):
        m = c.agent_request(node, "GET", "/metrics")
        assert _metric(m, "gpupool_agent_rpc_auth_total", 'result="rejected_') == 0, \
            [ln for ln in m.splitlines() if "rpc_auth" in ln or "signatures" in ln]
    mm = c.manager_metrics()
    assert _metric(mm, "gpupool_reconcile_total", 'result="error"') == 0
    capsys.readouterr()
    assert gpuctl.main(base + ["keys", "status"]) == 0
    out = capsys.readouterr().out
    assert f"signing:   {kid1}" in out and "ka: trusts" in out


def test_init_creates_a_key_pair_once(cluster_factory, capsys):
    c = cluster_factory(nodes=[NodeSpec("ki", count=1)], manager=False)
    base = ["--server", c.url]
    assert gpuctl.main(base + ["keys", "init", "--key-namespace", "keys-test"]) == 0
    st = keys.status(c.client, "keys-test")
    assert st["signing"] and st["published"] == [st["signing"]] and st["next"] is None
    sec = c.client.get(SECRETS, keys.SECRET, "keys-test")
    pem = base64.b64decode(sec["data"]["key"]).decode()
    assert pem.startswith("-----BEGIN PRIVATE KEY-----")
    assert gpuctl.main(base + ["keys", "init", "--key-namespace", "keys-test"]) == 1
    assert "rotate it instead" in capsys.readouterr().err
    assert gpuctl.main(base + ["keys", "prune", "--key-namespace", "keys-test"]) == 0
