"""kubeconfig as the connection source (the reference's `make run` path uses the current
kubeconfig, README.md:263): the C++ manager (`--kubeconfig`, own YAML reader, in-memory PEM via
OpenSSL) and gpuctl/Client (`--kubeconfig`, PyYAML) against an HTTPS apiserver-sim, with bearer
token and with mutual TLS (client-certificate-data)."""
from __future__ import annotations

import base64
import os
import signal
import subprocess
import sys

import pytest
import yaml

from gpupool.kube import AZUREVMPOOLS, MI355XPOOLS, NAMESPACES, Client, load_kubeconfig
from gpupool.testing.cluster import ROOT, _wait_file, issue_client_cert, make_test_pki, native_bin

from .helpers import mi_pool, wait_ready


def _b64(path: str) -> str:
    return base64.b64encode(open(path, "rb").read()).decode()


def _kubeconfig(path: str, server: str, ca: str, token: str | None = None,
                cert: str | None = None, key: str | None = None, ns: str = "default") -> str:
    user: dict = {}
    if token:
        user["token"] = token
    if cert:
        user["client-certificate-data"] = _b64(cert)
        user["client-key-data"] = _b64(key)
    cfg = {"apiVersion": "v1", "kind": "Config", "current-context": "sim",
           "clusters": [{"name": "sim", "cluster": {"server": server,
                                                    "certificate-authority-data": _b64(ca)}}],
           "contexts": [{"name": "sim", "context": {"cluster": "sim", "user": "me",
                                                    "namespace": ns}}],
           "users": [{"name": "me", "user": user}]}
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f, sort_keys=False)
    return path


@pytest.fixture
def mtls_sim(tmp_path):
    """HTTPS apiserver-sim that requires a client certificate signed by its CA."""
    ca, crt, key = make_test_pki(str(tmp_path))
    ccrt, ckey = issue_client_cert(str(tmp_path))
    pf = tmp_path / "port"
    log = open(tmp_path / "sim.log", "wb")
    p = subprocess.Popen([sys.executable, "-m", "gpupool.apiserver_sim", "--port", "0", "--port-file",
                          str(pf), "--crd-dir", os.path.join(ROOT, "config", "crd"),
                          "--tls-cert", crt, "--tls-key", key, "--client-ca", ca],
                         cwd=ROOT, stdout=log, stderr=subprocess.STDOUT, start_new_session=True,
                         env=dict(os.environ, PYTHONPATH=ROOT))
    port = int(_wait_file(str(pf), 60, p, str(tmp_path / "sim.log")))
    yield {"url": f"https://127.0.0.1:{port}", "ca": ca, "cert": ccrt, "key": ckey}
    os.killpg(p.pid, signal.SIGTERM)
    p.wait(timeout=10)


def test_manager_and_gpuctl_via_kubeconfig_token(cluster_factory, tmp_path):
    c = cluster_factory(tls=True, token="kc-token", manager=False)
    kc = _kubeconfig(str(tmp_path / "config"), c.url, c.ca_file, token="kc-token", ns="team-a")
    # the manager gets NOTHING but the kubeconfig (no --apiserver / --token / --ca-file)
    mlog = open(tmp_path / "mgr.log", "wb")
    env = {k: v for k, v in os.environ.items() if k not in ("GPUPOOL_APISERVER", "GPUPOOL_TOKEN")}
    env["GPUPOOL_AGENT_TOKEN"] = c.agent_token  # the agents' RPC secret (a mounted Secret in-cluster)
    m = subprocess.Popen([native_bin("gpupool-manager"), "--kubeconfig", kc, "--kinds", "mi355x",
                          "--progress-poll", "100ms"], stdout=mlog, stderr=subprocess.STDOUT,
                         start_new_session=True, env=env)
    try:
        k = c.client
        k.create(NAMESPACES, {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team-a"}})
        k.create(MI355XPOOLS, mi_pool("kc", 1), "team-a")
        wait_ready(k, "kc", 1, ns="team-a", timeout=30)
        assert "using kubeconfig" in open(tmp_path / "mgr.log").read()
        # gpuctl: namespace comes from the kubeconfig context
        genv = dict(env, PYTHONPATH=ROOT)
        genv.pop("GPUPOOL_CA_FILE", None)
        r = subprocess.run([sys.executable, "-m", "gpupool.cli", "--kubeconfig", kc, "get", "mxp"],
                           cwd=ROOT, env=genv, capture_output=True, text=True, timeout=60)
        assert r.returncode == 0 and "kc" in r.stdout, r.stdout + r.stderr
    finally:
        os.killpg(m.pid, signal.SIGTERM)
        m.wait(timeout=10)


def test_mutual_tls_kubeconfig(mtls_sim, tmp_path):
    s = mtls_sim
    kc = _kubeconfig(str(tmp_path / "config"), s["url"], s["ca"], cert=s["cert"], key=s["key"])
    resolved = load_kubeconfig(kc)
    assert resolved["cert_data"].startswith("-----BEGIN CERTIFICATE")
    c = Client.from_kubeconfig(kc)
    pool = {"apiVersion": "compute.my.domain/v1alpha1", "kind": "AzureVmPool",
            "metadata": {"name": "zero"},
            "spec": {"replicas": 0, "resourceGroupName": "rg", "location": "eastus",
                     "vmSize": "Standard_NC4as_T4_v3", "vnetName": "v", "subnetName": "s",
                     "azureCredentialSecret": "azure-credentials",
                     "imageReference": {"publisher": "p", "offer": "o", "sku": "s", "version": "v"}}}
    c.create(AZUREVMPOOLS, pool, "default")
    # without a client certificate the TLS handshake is refused
    import ssl
    with pytest.raises((ssl.SSLError, ConnectionError, OSError)):
        Client(s["url"], ca_file=s["ca"]).get(AZUREVMPOOLS, "zero", "default")
    # the C++ manager authenticates with client-certificate-data / client-key-data from memory
    mlog = tmp_path / "mgr.log"
    env = {k: v for k, v in os.environ.items() if k not in ("GPUPOOL_APISERVER", "GPUPOOL_TOKEN")}
    env["KUBECONFIG"] = kc  # env form of --kubeconfig
    with open(mlog, "wb") as lf:
        m = subprocess.Popen([native_bin("gpupool-manager"), "--kinds", "azure"], stdout=lf,
                             stderr=subprocess.STDOUT, start_new_session=True, env=env)
    try:
        o = c.wait_for(AZUREVMPOOLS, "zero", "default",
                       lambda o: any(x["type"] == "Ready" for x in
                                     ((o or {}).get("status") or {}).get("conditions", [])),
                       timeout=30)
        assert o["status"]["readyReplicas"] == 0
    finally:
        os.killpg(m.pid, signal.SIGTERM)
        m.wait(timeout=10)
    assert "TLS handshake" not in mlog.read_text()


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.slow
def test_agent_rpc_over_tls(cluster_factory, tmp_path):
    """Across nodes the agent RPC (claims, cordon, release, the event feed) and its bearer token
    travel over HTTPS: the agent serves --listen with --tls-cert, the Node annotation says
    https://, and the manager verifies the certificate with --agent-ca-file. A manager without
    that CA cannot talk to the agent (the pool reports it instead of claiming)."""
    from gpupool.testing.cluster import NodeSpec
    ca, crt, key = make_test_pki(str(tmp_path), "agent")
    port = _free_port()
    node = NodeSpec("tls-node", extra_args=["--listen", f"127.0.0.1:{port}", "--tls-cert", crt,
                                            "--tls-key", key,
                                            "--endpoint", f"https://127.0.0.1:{port}"])
    c = cluster_factory(nodes=[node], manager_args=["--agent-ca-file", ca])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    o = wait_ready(k, "p", 2)
    assert o["status"]["nodeName"] == "tls-node"
    # plain HTTP to the TLS listener is refused at the transport
    import urllib.error
    import urllib.request
    with pytest.raises((urllib.error.URLError, ConnectionError, OSError)):
        urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=3).read()


@pytest.mark.slow
def test_manager_without_agent_ca_cannot_reach_tls_agent(cluster_factory, tmp_path):
    from gpupool.testing.cluster import NodeSpec
    _ca, crt, key = make_test_pki(str(tmp_path), "agent")
    port = _free_port()
    node = NodeSpec("tls-node", extra_args=["--listen", f"127.0.0.1:{port}", "--tls-cert", crt,
                                            "--tls-key", key,
                                            "--endpoint", f"https://127.0.0.1:{port}"])
    c = cluster_factory(nodes=[node])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("p", 1, nodeName="tls-node"), "default")
    o = k.wait_for(MI355XPOOLS, "p", "default",
                   lambda x: bool(x) and any(cd["type"] == "Degraded" and cd["status"] == "True"
                                             for cd in (x.get("status") or {}).get("conditions", [])),
                   timeout=30)
    assert o["status"].get("readyReplicas", 0) == 0
