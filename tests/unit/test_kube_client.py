"""Python client connection config: in-cluster ServiceAccount discovery and TLS context wiring."""
from __future__ import annotations

import ssl

import pytest

from gpupool.kube import Client
from gpupool.testing.cluster import make_test_pki


def test_in_cluster_config(tmp_path, monkeypatch):
    ca, _, _ = make_test_pki(str(tmp_path))
    sa = tmp_path / "sa"
    sa.mkdir()
    (sa / "token").write_text("tok-123\n")
    (sa / "ca.crt").write_text(open(ca).read())
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST", raising=False)
    assert Client.in_cluster(str(sa)) is None
    monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "10.96.0.1")
    monkeypatch.setenv("KUBERNETES_SERVICE_PORT", "6443")
    c = Client.in_cluster(str(sa))
    assert c.server == "https://10.96.0.1:6443" and c.token == "tok-123"
    assert c.host == "10.96.0.1" and c.port == 6443
    assert isinstance(c._ssl, ssl.SSLContext) and c._ssl.verify_mode == ssl.CERT_REQUIRED
    monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "fd00::1")
    assert Client.in_cluster(str(sa)).server == "https://[fd00::1]:6443"


def test_connect_in_cluster_requires_serviceaccount(monkeypatch):
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST", raising=False)
    with pytest.raises(RuntimeError):
        Client.connect("in-cluster")
    assert Client.connect("http://127.0.0.1:1").scheme == "http"


def test_insecure_disables_verification():
    c = Client("https://127.0.0.1:1", insecure=True)
    assert c._ssl.verify_mode == ssl.CERT_NONE and not c._ssl.check_hostname
