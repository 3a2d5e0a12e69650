"""TLS + bearer-token transport between every component and the apiserver (the
manager runs in-cluster against https://kubernetes.default.svc with the ServiceAccount token and
CA). The simulator serves HTTPS with a throw-away CA; the C++ manager (OpenSSL), the Python
agent/kubelet/client (stdlib ssl) must verify it, and a manager holding the wrong CA must refuse."""
from __future__ import annotations

import os
import subprocess
import time

import pytest

from gpupool.kube import MI355XPOOLS, KubeError, Client
from gpupool.testing.cluster import make_test_pki, native_bin

from .helpers import mi_pool, wait_ready


def test_pool_ready_over_tls_with_token(cluster_factory):
    c = cluster_factory(tls=True, token="s3cret-token")
    assert c.url.startswith("https://")
    k = c.client
    k.create(MI355XPOOLS, mi_pool("tls", 2), "default")
    o = wait_ready(k, "tls", 2, timeout=30)
    assert o["status"]["readyReplicas"] == 2
    # the apiserver enforces the token: an anonymous TLS client is rejected
    anon = Client(c.url, None, ca_file=c.ca_file)
    with pytest.raises(KubeError) as ei:
        anon.get(MI355XPOOLS, "tls", "default")
    assert ei.value.code == 401
    # a client that does not trust the CA fails the handshake
    import ssl
    stranger = Client(c.url, "s3cret-token", ca_file=make_test_pki(str(c.workdir) + "/other")[0])
    with pytest.raises(ssl.SSLError):
        stranger.get(MI355XPOOLS, "tls", "default")


def test_manager_rejects_untrusted_ca(cluster_factory, tmp_path):
    c = cluster_factory(tls=True, token="t0k", manager=False)
    wrong_ca = make_test_pki(str(tmp_path / "wrong"))[0]
    log = tmp_path / "mgr.log"
    with open(log, "wb") as lf:
        p = subprocess.Popen([native_bin("gpupool-manager"), "--apiserver", c.url, "--ca-file", wrong_ca,
                              "--token", "t0k", "--kinds", "mi355x", "--metrics-addr", "127.0.0.1:0"],
                             stdout=lf, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        deadline = time.monotonic() + 15
        while time.monotonic() < deadline and "TLS handshake" not in log.read_text():
            time.sleep(0.1)
        text = log.read_text()
        assert "TLS handshake" in text and "certificate" in text, text[-2000:]
    finally:
        os.killpg(p.pid, 15)
        p.wait(timeout=10)
