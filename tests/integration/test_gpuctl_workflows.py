"""The reference's kubectl workflows through gpuctl against a running control plane: the GPU smoke
test pod (``kubectl run --rm -it --gpus=1 gpu-test ... nvidia-smi``, GPU调度平台搭建.md:134-138),
the Azure credentials Secret (``kubectl create secret generic azure-credentials``,
README.md:244-252), ``kubectl create namespace`` (GPU调度平台搭建.md:228) and ``kubectl logs``
through the pods/log subresource (GPU调度平台搭建.md:682)."""
from __future__ import annotations

import base64
import io
import threading

import pytest

from gpupool.cli import gpuctl
from gpupool.kube import MI355XPOOLS, NAMESPACES, PODS, SECRETS, Client
from gpupool.testing.cluster import NodeSpec

from .helpers import mi_pool, wait_ready

pytestmark = pytest.mark.slow


def test_run_rm_is_the_gpu_smoke_test(cluster_factory, capsys):
    c = cluster_factory(nodes=[NodeSpec("n1", count=2)])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("p", 1), "default")
    wait_ready(k, "p", 1, timeout=60)
    base = ["--server", c.url, "-n", "default"]
    rc = gpuctl.main(base + ["run", "--rm", "-it", "--gpus", "1", "gpu-test", "--image",
                             "rocm/dev-ubuntu-22.04", "--", "sh", "-c",
                             "echo visible=$ROCR_VISIBLE_DEVICES; echo done; exit 3"])
    out = capsys.readouterr()
    assert rc == 3, out
    assert "visible=" in out.out and "done" in out.out
    assert k.wait_for(PODS, "gpu-test", "default", lambda o: o is None, timeout=30) is None
    # without --rm the pod stays; logs come through pods/log (tail, follow to the end)
    assert gpuctl.main(base + ["run", "lines", "--image", "x", "--gpus", "1", "--", "sh", "-c",
                               "for i in 1 2 3 4; do echo line$i; sleep 0.2; done"]) == 0
    k.wait_for(PODS, "lines", "default",
               lambda o: o and o["status"].get("phase") in ("Running", "Succeeded"), 30)
    buf = io.StringIO()
    t = threading.Thread(target=lambda: gpuctl.pod_log(Client(c.url), "default", "lines",
                                                       follow=True, out=buf), daemon=True)
    t.start()
    t.join(30)
    assert not t.is_alive(), "follow did not end with the pod"
    assert buf.getvalue().split() == ["line1", "line2", "line3", "line4"]
    capsys.readouterr()
    assert gpuctl.main(base + ["logs", "lines", "--tail", "2"]) == 0
    assert capsys.readouterr().out.split() == ["line3", "line4"]


def test_create_secret_and_namespace(cluster_factory, tmp_path, capsys):
    c = cluster_factory(nodes=[NodeSpec("n1", count=1)], manager=False)
    base = ["--server", c.url, "-n", "default"]
    key = tmp_path / "client.pem"
    key.write_bytes(b"\x00pem-bytes\xff")
    assert gpuctl.main(base + ["create", "secret", "generic", "azure-credentials",
                               "--from-literal=AZURE_CLIENT_ID=abc",
                               "--from-literal=AZURE_CLIENT_SECRET=s3cr=t",
                               f"--from-file=cert={key}"]) == 0
    s = c.client.get(SECRETS, "azure-credentials", "default")
    dec = {k: base64.b64decode(v) for k, v in s["data"].items()}
    assert dec == {"AZURE_CLIENT_ID": b"abc", "AZURE_CLIENT_SECRET": b"s3cr=t",
                   "cert": b"\x00pem-bytes\xff"}
    assert gpuctl.main(base + ["create", "namespace", "rook-ceph"]) == 0
    assert c.client.get(NAMESPACES, "rook-ceph")["metadata"]["name"] == "rook-ceph"
    assert "secret/azure-credentials created" in capsys.readouterr().out
    assert gpuctl.main(base + ["create", "secret", "generic", "a", "b"]) == 1
