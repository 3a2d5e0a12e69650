"""apiserver-sim over HTTP with the Python client and gpuctl: watch streams (from RV, bookmarks,
410 Gone), server-side printing, discovery, scale subresource, auth."""
from __future__ import annotations

import asyncio
import io
import os
import threading
import time
from contextlib import redirect_stdout

import pytest

from gpupool.apiserver_sim.server import ApiServerSim, load_crd_dir
from gpupool.cli import gpuctl
from gpupool.kube import MI355XPOOLS, PODS, Client, KubeError

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class SimThread:
    def __init__(self, **kw):
        self.sim = ApiServerSim(**kw)
        load_crd_dir(self.sim.store, os.path.join(ROOT, "config", "crd"))
        self.loop = asyncio.new_event_loop()
        self.ready = threading.Event()
        self.port = 0
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()
        assert self.ready.wait(10)

    def _run(self):
        from aiohttp import web
        asyncio.set_event_loop(self.loop)
        runner = web.AppRunner(self.sim.app)
        self.loop.run_until_complete(runner.setup())
        site = web.TCPSite(runner, "127.0.0.1", 0)
        self.loop.run_until_complete(site.start())
        self.port = site._server.sockets[0].getsockname()[1]
        self.ready.set()
        self.loop.run_forever()

    @property
    def url(self):
        return f"http://127.0.0.1:{self.port}"


@pytest.fixture(scope="module")
def sim():
    return SimThread(bookmark_interval=0.3, window=200)


def pool(name, r=1):
    return {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xPool",
            "metadata": {"name": name}, "spec": {"replicas": r}}


def test_crud_and_conflict(sim):
    c = Client(sim.url)
    a = c.create(MI355XPOOLS, pool("h1"), "default")
    a["spec"]["replicas"] = 2
    b = c.update(MI355XPOOLS, a, "default")
    assert b["metadata"]["generation"] == 2
    with pytest.raises(KubeError) as e:
        c.update(MI355XPOOLS, a, "default")  # stale RV
    assert e.value.code == 409
    with pytest.raises(KubeError) as e:
        c.create(MI355XPOOLS, pool("h1"), "default")
    assert e.value.code == 409 and e.value.reason == "AlreadyExists"
    with pytest.raises(KubeError) as e:
        c.get(MI355XPOOLS, "nope", "default")
    assert e.value.code == 404


def test_watch_from_rv_and_bookmarks(sim):
    c = Client(sim.url)
    a = c.create(MI355XPOOLS, pool("w1"), "default")
    rv = a["metadata"]["resourceVersion"]
    c.patch(MI355XPOOLS, "w1", {"spec": {"replicas": 3}}, "default")
    c.delete(MI355XPOOLS, "w1", "default")
    types = []
    saw_bookmark = False
    for ev in c.watch(MI355XPOOLS, "default", resource_version=rv, timeout_seconds=1):
        if ev["type"] == "BOOKMARK":
            saw_bookmark = True
            continue
        if ev["object"]["metadata"]["name"] == "w1":
            types.append(ev["type"])
    assert types == ["MODIFIED", "DELETED"]
    assert saw_bookmark


def test_watch_expired_rv_gets_410(sim):
    c = Client(sim.url)
    for i in range(250):
        c.create(PODS, {"metadata": {"name": f"gone{i}"}, "spec": {"containers": [{}]}}, "w410")
    evs = list(c.watch(PODS, "w410", resource_version="1", timeout_seconds=1))
    assert evs[0]["type"] == "ERROR" and evs[0]["object"]["code"] == 410


def test_initial_list_semantics(sim):
    c = Client(sim.url)
    c.create(MI355XPOOLS, pool("init1"), "initns")
    evs = []
    for ev in c.watch(MI355XPOOLS, "initns", timeout_seconds=1):
        evs.append(ev)
    assert evs[0]["type"] == "ADDED" and evs[0]["object"]["metadata"]["name"] == "init1"


def test_wait_for_is_watch_driven(sim):
    c = Client(sim.url)
    c.create(MI355XPOOLS, pool("wf"), "default")

    def later():
        time.sleep(0.2)
        Client(sim.url).patch(MI355XPOOLS, "wf", {"spec": {"replicas": 5}}, "default")
    threading.Thread(target=later).start()
    t0 = time.monotonic()
    o = c.wait_for(MI355XPOOLS, "wf", "default", lambda o: o["spec"]["replicas"] == 5, timeout=5)
    assert o["spec"]["replicas"] == 5 and time.monotonic() - t0 < 2


def test_table_and_gpuctl(sim, tmp_path):
    c = Client(sim.url)
    c.create(MI355XPOOLS, pool("tbl", 2), "default")
    tbl = c.table(MI355XPOOLS, "default")
    names = [cd["name"] for cd in tbl["columnDefinitions"]]
    assert names[:3] == ["Name", "Desired", "Ready"]  # README.md:132-133 printer columns
    out = io.StringIO()
    with redirect_stdout(out):
        assert gpuctl.main(["--server", sim.url, "get", "mxp"]) == 0
    assert "DESIRED" in out.getvalue() and "tbl" in out.getvalue()
    sample = os.path.join(ROOT, "config", "samples", "compute_v1alpha1_azurevmpool.yaml")
    out = io.StringIO()
    with redirect_stdout(out):
        assert gpuctl.main(["--server", sim.url, "apply", "-f", sample]) == 0
        assert gpuctl.main(["--server", sim.url, "apply", "-f", sample]) == 0
    assert "created" in out.getvalue() and "unchanged" in out.getvalue()
    out = io.StringIO()
    with redirect_stdout(out):
        assert gpuctl.main(["--server", sim.url, "scale", "azurevmpool", "gpu-pool-prod",
                            "--replicas", "3"]) == 0
        assert gpuctl.main(["--server", sim.url, "describe", "azurevmpool", "gpu-pool-prod"]) == 0
    assert "replicas: 3" in out.getvalue()
    assert gpuctl.main(["--server", sim.url, "wait", "azurevmpool", "gpu-pool-prod",
                        "--for", "jsonpath=.spec.replicas=3", "--timeout", "5"]) == 0


def test_discovery_and_dry_run(sim):
    c = Client(sim.url)
    groups = c.request("GET", "/apis")["groups"]
    assert any(g["name"] == "compute.my.domain" for g in groups)
    res = gpuctl.resolve(c, "avp")
    assert res.plural == "azurevmpools"
    out = c.create(MI355XPOOLS, pool("dry"), "default", dry_run=True)
    assert out["spec"]["resourceName"] == "amd.com/gpu"
    with pytest.raises(KubeError):
        c.get(MI355XPOOLS, "dry", "default")


def test_auth_token():
    s = SimThread(token="s3cret")
    with pytest.raises(KubeError) as e:
        Client(s.url).list(MI355XPOOLS, "default")
    assert e.value.code == 401
    assert Client(s.url, "s3cret").list(MI355XPOOLS, "default")["items"] == []


def test_render_job_template():
    tpl = {"title": "FashionMNIST CNN", "description": "demo", "image": "rocm/pytorch:latest",
           "command": "python examples/fmnist_train.py --epochs 1", "env": {"A": 1},
           "mode": "Single", "spec": {"singleInstanceType": "gpu-2x-16c-32g-2gpu"}}
    pod = gpuctl.render_job(tpl)
    lim = pod["spec"]["containers"][0]["resources"]["limits"]
    assert lim == {"amd.com/gpu": 2}
    assert pod["metadata"]["annotations"]["gpupool.amd.com/mode"] == "single"
