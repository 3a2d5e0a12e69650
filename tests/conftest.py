"""Shared pytest setup.

Markers:
  gpu   — needs a real MI355X (run by the driver on the GPU box with ``-m gpu``);
  slow  — multi-second integration/property runs (still part of the default CPU suite).
The native artefacts (build/native) are built once per session with ``make -C native``.
"""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires a real MI355X GPU (gfx950)")
    config.addinivalue_line("markers", "slow: multi-second integration test")


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_makereport(item, call):
    outcome = yield
    rep = outcome.get_result()
    setattr(item, "rep_" + rep.when, rep)


def make_native(target: str, san: str = "", timeout: float | None = None):
    """``make -C native`` under an exclusive file lock: pytest-xdist workers share one build tree,
    and a worker relinking a binary another worker is executing fails that exec (ETXTBSY/EACCES)."""
    import fcntl
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    argv = ["make", "-C", os.path.join(ROOT, "native")] + ([f"SAN={san}"] if san else []) + \
        [target, "-j8"]
    with open(os.path.join(ROOT, "build", ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        return subprocess.run(argv, capture_output=True, text=True, timeout=timeout)


@pytest.fixture(scope="session")
def native_built():
    """Build the native targets (host-only unless hipcc is present) once per session."""
    target = "all" if os.path.exists("/opt/rocm/bin/hipcc") else "host"
    r = make_native(target)
    if r.returncode != 0:
        pytest.fail("native build failed:\n" + r.stdout[-4000:] + r.stderr[-4000:])
    return os.path.join(ROOT, "build", "native")


@pytest.fixture
def cluster_factory(request, tmp_path, native_built):
    """Start local control planes; all are stopped at test teardown. A failed test's cluster logs
    are copied to ``$GPUPOOL_FAILED_LOGS`` (default /tmp/gpupool-failed/<test>): pytest rotates its
    tmp dirs away after three sessions, and a rare flake is only diagnosable from its own logs."""
    from gpupool.testing.cluster import Cluster
    made = []

    def make(**kw):
        c = Cluster(str(tmp_path / f"cluster{len(made)}"), **kw)
        made.append(c)
        c.start()
        return c
    yield make
    rep = getattr(request.node, "rep_call", None)
    if made and rep is not None and rep.failed:
        _keep_cluster_logs(request.node.nodeid, made)
    for c in made:
        c.stop()


def _keep_cluster_logs(nodeid: str, clusters: list) -> None:
    """Copy the control planes' logs and the pods' logs (under the kubelets' socket dirs, which
    ``Cluster.stop`` removes) before the clusters are stopped."""
    import re
    import shutil
    dest = os.path.join(os.environ.get("GPUPOOL_FAILED_LOGS", "/tmp/gpupool-failed"),
                        re.sub(r"[^A-Za-z0-9_.-]+", "_", nodeid))

    def only_logs(d, names):
        return [n for n in names if not n.endswith((".log", ".json"))
                and not os.path.isdir(os.path.join(d, n))]
    for i, c in enumerate(clusters):
        try:
            shutil.copytree(c.workdir, os.path.join(dest, f"cluster{i}"), dirs_exist_ok=True,
                            ignore=only_logs)
            for node in c.nodes:
                pods = os.path.join(c.kubelet_root(node), "pod-logs")
                if os.path.isdir(pods):
                    shutil.copytree(pods, os.path.join(dest, f"cluster{i}", f"pod-logs-{node.name}"),
                                    dirs_exist_ok=True)
        except OSError as e:
            sys.stderr.write(f"\nkeeping cluster logs failed: {e}\n")
    sys.stderr.write(f"\ncluster logs of the failed test kept in {dest}\n")
