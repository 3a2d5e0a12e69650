"""The agent DaemonSet against what the agent's Allocate hands the container runtime.

A device plugin's Allocate answers with HOST paths (mounts, device nodes) that the container
runtime resolves on the node, not inside the agent's container. So every path the agent can return
must exist on the host at the path the agent sees: it must lie under a same-path hostPath volume of
config/agent/agent-daemonset.yaml (hostPath.path == mountPath). And the agent itself opens
/dev/kfd and /dev/dri (amdsmi, HIP probe), which a non-privileged container's device cgroup denies
— a hostPath mount alone does not grant it. The fake kubelet cannot see either defect without its
strict-mounts mode (gpupool/kubelet_fake/kubelet.py ``host_paths``), which this file also pins.
"""
from __future__ import annotations

import os

import yaml

from gpupool.agent.agent import SLOT_SEP, Agent, AgentConfig

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "node_8x_mi355x.json")
DAEMONSET = os.path.join(ROOT, "config", "agent", "agent-daemonset.yaml")


def _daemonset() -> tuple[dict, dict]:
    ds = yaml.safe_load(open(DAEMONSET))
    pod = ds["spec"]["template"]["spec"]
    agent = next(c for c in pod["containers"] if c["name"] == "agent")
    return pod, agent


def _same_path_roots(pod: dict, agent: dict) -> list[str]:
    host = {v["name"]: v["hostPath"]["path"] for v in pod["volumes"] if "hostPath" in v}
    return [m["mountPath"] for m in agent["volumeMounts"]
            if m["name"] in host and host[m["name"]].rstrip("/") == m["mountPath"].rstrip("/")]


def _under(path: str, roots: list[str]) -> bool:
    p = os.path.normpath(path)
    return any(p == r.rstrip("/") or p.startswith(r.rstrip("/") + "/") for r in roots)


def _arg(agent: dict, flag: str) -> str:
    args = agent.get("args") or []
    return args[args.index(flag) + 1]


def test_agent_container_can_open_the_gpu_device_nodes():
    pod, agent = _daemonset()
    assert (agent.get("securityContext") or {}).get("privileged") is True, \
        "the agent opens /dev/kfd and /dev/dri itself: without privileged its device cgroup denies it"
    roots = _same_path_roots(pod, agent)
    for dev in ("/dev/kfd", "/dev/dri/renderD128"):
        assert _under(dev, roots), (dev, roots)


def test_every_allocate_host_path_is_a_same_path_host_volume(tmp_path, native_built):
    """Claim an isolated shared GPU on a fake agent, Allocate a slot, and map the agent's state dir
    onto the DaemonSet's --state-dir: every returned mount and device host path must lie under a
    same-path hostPath volume. (Mounting the library from the agent's own tree — its image path —
    fails here: the runtime would not find it on the host.)"""
    pod, agent_c = _daemonset()
    roots = _same_path_roots(pod, agent_c)
    state_deployed = _arg(agent_c, "--state-dir")
    state = str(tmp_path / "state")
    cfg = AgentConfig(node="n0", backend="fake", fixture=FIXTURE, state_dir=state,
                      probe_mode="simulated", probe_sim_ms=1, fsync=False)
    a = Agent(cfg)
    try:
        policy = {"sharing": {"replicasPerGPU": 4, "hbmBytesPerSlot": 8 << 30, "cuPerSlot": 64}}
        r = a.claim({"poolUID": "p1", "pool": "default/p", "count": 1, "resourceName": "amd.com/gpu",
                     "policy": policy, "topologyPolicy": "xgmi-packed", "probe": {"enabled": True}})
        assert r["ok"], r
        uuid = r["devices"][0]["uuid"]
        spec = a.allocate_spec("amd.com/gpu", [f"{uuid}{SLOT_SEP}1"])
        assert spec["envs"]["HSA_TOOLS_LIB"].endswith("libgpupool_share.so")
        paths = [m["host_path"] for m in spec["mounts"]] + list(spec["devices"])
        paths += a.share_mounts()
        assert any(p.endswith("/lib") for p in paths) and any(p.endswith(".acct") for p in paths)

        def deployed(p: str) -> str:  # the agent's state dir is --state-dir on the node
            return state_deployed + p[len(state):] if p.startswith(state) else p
        off = [p for p in map(deployed, paths) if not _under(p, roots)]
        assert not off, f"Allocate host paths outside the DaemonSet's same-path hostPaths: {off}"
        # the library really is at the mounted host path
        lib_dir = next(m["host_path"] for m in spec["mounts"] if m["host_path"].endswith("/lib"))
        assert os.path.exists(os.path.join(lib_dir, "libgpupool_share.so"))
    finally:
        a.stop()


def test_fake_kubelet_strict_mounts_reject_off_node_paths():
    """The strict-mounts check itself: a mount or device outside the declared host paths is
    reported; inside (including the roots themselves) is not."""
    from types import SimpleNamespace as NS

    from gpupool.kubelet_fake.kubelet import FakeKubelet
    k = FakeKubelet.__new__(FakeKubelet)
    k.host_paths = ["/var/lib/gpupool", "/dev/kfd", "/dev/dri"]
    ok = NS(mounts=[NS(host_path="/var/lib/gpupool/lib"), NS(host_path="/var/lib/gpupool/share/x.acct")],
            devices=[NS(host_path="/dev/kfd"), NS(host_path="/dev/dri/renderD128")])
    assert k._off_node_paths(ok) == []
    bad = NS(mounts=[NS(host_path="/opt/gpupool/build/native")],
             devices=[NS(host_path="/dev/kfd2")])
    assert k._off_node_paths(bad) == ["/opt/gpupool/build/native", "/dev/kfd2"]
    k.host_paths = None
    assert k._off_node_paths(bad) == []
