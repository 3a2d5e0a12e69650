"""Per-hop RPC latency after an idle gap (no GPU work): agent /healthz (transport + wake-up only),
agent /v1/node (view incl. the kubelet PodResources lookup), apiserver GET, kubelet PodResources
List. Run on the GPU box to see that host's idle-wake costs; prints JSON."""
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, ".")
from gpupool.agent.podresources import list_pod_devices  # noqa: E402
from gpupool.kube import Client, NODES  # noqa: E402
from gpupool.testing.cluster import Cluster, NodeSpec  # noqa: E402

node = NodeSpec("n0", backend="fake", probe="simulated", count=8)
cl = Cluster(tempfile.mkdtemp(prefix="rpc-"), nodes=[node], manager=False)
cl.start()
try:
    agent = Client("unix://" + cl.agent_socket("n0"), cl.agent_token)
    prs = os.path.join(cl.kubelet_root(node), "pod-resources", "kubelet.sock")
    ops = {"agent_healthz": lambda: agent.request("GET", "/healthz"),
           "agent_node": lambda: agent.request("GET", "/v1/node"),
           "apiserver_get_node": lambda: cl.client.get(NODES, "n0"),
           "kubelet_podresources_list": lambda: list_pod_devices(prs)}
    res = {}
    for gap in (0.0, 0.2, 1.0):
        for name, op in ops.items():
            xs = []
            for _ in range(10):
                if gap:
                    time.sleep(gap)
                t0 = time.perf_counter()
                op()
                xs.append((time.perf_counter() - t0) * 1e3)
            res[f"{name}@gap{gap}"] = round(statistics.median(xs), 3)
    print(json.dumps(res, indent=1))
finally:
    cl.stop()
