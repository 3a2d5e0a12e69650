"""Node-agent views: ``devices``, ``top``, ``gpu cordon|uncordon`` — the agent found through its
Pod / Node, called with the manager's signing key or token when one is configured."""
from __future__ import annotations

import json
import os
import sys

from ..api import schema
from ..kube import NODES, PODS, Client, KubeError
from .common import dump


def cmd_devices(c: Client, ns: str, args) -> int:
    node = c.get(NODES, args.node)
    ep = _agent_endpoint(c, node)
    if not ep:
        print(f"error: node {args.node} has no gpupool agent", file=sys.stderr)
        return 1
    view = _agent_client(args.node, ep).request("GET", "/v1/node")
    if args.output in ("json", "yaml"):
        dump(view, args.output)
        return 0
    src = view.get("eventSources") or {}
    print(f"node {view['node']}  backend {view['backend']}  probe {view.get('probeMode')}  "
          f"events {','.join(k for k, v in sorted(src.items()) if v) or '-'}")
    helpers = view.get("probeHelpers") or {}
    if helpers:  # the per-GPU probe processes (and the xGMI fabric helper)
        by_uuid = {d["uuid"]: d.get("index") for d in view["devices"]}
        up = sum(1 for v in helpers.values() if v.get("alive"))
        fabric = helpers.get("fabric") or {}
        line = f"probe helpers {up}/{len(helpers)} up"
        if fabric:
            line += (f"  fabric {'up' if fabric.get('alive') else 'DOWN'}"
                     + (f" (warm {fabric['warmMs']:.0f} ms)" if fabric.get("warmMs") is not None else ""))
        print(line)
        for key, v in sorted(helpers.items(), key=lambda kv: str(by_uuid.get(kv[0], kv[0]))):
            if not v.get("alive") or v.get("lastExit"):
                who = "fabric" if key == "fabric" else f"gpu {by_uuid.get(key, key)}"
                print(f"  helper {who}: {'up' if v.get('alive') else 'DOWN'}"
                      + (f", last exit: {v['lastExit']}" if v.get("lastExit") else ""))
    print(f"{'IDX':<4}{'HIP UUID':<24}{'BDF':<15}{'PART':<5}{'STATE':<12}{'HEALTHY':<8}{'GFX%':<5}"
          f"{'VRAM(GiB)':<11}{'POWER':<7}{'POOL':<24}REASONS")
    for d in sorted(view["devices"], key=lambda x: x.get("index", 0)):
        t = d.get("telemetry") or {}
        used, total = t.get("memUsedBytes"), t.get("memTotalBytes")
        vram = f"{used / 2**30:.0f}/{total / 2**30:.0f}" if used is not None and total else "-"
        gfx = "-" if t.get("gfxActivity") is None else str(t["gfxActivity"])
        power = "-" if t.get("powerW") is None else f"{t['powerW']}W"
        print(f"{d.get('index', ''):<4}{d.get('hipUUID', ''):<24}{d.get('bdf', ''):<15}"
              f"{(d.get('partition') or {}).get('compute', '-'):<5}"
              f"{d.get('state', '') + ('!' if d.get('probeOverdue') else ''):<12}"
              f"{'yes' if d.get('healthy') else 'NO':<8}{gfx:<5}{vram:<11}"
              f"{power:<7}{d.get('pool', '') or '-':<24}"
              f"{'; '.join((d.get('verdict') or {}).get('reasons', []))}")
    for e in view.get("recentEvents") or []:
        print(f"event {e.get('at', '')} {e.get('source', '')} {e.get('type', '')} "
              f"gpu={e.get('index', '-')} {e.get('message', '')}".rstrip())
    return 0


def cmd_top(c: Client, ns: str, args) -> int:
    """gpuctl top [pools|gpus|pods]: live GPU utilisation (kubectl top for the pools; the
    reference's "Prometheus + Grafana, GPU utilisation", GPU调度平台搭建.md:800) read from every
    node agent; ``pods`` is the per-pod accounting of (time-shared) GPUs: VRAM and GPU-time share
    per pod (GPU调度平台搭建.md:800-802)."""
    rows = []
    for n in c.list(NODES)["items"]:
        ep = _agent_endpoint(c, n)
        if not ep:
            continue
        try:
            view = _agent_client(n["metadata"]["name"], ep).request("GET", "/v1/node")
        except Exception as e:  # an unreachable agent is a row, not a failure
            print(f"warning: node {n['metadata']['name']}: {e}", file=sys.stderr)
            continue
        for d in view["devices"]:
            rows.append((view["node"], d))
    num = lambda v: float(v) if isinstance(v, (int, float)) else 0.0  # noqa: E731
    if args.what == "pods":  # per-pod accounting on (shared) GPUs: the agent's process -> pod map
        print(f"{'NAMESPACE/POD':<36}{'NODE':<18}{'IDX':<5}{'POOL':<28}{'VRAM(GiB)':<11}{'GPU%':<6}"
              f"{'PIDS':<16}BUDGET(GiB)")
        for node, d in sorted(rows, key=lambda r: (r[0], r[1].get("index", 0))):
            for e in d.get("usage") or []:
                busy = e.get("gfxBusy")
                # isolated slots: the pod's HBM budget on this GPU, "!" when it holds more (its
                # in-pod limit is not in force)
                bud = e.get("slotBudgetBytes")
                budget = "-" if not bud else f"{bud / 2**30:.2f}" + ("!" if e.get("overBudget") else "")
                print(f"{e.get('namespace', '')}/{e.get('pod', ''):<{35 - len(e.get('namespace', ''))}}"
                      f" {node:<18}{d.get('index', ''):<5}{d.get('pool', '') or '-':<28}"
                      f"{num(e.get('vramBytes')) / 2**30:<11.2f}"
                      f"{'-' if busy is None else f'{100 * busy:.0f}':<6}"
                      f"{','.join(str(x) for x in e.get('pids') or []):<16}{budget}")
        return 0
    if args.what == "gpus":
        print(f"{'NODE':<18}{'IDX':<5}{'POOL':<28}{'GFX%':<6}{'UMC%':<6}{'POWER(W)':<10}VRAM(GiB)")
        for node, d in sorted(rows, key=lambda r: (r[0], r[1].get("index", 0))):
            t = d.get("telemetry") or {}
            print(f"{node:<18}{d.get('index', ''):<5}{d.get('pool', '') or '-':<28}"
                  f"{num(t.get('gfxActivity')):<6.0f}{num(t.get('umcActivity')):<6.0f}"
                  f"{num(t.get('powerW')):<10.0f}"
                  f"{num(t.get('memUsedBytes')) / 2**30:.0f}/{num(t.get('memTotalBytes')) / 2**30:.0f}")
        return 0
    pools: dict[str, list[dict]] = {}
    for _, d in rows:
        if d.get("pool"):
            pools.setdefault(d["pool"], []).append(d.get("telemetry") or {})
    print(f"{'POOL':<32}{'GPUS':<6}{'GFX%':<6}{'UMC%':<6}{'POWER(W)':<10}VRAM(GiB)")
    for p, ts in sorted(pools.items()):
        k = len(ts)
        print(f"{p:<32}{k:<6}{sum(num(t.get('gfxActivity')) for t in ts) / k:<6.0f}"
              f"{sum(num(t.get('umcActivity')) for t in ts) / k:<6.0f}"
              f"{sum(num(t.get('powerW')) for t in ts):<10.0f}"
              f"{sum(num(t.get('memUsedBytes')) for t in ts) / 2**30:.0f}/"
              f"{sum(num(t.get('memTotalBytes')) for t in ts) / 2**30:.0f}")
    return 0


def _agent(c: Client, node: str) -> Client | None:
    n = c.get(NODES, node)
    ep = _agent_endpoint(c, n)
    if not ep:
        print(f"error: node {node} has no gpupool agent", file=sys.stderr)
        return None
    return _agent_client(node, ep)


class _SignedAgentClient:
    """Calls one node's agent with a per-request signature for that node (the manager's key,
    $GPUPOOL_AGENT_SIGNING_KEY: an admin's copy of the gpupool-manager-signing-key Secret)."""

    def __init__(self, node: str, ep: str, key_file: str):
        from ..utils import edsig
        self.node, self.client, self.signer = node, Client(ep), edsig.Signer(key_file)

    def request(self, method: str, path: str, body=None):
        data = b"" if body is None else json.dumps(body).encode()
        return self.client.request(method, path, body, extra_headers={
            "X-Gpupool-Signature": self.signer.header(method, path, self.node, data)})


def _agent_endpoint(c: Client, node: dict) -> str | None:
    """The node's agent endpoint: its annotation, cross-checked against the agent Pod bound to
    the node (gpupool-system, app.kubernetes.io/name=gpupool-agent) when there is one — an
    annotation whose host is not that Pod's IP is refused, as the manager refuses it."""
    name = node["metadata"]["name"]
    ep = (node["metadata"].get("annotations") or {}).get(schema.ANN_AGENT_ENDPOINT)
    try:
        pods = c.list(PODS, schema.AGENT_NAMESPACE, label_selector="app.kubernetes.io/name=gpupool-agent",
                      field_selector=f"spec.nodeName={name}")["items"]
    except KubeError:
        pods = []
    ips = {(p.get("status") or {}).get("podIP") for p in pods
           if (p.get("status") or {}).get("phase") == "Running"} - {None, ""}
    if not ips:
        return ep
    import urllib.parse
    if ep and urllib.parse.urlparse(ep).hostname in ips:
        return ep
    ip = sorted(ips)[0]
    scheme = os.environ.get("GPUPOOL_AGENT_SCHEME", "https")
    port = os.environ.get("GPUPOOL_AGENT_PORT", "9443")
    if ep:
        print(f"warning: node {name}: agent-endpoint annotation {ep} is not its agent Pod "
              f"({ip}); using the Pod", file=sys.stderr)
    return f"{scheme}://{'[' + ip + ']' if ':' in ip else ip}:{port}"


def _agent_client(node: str, ep: str):
    key = os.environ.get("GPUPOOL_AGENT_SIGNING_KEY")
    if key and os.path.exists(key):
        return _SignedAgentClient(node, ep, key)
    return Client(ep, _agent_token())


def _agent_token() -> str | None:
    """The node agents' shared RPC secret: $GPUPOOL_AGENT_TOKEN or the file named by
    $GPUPOOL_AGENT_TOKEN_FILE (the gpupool-agent-token Secret in a cluster)."""
    tok = os.environ.get("GPUPOOL_AGENT_TOKEN")
    path = os.environ.get("GPUPOOL_AGENT_TOKEN_FILE")
    if not tok and path and os.path.exists(path):
        with open(path) as f:
            tok = f.read().strip()
    return tok or None


def cmd_gpu(c: Client, ns: str, args) -> int:
    """gpuctl gpu cordon|uncordon NODE GPU [--reason R]: per-GPU maintenance (the per-device
    analogue of `kubectl cordon`): never claimed while cordoned; a pool holding it replaces it."""
    agent = _agent(c, args.node)
    if agent is None:
        return 1
    try:
        out = agent.request("POST", "/v1/maintenance", {"gpu": args.gpu, "on": args.action == "cordon",
                                                        "reason": args.reason or ""})
    except KubeError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    what = "cordoned" if out["maintenance"] else "uncordoned"
    held = f" (held by pool {out['claimedBy']}: it will be replaced)" if out.get("claimedBy") and \
        out["maintenance"] else ""
    print(f"gpu/{out['uuid']} on {args.node} {what}{held}")
    return 0
