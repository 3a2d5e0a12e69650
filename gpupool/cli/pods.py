"""Pod workflows: ``logs`` (pods/log), ``create namespace|secret|configmap``, ``run`` (the
reference's one-off GPU smoke-test pod) and ``events``."""
from __future__ import annotations

import json
import os
import sys
from typing import Any

from ..kube import EVENTS, PODS, Client, KubeError
from .common import print_table


def pod_log(c: Client, ns: str, name: str, tail: int | None = None, follow: bool = False,
            out=None) -> int:
    """``pods/{name}/log`` (the kubelet's log through the apiserver, as ``kubectl logs``)."""
    out = out or sys.stdout
    q = {"tailLines": tail, "follow": "true" if follow else None}
    path = PODS.path(ns, name, "log")
    if not follow:
        try:
            text = c.request("GET", path, query=q, accept="text/plain")
        except KubeError as e:
            print(f"error: {e}", file=sys.stderr)
            return 1
        out.write(text if isinstance(text, str) else json.dumps(text) + "\n")
        return 0
    conn = c._conn(timeout=None)
    conn.request("GET", path + "?" + "&".join(f"{k}={v}" for k, v in q.items() if v is not None),
                 headers=c._headers("application/json", "text/plain"))
    resp = conn.getresponse()
    if resp.status >= 400:
        print(f"error: HTTP {resp.status}: {resp.read().decode(errors='replace')}", file=sys.stderr)
        return 1
    while True:
        chunk = resp.read1(65536) if hasattr(resp, "read1") else resp.read(4096)
        if not chunk:
            break
        out.write(chunk.decode(errors="replace"))
        out.flush()
    conn.close()
    return 0


def cmd_logs(c: Client, ns: str, args) -> int:
    return pod_log(c, ns, args.pod, args.tail, args.follow)


def cmd_create(c: Client, ns: str, args) -> int:
    """``kubectl create namespace|secret generic|configmap`` (README.md:244-252 creates the
    Azure credentials Secret this way)."""
    import base64
    from ..kube import CONFIGMAPS, NAMESPACES, SECRETS
    names = list(args.name)
    if args.what == "secret" and names[0] == "generic":
        names = names[1:]
    if len(names) != 1:
        print(f"error: create {args.what} takes one name", file=sys.stderr)
        return 1
    name = names[0]
    if args.what == "namespace":
        c.create(NAMESPACES, {"apiVersion": "v1", "kind": "Namespace",
                              "metadata": {"name": name}})
        print(f"namespace/{name} created")
        return 0
    data: dict[str, str] = {}
    for lit in args.from_literal or []:
        k, sep, v = lit.partition("=")
        if not sep:
            print(f"error: --from-literal {lit!r} is not key=value", file=sys.stderr)
            return 1
        data[k] = v
    for spec in args.from_file or []:
        k, sep, f = spec.partition("=")
        if not sep:
            k, f = os.path.basename(spec), spec
        with open(f, "rb") as fh:
            raw = fh.read()
        data[k] = raw.decode() if args.what == "configmap" else raw  # type: ignore[assignment]
    if args.what == "configmap":
        c.create(CONFIGMAPS, {"apiVersion": "v1", "kind": "ConfigMap",
                              "metadata": {"name": name}, "data": data}, ns)
        print(f"configmap/{name} created")
        return 0
    enc = {k: base64.b64encode(v if isinstance(v, bytes) else v.encode()).decode()
           for k, v in data.items()}
    c.create(SECRETS, {"apiVersion": "v1", "kind": "Secret", "type": "Opaque",
                       "metadata": {"name": name}, "data": enc}, ns)
    print(f"secret/{name} created")
    return 0


def cmd_run(c: Client, ns: str, args) -> int:
    """``kubectl run NAME --image IMG [--gpus N] [--rm] -- CMD...``: one pod (restartPolicy
    Never) asking for N GPUs of ``--resource``; with ``--rm`` wait for it, print its log, delete
    it, and exit with its exit code — the reference's GPU smoke test
    (``kubectl run --rm -it --gpus=1 gpu-test ... nvidia-smi``, GPU调度平台搭建.md:134-138) is
    ``gpuctl run --rm --gpus 1 gpu-test --image rocm/dev-ubuntu-22.04 -- amd-smi static``."""
    cmd = list(args.command or [])
    ctr: dict[str, Any] = {"name": args.name, "image": args.image}
    if cmd:
        ctr["command"] = cmd
    if args.gpus:
        ctr["resources"] = {"limits": {args.resource: args.gpus}}
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"name": args.name, "labels": {"run": args.name}},
           "spec": {"restartPolicy": "Never", "containers": [ctr]}}
    c.create(PODS, pod, ns)
    if not args.rm:
        print(f"pod/{args.name} created")
        return 0
    try:
        o = c.wait_for(PODS, args.name, ns, lambda o: not o or o.get("status", {}).get("phase")
                       in ("Succeeded", "Failed"), timeout=args.timeout)
        pod_log(c, ns, args.name)
        code = 1
        if o:
            cs = (o.get("status") or {}).get("containerStatuses") or []
            term = ((cs[0].get("state") or {}).get("terminated") or {}) if cs else {}
            code = int(term.get("exitCode", 0 if o["status"].get("phase") == "Succeeded" else 1))
    except TimeoutError:
        print(f"error: pod/{args.name} did not finish within {args.timeout:g} s", file=sys.stderr)
        code = 1
    try:
        c.delete(PODS, args.name, ns, grace=0)
    except KubeError:
        pass
    print(f'pod "{args.name}" deleted', file=sys.stderr)
    return code


def cmd_events(c: Client, ns: str, args) -> int:
    print_table(c.table(EVENTS, None if args.all_namespaces else ns), with_ns=args.all_namespaces)
    return 0
