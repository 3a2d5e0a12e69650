"""gpuctl — the kubectl stand-in for the gpupool operator.

  gpuctl apply -f FILE [--dry-run] [--server-side [--force-conflicts] [--field-manager M]]
                                          kubectl apply (README.md:288-290): three-way merge with
                                          the last applied configuration, or server-side apply
  gpuctl diff -f FILE [--server-side]     what apply would change (server dry run), exit 1 if any
  gpuctl get KIND [NAME] [-o wide|yaml|json|name|jsonpath=TPL] [-l SEL] [-A]   server-side printing
  gpuctl describe KIND NAME               spec/status, conditions table, devices, events
  gpuctl delete KIND NAME | -f FILE [--wait]
  gpuctl scale KIND NAME --replicas N     via the scale subresource
  gpuctl wait KIND NAME --for condition=Ready|delete|jsonpath=.status.readyReplicas=N [--timeout 60]
  gpuctl logs POD [-f] [--tail N]         the pod's log (pods/log)
  gpuctl create namespace NAME | secret generic NAME --from-literal k=v | configmap NAME ...
  gpuctl run NAME --image IMG [--gpus N] [--rm] -- CMD...   one pod; --rm: wait, log, delete
  gpuctl keys [status|init|rotate|prune]  the manager's agent-RPC signing key, rotated in steps
  gpuctl events [-n NS]
  gpuctl devices NODE                     the node agent's live device view
  gpuctl gpu cordon|uncordon NODE GPU     per-GPU maintenance (replace it in its pool, never claim)
  gpuctl install [--crd-dir config/crd]   install CRDs (make install)
  gpuctl render job -f TEMPLATE           GoHai train-job template -> Pod requesting amd.com/gpu
  gpuctl config view | set-context NAME --server URL [--namespace NS] [--token T] | use-context NAME

Connection (first match wins): --server/--token/-n flags or GPUPOOL_APISERVER/GPUPOOL_TOKEN;
--kubeconfig/--context or $KUBECONFIG (kubectl's file: token, tokenFile, client certificates,
CA); the current context of ~/.config/gpupool/config.yaml (the GoHai CLI context schema,
GPU调度平台搭建.md:461-472); ~/.kube/config.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import sys
import time
from typing import Any

import yaml

from ..api import schema
from ..kube import EVENTS, MI355XJOBS, NODES, PODS, Client, KubeError, Res, res_for

CONFIG_PATH = os.path.expanduser(os.environ.get("GPUPOOL_CONFIG", "~/.config/gpupool/config.yaml"))


# ------------------------------------------------------------------ config / contexts
def load_config() -> dict:
    if os.path.exists(CONFIG_PATH):
        with open(CONFIG_PATH) as f:
            return yaml.safe_load(f) or {}
    return {}


def save_config(cfg: dict) -> None:
    os.makedirs(os.path.dirname(CONFIG_PATH), exist_ok=True)
    with open(CONFIG_PATH, "w") as f:
        yaml.safe_dump(cfg, f, sort_keys=False)


USER_AGENT = "gpuctl/0.1"  # the field manager the apiserver records for gpuctl's plain writes


def connection(args) -> tuple[Client, str]:
    """First match wins: --server / $GPUPOOL_APISERVER, --kubeconfig / $KUBECONFIG, the current
    gpuctl context, ~/.kube/config, http://127.0.0.1:6443."""
    cfg = load_config()
    ctx = (cfg.get("contexts") or {}).get(cfg.get("current-context", ""), {})
    server = args.server or os.environ.get("GPUPOOL_APISERVER")
    kubeconfig = getattr(args, "kubeconfig", None) or os.environ.get("KUBECONFIG")
    if not server and not ctx.get("server") and not kubeconfig and \
            os.path.exists(os.path.expanduser("~/.kube/config")):
        kubeconfig = os.path.expanduser("~/.kube/config")
    if not server and kubeconfig:
        c = Client.from_kubeconfig(kubeconfig, getattr(args, "context", None))
        if args.token:
            c.token = args.token
        c.user_agent = USER_AGENT
        return c, args.namespace or c.namespace or "default"
    server = server or ctx.get("server") or "http://127.0.0.1:6443"
    token = args.token or os.environ.get("GPUPOOL_TOKEN") or ctx.get("token")
    ns = args.namespace or ctx.get("namespace") or "default"
    c = Client(server, token)
    c.user_agent = USER_AGENT
    return c, ns


# ------------------------------------------------------------------ discovery
def resolve(c: Client, name: str) -> Res:
    n = name.lower()
    for path in ["/api/v1"] + [f"/apis/{g['name']}/{g['preferredVersion']['version']}"
                               for g in c.request("GET", "/apis").get("groups", [])]:
        lst = c.request("GET", path)
        gv = lst["groupVersion"]
        g, v = gv.split("/", 1) if "/" in gv else ("", gv)
        for r in lst["resources"]:
            if "/" in r["name"]:
                continue
            names = {r["name"], r.get("singularName", ""), r["kind"].lower(),
                     *r.get("shortNames", [])}
            if n in names or n == f"{r['name']}.{g}":
                return Res(g, v, r["name"], r["namespaced"])
    raise SystemExit(f"error: the server doesn't have a resource type \"{name}\"")


def load_docs(path: str) -> list[dict]:
    paths = sorted(glob.glob(os.path.join(path, "*.y*ml"))) if os.path.isdir(path) else [path]
    docs = []
    for p in paths:
        with (sys.stdin if p == "-" else open(p)) as f:
            docs += [d for d in yaml.safe_load_all(f) if d]
    return docs


# ------------------------------------------------------------------ printing
def print_table(tbl: dict, wide: bool = False, with_ns: bool = False) -> None:
    cols = [cd["name"].upper() for cd in tbl["columnDefinitions"]]
    rows = []
    for r in tbl["rows"]:
        cells = ["" if x is None else str(x) for x in r["cells"]]
        if with_ns:
            cells = [r["object"]["metadata"].get("namespace", "")] + cells
        rows.append(cells)
    if with_ns:
        cols = ["NAMESPACE"] + cols
    if not rows:
        print("No resources found.")
        return
    widths = [max(len(cols[i]), *(len(r[i]) for r in rows)) for i in range(len(cols))]
    print("   ".join(c.ljust(w) for c, w in zip(cols, widths)).rstrip())
    for r in rows:
        print("   ".join(c.ljust(w) for c, w in zip(r, widths)).rstrip())


def dump(obj: Any, fmt: str) -> None:
    if fmt == "json":
        print(json.dumps(obj, indent=2))
    else:
        print(yaml.safe_dump(obj, sort_keys=False).rstrip())


# ------------------------------------------------------------------ commands
def cmd_apply(c: Client, ns: str, args) -> int:
    from .convert import ConvertError, convert, convertible
    rc = 0
    for doc in load_docs(args.filename):
        if convertible(doc):  # the reference's Volcano Job / Kubeflow PyTorchJob: as a Mi355xJob
            try:
                doc, warns = convert(doc)
            except ConvertError as e:
                print(f"error: {e}", file=sys.stderr)
                rc = 1
                continue
            print(f"converted {doc['metadata']['annotations']['gpupool.amd.com/converted-from']} "
                  f"{doc['metadata']['name']} to Mi355xJob", file=sys.stderr)
            for w in warns:
                print(f"warning: {w}", file=sys.stderr)
        try:
            action, out = c.apply(doc, ns, dry_run=args.dry_run, server_side=args.server_side,
                                  field_manager=args.field_manager, force=args.force_conflicts)
            suffix = " (dry run)" if args.dry_run else ""
            print(f"{doc['kind'].lower()}.{res_for(doc).group or 'core'}/{doc['metadata']['name']} "
                  f"{action}{suffix}")
            if args.dry_run and args.output:
                dump(out, args.output)
        except KubeError as e:
            print(f"error: {e}", file=sys.stderr)
            rc = 1
    return rc


_DIFF_SKIP_META = ("resourceVersion", "generation", "managedFields", "uid", "creationTimestamp")


def _diff_view(obj: dict | None) -> str:
    """An object as ``kubectl diff`` compares it: server bookkeeping and apply's own annotation
    left out, YAML with stable key order."""
    if obj is None:
        return ""
    o = json.loads(json.dumps(obj))
    md = o.get("metadata") or {}
    for k in _DIFF_SKIP_META:
        md.pop(k, None)
    ann = md.get("annotations") or {}
    ann.pop(Client.LAST_APPLIED, None)
    if not ann:
        md.pop("annotations", None)
    return yaml.safe_dump(o, sort_keys=True)


def cmd_diff(c: Client, ns: str, args) -> int:
    """``kubectl diff``: what ``apply`` would change, from a server-side dry run of that apply
    (defaulting, admission and the merge as the server does them). Exit 1 when anything would
    change, 0 when nothing would, >1 on errors."""
    import difflib
    changed = False
    from .convert import convert, convertible
    for doc in load_docs(args.filename):
        if convertible(doc):
            doc, _ = convert(doc)
        res = res_for(doc)
        name = doc["metadata"]["name"]
        dns = (doc["metadata"].get("namespace") or ns) if res.namespaced else None
        try:
            cur = c.get(res, name, dns)
        except KubeError as e:
            if e.code != 404:
                print(f"error: {e}", file=sys.stderr)
                return 2
            cur = None
        try:
            _, out = c.apply(doc, dns, dry_run=True, server_side=args.server_side,
                             field_manager=args.field_manager, force=args.force_conflicts)
        except KubeError as e:
            print(f"error: {e}", file=sys.stderr)
            return 2
        a, b = _diff_view(cur), _diff_view(out)
        if a == b:
            continue
        changed = True
        label = f"{res.group or 'v1'}.{doc['kind']}.{dns + '.' if dns else ''}{name}"
        sys.stdout.writelines(difflib.unified_diff(
            a.splitlines(keepends=True), b.splitlines(keepends=True),
            fromfile=f"live/{label}", tofile=f"merged/{label}"))
    return 1 if changed else 0


def cmd_get(c: Client, ns: str, args) -> int:
    res = resolve(c, args.kind)
    target_ns = None if (args.all_namespaces or not res.namespaced) else ns
    if args.output in ("yaml", "json") or args.output.startswith("jsonpath=") or \
            args.output == "name":
        out = c.get(res, args.name, target_ns) if args.name else \
            c.list(res, target_ns, label_selector=args.selector)
        if args.output == "name":  # kubectl get -o name: kind.group/name per object
            for o in ([out] if args.name else out["items"]):
                kind = (o.get("kind") or res.plural.rstrip("s")).lower()
                print(f"{kind}{'.' + res.group if res.group else ''}/{o['metadata']['name']}")
            return 0
        if args.output.startswith("jsonpath="):
            from .jsonpath import JsonPathError, render
            try:
                sys.stdout.write(render(out, args.output.split("=", 1)[1]))
            except JsonPathError as e:
                print(f"error: {e}", file=sys.stderr)
                return 1
            return 0
        dump(out, args.output)
        return 0
    tbl = c.table(res, target_ns, args.name, label_selector=args.selector)
    print_table(tbl, wide=args.output == "wide", with_ns=args.all_namespaces and res.namespaced)
    if args.watch:  # `kubectl get -w` (GPU调度平台搭建.md:682): one row per change, no header
        sys.stdout.flush()
        rv = tbl.get("metadata", {}).get("resourceVersion")
        deadline = time.monotonic() + args.watch_timeout if args.watch_timeout else None
        for ev in c.watch(res, target_ns, resource_version=rv, label_selector=args.selector,
                          field_selector=f"metadata.name={args.name}" if args.name else None,
                          timeout_seconds=int(args.watch_timeout) if args.watch_timeout else None,
                          bookmarks=False):
            obj = ev.get("object") or {}
            md = obj.get("metadata") or {}
            if ev.get("type") == "DELETED":
                print(f"{md.get('name', '')}   <deleted>", flush=True)
            elif ev.get("type") in ("ADDED", "MODIFIED"):
                try:
                    row = c.table(res, md.get("namespace") if res.namespaced else None, md["name"])
                except KubeError:
                    continue  # gone between the event and the GET
                for r in row["rows"]:
                    cells = ["" if x is None else str(x) for x in r["cells"]]
                    if args.all_namespaces and res.namespaced:
                        cells = [md.get("namespace", "")] + cells
                    print("   ".join(cells), flush=True)
            if deadline and time.monotonic() > deadline:
                break
    return 0


def _events_for(c: Client, ns: str, uid: str) -> list[dict]:
    evs = [e for e in c.list(EVENTS, ns)["items"] if e.get("involvedObject", {}).get("uid") == uid]
    return sorted(evs, key=lambda e: e.get("lastTimestamp", ""))


def cmd_describe(c: Client, ns: str, args) -> int:
    res = resolve(c, args.kind)
    obj = c.get(res, args.name, ns if res.namespaced else None)
    md = obj["metadata"]
    print(f"Name:         {md['name']}")
    if res.namespaced:
        print(f"Namespace:    {md.get('namespace')}")
    print(f"Kind:         {obj['kind']}")
    print(f"UID:          {md.get('uid')}")
    print(f"Generation:   {md.get('generation')}")
    if md.get("finalizers"):
        print(f"Finalizers:   {', '.join(md['finalizers'])}")
    if md.get("deletionTimestamp"):
        print(f"Deleting:     since {md['deletionTimestamp']}")
    for k in ("labels", "annotations"):
        if md.get(k):
            print(f"{k.capitalize()}:")
            for kk, vv in md[k].items():
                print(f"  {kk}={vv}")
    if "spec" in obj:
        print("Spec:")
        print("  " + yaml.safe_dump(obj["spec"], sort_keys=False).rstrip().replace("\n", "\n  "))
    st = dict(obj.get("status") or {})
    conds = st.pop("conditions", [])
    devs = st.pop("devices", None)
    if st:
        print("Status:")
        print("  " + yaml.safe_dump(st, sort_keys=False).rstrip().replace("\n", "\n  "))
    if devs:
        print("Devices:")
        print(f"  {'INDEX':<6}{'UUID':<42}{'HEALTH':<11}{'ADV':<5}{'PROBE':<28}PODS")
        for d in devs:
            p = d.get("probe") or {}
            probe = (f"{'ok' if p.get('passed') else 'FAIL'} {p.get('hbmGBps', 0):.0f}GB/s "
                     f"{p.get('mfmaTflops', 0):.0f}TF") if p else "-"
            print(f"  {d.get('index', ''):<6}{d.get('hipUUID') or d['uuid']:<42}"
                  f"{d.get('health', ''):<11}{'yes' if d.get('advertised') else 'no':<5}"
                  f"{probe:<28}{','.join(d.get('pods', [])) or '-'}")
            for r in d.get("reasons") or []:
                print(f"        ! {r}")
    if conds:
        print("Conditions:")
        print(f"  {'TYPE':<20}{'STATUS':<9}{'REASON':<24}MESSAGE")
        for cd in conds:
            print(f"  {cd['type']:<20}{cd['status']:<9}{cd.get('reason', ''):<24}{cd.get('message', '')}")
    if res.namespaced:
        evs = _events_for(c, md.get("namespace"), md.get("uid"))
        print("Events:" + ("" if evs else "  <none>"))
        for e in evs[-20:]:
            print(f"  {e.get('type', ''):<8}{e.get('reason', ''):<20}x{e.get('count', 1):<4}"
                  f"{e.get('message', '')}")
    return 0


def cmd_delete(c: Client, ns: str, args) -> int:
    targets = []
    if args.filename:
        for d in load_docs(args.filename):
            r = res_for(d)
            targets.append((r, d["metadata"]["name"], d["metadata"].get("namespace") or ns))
    else:
        r = resolve(c, args.kind)
        targets.append((r, args.name, ns))
    for r, name, tns in targets:
        try:
            c.delete(r, name, tns if r.namespaced else None)
            print(f"{r.plural}/{name} deleted")
        except KubeError as e:
            print(f"error: {e}", file=sys.stderr)
            continue
        if args.wait:
            c.wait_for(r, name, tns if r.namespaced else None, lambda o: o is None,
                       timeout=args.timeout)
    return 0


def cmd_scale(c: Client, ns: str, args) -> int:
    res = resolve(c, args.kind)
    cur = c.get(res, args.name, ns, sub="scale")
    cur["spec"]["replicas"] = args.replicas
    c.request("PUT", res.path(ns, args.name, "scale"), cur)
    print(f"{res.plural}/{args.name} scaled")
    return 0


def parse_for(cond: str):
    if cond == "delete":
        return lambda o: o is None
    if cond.startswith("condition="):
        spec = cond.split("=", 1)[1]
        ctype, _, want = spec.partition("=")
        want = want or "True"
        return lambda o: bool(o) and any(
            x["type"] == ctype and x["status"] == want and
            x.get("observedGeneration", o["metadata"].get("generation")) ==
            o["metadata"].get("generation")
            for x in (o.get("status") or {}).get("conditions", []))
    if cond.startswith("jsonpath="):
        from .jsonpath import _str, evaluate
        spec = cond.split("=", 1)[1]
        if spec.startswith("{"):  # kubectl form: jsonpath='{.status.readyReplicas}'=2
            j = spec.index("}")
            path, want = spec[1:j], spec[j + 1:].lstrip("=")
        else:
            path, _, want = spec.partition("=")

        def pred(o):
            return o is not None and any(_str(v) == want for v in evaluate(o, path))
        return pred
    raise SystemExit(f"error: unsupported --for {cond}")


def cmd_wait(c: Client, ns: str, args) -> int:
    res = resolve(c, args.kind)
    t0 = time.monotonic()
    try:
        c.wait_for(res, args.name, ns if res.namespaced else None, parse_for(args.for_),
                   timeout=args.timeout)
    except TimeoutError:
        print(f"error: timed out waiting for the condition on {res.plural}/{args.name}",
              file=sys.stderr)
        return 1
    print(f"{res.plural}/{args.name} condition met ({time.monotonic() - t0:.3f}s)")
    return 0


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


def cmd_keys(c: Client, ns: str, args) -> int:
    from . import keys
    return keys.main(c, args)


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


def cmd_install(c: Client, ns: str, args) -> int:
    from ..kube import CRDS
    for doc in load_docs(args.crd_dir):
        action, _ = c.apply(doc)
        print(f"customresourcedefinition.apiextensions.k8s.io/{doc['metadata']['name']} {action}")
        c.wait_for(CRDS, doc["metadata"]["name"], None, lambda o: bool(o) and any(
            x["type"] == "Established" and x["status"] == "True"
            for x in (o.get("status") or {}).get("conditions", [])), timeout=30)
    return 0


def render_job(tpl: dict) -> dict:
    """GoHai train-job template (GPU调度平台搭建.md:512-535) -> Pod requesting amd.com/gpu."""
    spec = tpl.get("spec") or {}
    inst = str(spec.get("singleInstanceType", "gpu-1x"))
    gpus = 1
    for part in inst.split("-"):
        if part.endswith("gpu") and part[:-3].isdigit():
            gpus = int(part[:-3])
    env = [{"name": k, "value": str(v)} for k, v in (tpl.get("env") or {}).items()] \
        if isinstance(tpl.get("env"), dict) else list(tpl.get("env") or [])
    cmd = tpl.get("command") or "python train.py"
    name = str(tpl.get("title", "trainjob")).lower().replace(" ", "-").replace("_", "-")
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"generateName": name + "-",
                         "annotations": {"gpupool.amd.com/description": str(tpl.get("description", "")),
                                         "gpupool.amd.com/mode": str(tpl.get("mode", "single")).lower()}},
            "spec": {"restartPolicy": "OnFailure",
                     "containers": [{"name": "train", "image": tpl.get("image", "rocm/pytorch:latest"),
                                     "command": ["bash", "-lc", cmd], "env": env,
                                     "resources": {"limits": {schema.DEFAULT_RESOURCE: gpus}}}]}}


def _dns_name(title: str, limit: int = 50) -> str:
    out = re.sub(r"[^a-z0-9-]+", "-", str(title).lower()).strip("-")
    return (out[:limit].rstrip("-")) or "trainjob"


def _gpus_of(instance_type: str) -> int:
    """``gpu-1x-16c-32g-1gpu`` -> 1 (the trailing ``<N>gpu`` part; GPU调度平台搭建.md:534)."""
    for part in str(instance_type).split("-"):
        if part.endswith("gpu") and part[:-3].isdigit():
            return int(part[:-3])
    return 1


def render_trainjob(tpl: dict) -> dict:
    """GoHai train-job template (GPU调度平台搭建.md:512-535, full form :828-851) -> Mi355xJob.

    ``mode: single`` (either case, the reference uses both :532/:848) is one worker; ``mode:
    distributed`` takes ``spec.replicas`` (or ``spec.workers``) workers. GPUs per worker come from
    the instance type's ``<N>gpu`` suffix. Repository/dataset/model references are kept as
    annotations (the platform services that would mount them are out of scope)."""
    spec = tpl.get("spec") or {}
    mode = str(tpl.get("mode", "single")).lower()
    replicas = 1 if mode == "single" else int(spec.get("replicas") or spec.get("workers") or 2)
    inst = spec.get("singleInstanceType") or spec.get("instanceType") or "gpu-1x"
    env = [{"name": k, "value": str(v)} for k, v in (tpl.get("env") or {}).items()] \
        if isinstance(tpl.get("env"), dict) else list(tpl.get("env") or [])
    cmd = tpl.get("command") or "python train.py"
    ann = {"gpupool.amd.com/description": str(tpl.get("description", "")),
           "gpupool.amd.com/title": str(tpl.get("title", "")),
           "gpupool.amd.com/mode": mode, "gpupool.amd.com/instance-type": str(inst)}
    for key in ("repository", "dataset", "model"):
        if tpl.get(key):
            ann[f"gpupool.amd.com/{key}"] = json.dumps(tpl[key], sort_keys=True)
    job_spec = {"replicas": replicas, "gpusPerReplica": _gpus_of(inst),
                "restartPolicy": "OnFailure",
                "template": {"metadata": {"labels": {"app": "trainjob"}},
                             "spec": {"containers": [{
                                 "name": "train", "image": tpl.get("image", "rocm/pytorch:latest"),
                                 "command": ["bash", "-lc", cmd], "env": env}]}}}
    for k in ("poolRef", "queue", "priority", "preemptionPolicy", "backoffLimit",
              "activeDeadlineSeconds", "ttlSecondsAfterFinished", "masterPort", "minAvailable",
              "checkpointDir"):
        if k in spec:
            job_spec[k] = spec[k]
    return {"apiVersion": schema.API_VERSION, "kind": "Mi355xJob",
            "metadata": {"name": _dns_name(tpl.get("title", "trainjob")), "annotations": ann},
            "spec": job_spec}


def job_to_template(job: dict) -> dict:
    """``trainjob template -s JOB``: export an existing Mi355xJob as a GoHai template."""
    md, spec = job["metadata"], job["spec"]
    ann = md.get("annotations") or {}
    c = ((spec.get("template") or {}).get("spec") or {}).get("containers", [{}])[0]
    cmd = c.get("command") or []
    cmd = cmd[-1] if len(cmd) == 3 and cmd[:2] == ["bash", "-lc"] else " ".join(cmd + c.get("args", []))
    out = {"title": ann.get("gpupool.amd.com/title") or md["name"],
           "description": ann.get("gpupool.amd.com/description", ""),
           "image": c.get("image", ""), "command": cmd,
           "env": {e["name"]: e.get("value", "") for e in c.get("env", []) if "value" in e}}
    for key in ("repository", "dataset", "model"):
        out[key] = json.loads(ann[f"gpupool.amd.com/{key}"]) if ann.get(f"gpupool.amd.com/{key}") else []
    n = int(spec.get("replicas", 1))
    out["mode"] = "single" if n == 1 else "distributed"
    out["spec"] = {"singleInstanceType": ann.get("gpupool.amd.com/instance-type")
                   or f"gpu-{spec.get('gpusPerReplica', 1)}gpu"}
    if n > 1:
        out["spec"]["replicas"] = n
    return out


SAMPLE_TRAINJOB = {
    "title": "fashion-mnist-demo",
    "description": "Fashion-MNIST CNN training via CLI template",
    "image": "rocm/pytorch:latest",
    "command": "python examples/fmnist_train.py --epochs 5 --batch_size 128",
    "env": {"GPUPOOL_CLI": "true"},
    "repository": [], "dataset": [], "model": [],
    "mode": "single",
    "spec": {"singleInstanceType": "gpu-1x-16c-32g-1gpu"},
}


def cmd_trainjob(c: Client, ns: str, args) -> int:
    """GoHai CLI's `trainjob` verbs (GPU调度平台搭建.md:503-505, :540-550) over Mi355xJob."""
    if args.tj_cmd == "template":
        tpl = job_to_template(c.get(MI355XJOBS, args.source, ns)) if args.source else SAMPLE_TRAINJOB
        print(yaml.safe_dump(tpl, sort_keys=False, allow_unicode=True).rstrip())
        return 0
    if args.tj_cmd == "create":
        rc = 0
        for d in load_docs(args.filename):
            job = d if args.bare else render_trainjob(d)
            if args.dry_run:
                dump(job, args.output or "yaml")
                continue
            out = c.create(MI355XJOBS, job, job.get("metadata", {}).get("namespace") or ns)
            print(f"mi355xjob.{schema.GROUP}/{out['metadata']['name']} created")
        return rc
    if args.tj_cmd == "list":
        print_table(c.table(MI355XJOBS, ns))
        return 0
    if args.tj_cmd in ("suspend", "resume"):
        c.patch(MI355XJOBS, args.job, {"spec": {"suspend": args.tj_cmd == "suspend"}}, ns)
        print(f"mi355xjob.{schema.GROUP}/{args.job} {args.tj_cmd}d")
        return 0
    if args.tj_cmd == "delete":
        c.delete(MI355XJOBS, args.job, ns)
        print(f"mi355xjob.{schema.GROUP}/{args.job} deleted")
        return 0
    if args.tj_cmd == "logs":
        pods = c.list(PODS, ns, label_selector=f"{schema.LABEL_JOB}={args.job}")["items"]
        pods.sort(key=lambda p: int(p["metadata"]["labels"].get(schema.LABEL_JOB_INDEX, 0)))
        if args.rank is not None:
            pods = [p for p in pods
                    if p["metadata"]["labels"].get(schema.LABEL_JOB_INDEX) == str(args.rank)]
        if not pods:
            print(f"error: no pods for trainjob {args.job}", file=sys.stderr)
            return 1
        for p in pods:
            if len(pods) > 1:
                print(f"==> {p['metadata']['name']} <==")
            pod_log(c, ns, p["metadata"]["name"])
        return 0
    return 2


def cmd_convert(args) -> int:
    """``gpuctl convert -f vcjob.yaml``: a Volcano Job or Kubeflow PyTorchJob as a Mi355xJob (no
    server needed); warnings for what has no equivalent go to stderr."""
    from .convert import ConvertError, convert
    rc, out = 0, []
    for doc in load_docs(args.filename):
        try:
            job, warns = convert(doc, pool=args.pool, resource=args.resource, image=args.image)
        except ConvertError as e:
            print(f"error: {e}", file=sys.stderr)
            rc = 1
            continue
        for w in warns:
            print(f"warning: {job['metadata']['name']}: {w}", file=sys.stderr)
        out.append(job)
    if args.output == "json":
        print(json.dumps(out[0] if len(out) == 1 else {"apiVersion": "v1", "kind": "List",
                                                         "items": out}, indent=2))
    else:
        print(yaml.safe_dump_all(out, sort_keys=False, allow_unicode=True).rstrip())
    return rc


def cmd_render(c, ns, args) -> int:
    for d in load_docs(args.filename):
        dump(render_job(d), args.output or "yaml")
    return 0


def cmd_config(args) -> int:
    cfg = load_config()
    cfg.setdefault("contexts", {})
    if args.config_cmd == "view":
        print(yaml.safe_dump(cfg, sort_keys=False).rstrip() or "{}")
    elif args.config_cmd == "set-context":
        ctx = cfg["contexts"].setdefault(args.name, {})
        for k in ("server", "namespace", "token"):
            v = getattr(args, k)
            if v:
                ctx[k] = v
        cfg.setdefault("current-context", args.name)
        save_config(cfg)
        print(f"context {args.name} set")
    elif args.config_cmd == "use-context":
        if args.name not in cfg["contexts"]:
            print(f"error: no context {args.name}", file=sys.stderr)
            return 1
        cfg["current-context"] = args.name
        save_config(cfg)
        print(f"switched to context {args.name}")
    elif args.config_cmd == "get-contexts":  # GoHai `context list` (GPU调度平台搭建.md:476-482)
        cur = cfg.get("current-context")
        print("CURRENT   NAME   SERVER   NAMESPACE")
        for name, ctx in sorted(cfg["contexts"].items()):
            print(f"{'*' if name == cur else ' '}   {name}   {ctx.get('server', '')}   "
                  f"{ctx.get('namespace', 'default')}")
    return 0


def cmd_login(args) -> int:
    """GoHai `login` (GPU调度平台搭建.md:476): store a bearer token (e.g. an OIDC id-token from
    the identity provider) in a context, creating or switching to it."""
    cfg = load_config()
    cfg.setdefault("contexts", {})
    name = args.context_name or cfg.get("current-context") or "default"
    ctx = cfg["contexts"].setdefault(name, {})
    token = args.token_value if args.token_value is not None else sys.stdin.readline().strip()
    if not token:
        print("error: empty token", file=sys.stderr)
        return 1
    ctx["token"] = token
    if args.server:
        ctx["server"] = args.server
    cfg["current-context"] = name
    save_config(cfg)
    print(f"logged in: context {name}")
    return 0


def cmd_whoami(c: Client, ns: str, args) -> int:
    """GoHai `whoami` (GPU调度平台搭建.md:482): the context, apiserver, namespace and credential in
    use, and whether the apiserver accepts it."""
    cfg = load_config()
    ok = True
    try:
        c.request("GET", "/version")
    except KubeError as e:
        ok = e.code not in (401, 403)
    except OSError:
        ok = False
    auth = "bearer token" if c.token else "no bearer token (anonymous or client certificate)"
    print(f"context:    {args.context or cfg.get('current-context') or '-'}")
    print(f"server:     {c.server}")
    print(f"namespace:  {ns}")
    print(f"credential: {auth}")
    print(f"reachable:  {'yes' if ok else 'no'}")
    return 0 if ok else 1


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="gpuctl", description="kubectl-like CLI for gpupool")
    ap.add_argument("--server", default=None)
    ap.add_argument("--token", default=None)
    ap.add_argument("--kubeconfig", default=None, help="kubeconfig file (default $KUBECONFIG)")
    ap.add_argument("--context", default=None, help="kubeconfig context (default current)")
    ap.add_argument("-n", "--namespace", default=None)
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("apply")
    p.add_argument("-f", "--filename", required=True)
    p.add_argument("--dry-run", action="store_true")
    p.add_argument("-o", "--output", default=None)
    p.add_argument("--server-side", action="store_true",
                   help="server-side apply (field ownership in managedFields)")
    p.add_argument("--field-manager", default="gpuctl")
    p.add_argument("--force-conflicts", action="store_true",
                   help="server-side apply: take fields other managers own")
    p = sub.add_parser("diff")
    p.add_argument("-f", "--filename", required=True)
    p.add_argument("--server-side", action="store_true")
    p.add_argument("--field-manager", default="gpuctl")
    p.add_argument("--force-conflicts", action="store_true")
    p = sub.add_parser("get")
    p.add_argument("kind")
    p.add_argument("name", nargs="?")
    p.add_argument("-o", "--output", default="")
    p.add_argument("-l", "--selector", default=None)
    p.add_argument("-A", "--all-namespaces", action="store_true")
    p.add_argument("-w", "--watch", action="store_true", help="after the table, print a row per change")
    p.add_argument("--watch-timeout", type=float, default=0, help="stop watching after N seconds")
    p = sub.add_parser("describe")
    p.add_argument("kind")
    p.add_argument("name")
    p = sub.add_parser("delete")
    p.add_argument("kind", nargs="?")
    p.add_argument("name", nargs="?")
    p.add_argument("-f", "--filename", default=None)
    p.add_argument("--wait", action="store_true")
    p.add_argument("--timeout", type=float, default=120)
    p = sub.add_parser("scale")
    p.add_argument("kind")
    p.add_argument("name")
    p.add_argument("--replicas", type=int, required=True)
    p = sub.add_parser("wait")
    p.add_argument("kind")
    p.add_argument("name")
    p.add_argument("--for", dest="for_", required=True)
    p.add_argument("--timeout", type=float, default=60)
    p = sub.add_parser("logs")
    p.add_argument("pod")
    p.add_argument("-f", "--follow", action="store_true")
    p.add_argument("--tail", type=int, default=None)
    p = sub.add_parser("keys", help="the manager's agent-RPC signing key (gpupool/cli/keys.py)")
    p.add_argument("keys_cmd", choices=["status", "init", "rotate", "prune"], nargs="?",
                   default="status")
    p.add_argument("--force", action="store_true", help="skip the check on the agents")
    p.add_argument("--key-namespace", default=None, help="default: gpupool-system")
    p = sub.add_parser("create")
    p.add_argument("what", choices=["namespace", "secret", "configmap"])
    p.add_argument("name", nargs="+", help="NAME, or 'generic NAME' for a secret")
    p.add_argument("--from-literal", action="append")
    p.add_argument("--from-file", action="append")
    p = sub.add_parser("run")
    p.add_argument("name")
    p.add_argument("--image", required=True)
    p.add_argument("--gpus", type=int, default=0)
    p.add_argument("--resource", default=schema.DEFAULT_RESOURCE)
    p.add_argument("--rm", action="store_true", help="wait, print the log, delete the pod")
    p.add_argument("-i", "--stdin", action="store_true", help="accepted for kubectl parity")
    p.add_argument("-t", "--tty", action="store_true", help="accepted for kubectl parity")
    p.add_argument("--timeout", type=float, default=300.0)
    p.add_argument("command", nargs="*", help="after --: the container's command")
    p = sub.add_parser("events")
    p.add_argument("-A", "--all-namespaces", action="store_true")
    p = sub.add_parser("devices")
    p.add_argument("node")
    p.add_argument("-o", "--output", default="")
    p = sub.add_parser("top", help="GPU utilisation per pool (or per GPU) from the node agents")
    p.add_argument("what", nargs="?", default="pools", choices=["pools", "gpus", "pods"])
    p = sub.add_parser("gpu", help="per-GPU maintenance: cordon | uncordon")
    p.add_argument("action", choices=["cordon", "uncordon"])
    p.add_argument("node")
    p.add_argument("gpu", help="uuid, hipUUID or index on the node")
    p.add_argument("--reason", default="")
    p = sub.add_parser("install")
    p.add_argument("--crd-dir", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.dirname(os.path.abspath(__file__)))), "config", "crd"))
    p = sub.add_parser("trainjob", help="GoHai-style train jobs (Mi355xJob)")
    tsub = p.add_subparsers(dest="tj_cmd", required=True)
    t = tsub.add_parser("template", help="print a train-job template (or export one from a job)")
    t.add_argument("-s", "--source", default=None, help="existing Mi355xJob to export")
    t = tsub.add_parser("create")
    t.add_argument("-f", "--filename", required=True)
    t.add_argument("--dry-run", action="store_true", help="print the generated Mi355xJob")
    t.add_argument("--bare", action="store_true", help="the file is a full Mi355xJob manifest")
    t.add_argument("-o", "--output", default=None)
    tsub.add_parser("list")
    t = tsub.add_parser("logs")
    t.add_argument("job")
    t.add_argument("--rank", type=int, default=None)
    t = tsub.add_parser("delete")
    t.add_argument("job")
    for verb in ("suspend", "resume"):
        t = tsub.add_parser(verb, help=f"{verb} a job (spec.suspend): GPUs freed / re-queued")
        t.add_argument("job")
    p = sub.add_parser("convert", help="Volcano Job / Kubeflow PyTorchJob -> Mi355xJob")
    p.add_argument("-f", "--filename", required=True)
    p.add_argument("--pool", default=None, help="spec.poolRef of the converted job")
    p.add_argument("--resource", default=None, help="spec.resourceName (default: the pool's)")
    p.add_argument("--image", default=None, help="replace the containers' image (e.g. a ROCm one)")
    p.add_argument("-o", "--output", default="yaml", choices=["yaml", "json"])
    p = sub.add_parser("render")
    p.add_argument("what", choices=["job"])
    p.add_argument("-f", "--filename", required=True)
    p.add_argument("-o", "--output", default=None)
    p = sub.add_parser("config")
    csub = p.add_subparsers(dest="config_cmd", required=True)
    csub.add_parser("view")
    sc = csub.add_parser("set-context")
    sc.add_argument("name")
    sc.add_argument("--server", dest="server", default=None)
    sc.add_argument("--namespace", dest="namespace", default=None)
    sc.add_argument("--token", dest="token", default=None)
    uc = csub.add_parser("use-context")
    uc.add_argument("name")
    csub.add_parser("get-contexts")
    p = sub.add_parser("login", help="store a bearer token in a context (reads stdin without --token-value)")
    p.add_argument("--token-value", default=None)
    p.add_argument("--context-name", default=None)
    sub.add_parser("whoami")
    return ap


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    command: list[str] = []
    if "run" in argv and "--" in argv[argv.index("run"):]:  # `run NAME ... -- CMD ARGS...`
        i = argv.index("--", argv.index("run"))
        argv, command = argv[:i], argv[i + 1:]
    args = build_parser().parse_args(argv)
    if args.cmd == "run":
        args.command = command + list(args.command or [])
    if args.cmd == "config":
        return cmd_config(args)
    if args.cmd == "login":
        return cmd_login(args)
    if args.cmd == "convert":
        return cmd_convert(args)
    c, ns = connection(args)
    fn = {"apply": cmd_apply, "diff": cmd_diff, "get": cmd_get, "describe": cmd_describe,
          "delete": cmd_delete,
          "scale": cmd_scale, "wait": cmd_wait, "logs": cmd_logs, "events": cmd_events,
          "create": cmd_create, "run": cmd_run, "keys": cmd_keys,
          "devices": cmd_devices, "install": cmd_install, "render": cmd_render,
          "gpu": cmd_gpu, "trainjob": cmd_trainjob, "whoami": cmd_whoami, "top": cmd_top}[args.cmd]
    try:
        return fn(c, ns, args)
    except KubeError as e:
        print(f"Error from server ({e.reason or e.code}): {e}", file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
