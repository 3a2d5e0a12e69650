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
import json
import os
import re
import sys
import time

import yaml

from ..api import schema
from ..kube import EVENTS, Client, KubeError, res_for
from .agents import (_agent, _agent_client, _agent_endpoint, _agent_token,  # noqa: F401
                     _SignedAgentClient, cmd_devices, cmd_gpu, cmd_top)
from .common import (CONFIG_PATH, USER_AGENT, connection, dump, load_config,  # noqa: F401
                     load_docs, print_table, resolve, save_config)
from .manifests import cmd_apply, cmd_diff
from .pods import cmd_create, cmd_events, cmd_logs, cmd_run, pod_log  # noqa: F401
from .trainjob import (SAMPLE_TRAINJOB, cmd_convert, cmd_render, cmd_trainjob,  # noqa: F401
                       job_to_template, render_job, render_trainjob)

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


def cmd_keys(c: Client, ns: str, args) -> int:
    from . import keys
    return keys.main(c, args)


def cmd_install(c: Client, ns: str, args) -> int:
    from ..kube import CRDS
    for doc in load_docs(args.crd_dir):
        action, _ = c.apply(doc)
        print(f"customresourcedefinition.apiextensions.k8s.io/{doc['metadata']['name']} {action}")
        c.wait_for(CRDS, doc["metadata"]["name"], None, lambda o: bool(o) and any(
            x["type"] == "Established" and x["status"] == "True"
            for x in (o.get("status") or {}).get("conditions", [])), timeout=30)
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
