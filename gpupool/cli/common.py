"""gpuctl plumbing: connection (flags, kubeconfig, gpuctl contexts), resource discovery, manifest
loading and kubectl-style printing."""
from __future__ import annotations

import glob
import json
import os
import sys
from typing import Any

import yaml

from ..kube import Client, Res


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
