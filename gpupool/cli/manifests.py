"""``gpuctl apply`` and ``gpuctl diff``: kubectl apply semantics (three-way with the last applied
configuration, or server-side apply) and a server-side dry run of it."""
from __future__ import annotations

import json
import sys

import yaml

from ..kube import Client, KubeError, res_for
from .common import dump, load_docs


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
