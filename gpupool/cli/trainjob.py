"""GoHai-style train jobs: ``trainjob`` (template/create/list/logs/delete), ``render job`` and
``convert`` (Volcano Job / PyTorchJob -> Mi355xJob)."""
from __future__ import annotations

import json
import re
import sys

import yaml

from ..api import schema
from ..kube import MI355XJOBS, PODS, Client
from .common import dump, load_docs, print_table
from .pods import pod_log


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
