"""Foreign training-job manifests -> Mi355xJob (``gpuctl convert``; ``gpuctl apply`` converts them
on the way in).

The reference platform submits training as a Volcano ``batch.volcano.sh/v1alpha1 Job``
(GPU调度平台搭建.md:643-672: minAvailable / queue / schedulerName volcano, one task asking for
``nvidia.com/gpu``, restartPolicy OnFailure) or, through the Kubeflow Training Operator it installs
(:300-306), a ``kubeflow.org/v1 PyTorchJob`` (Master + Worker replica specs; the operator sets the
``PET_*`` env the workload reads at :623). Both map onto one Mi355xJob: a gang of identical
workers, placed all-or-nothing (or elastically from ``minAvailable``) on pool GPUs, wired for
torchrun/RCCL by the job controller (which also writes the pod's GPU requests, so the source's GPU
limits become ``gpusPerReplica`` and its vendor resource name is dropped).

What has no Mi355xJob equivalent is reported, not silently dropped: ``convert`` returns the job and
a list of warnings (a CUDA image, a volume nothing mounts, tasks with different pod templates).
"""
from __future__ import annotations

import copy
import json
import re

from ..api import schema

VOLCANO = ("batch.volcano.sh", "Job")
PYTORCHJOB = ("kubeflow.org", "PyTorchJob")
GPU_RESOURCES = ("nvidia.com/gpu", "amd.com/gpu")
CONVERTED_FROM = "gpupool.amd.com/converted-from"


class ConvertError(ValueError):
    pass


def kind_of(doc: dict) -> tuple[str, str]:
    return str(doc.get("apiVersion", "")).split("/")[0], str(doc.get("kind", ""))


def convertible(doc: dict) -> bool:
    return kind_of(doc) in (VOLCANO, PYTORCHJOB)


def _gpus(template: dict, warnings: list[str]) -> int:
    """GPUs per pod from the containers' limits/requests of any GPU resource (summed over
    containers, as the kubelet would); the resource names are removed (the controller writes the
    pool's own)."""
    total = 0
    for c in ((template.get("spec") or {}).get("containers") or []):
        res = c.get("resources") or {}
        per = 0
        for sect in ("limits", "requests"):
            for name in GPU_RESOURCES + tuple(k for k in (res.get(sect) or {}) if k.endswith("/gpu")):
                v = (res.get(sect) or {}).pop(name, None)
                if v is not None:
                    per = max(per, int(str(v)))
            if sect in res and not res[sect]:
                del res[sect]
        if "resources" in c and not c["resources"]:
            del c["resources"]
        total += per
    return total


def _pod_key(template: dict) -> str:
    """What must agree between replica groups for them to be one gang of identical workers."""
    spec = copy.deepcopy(template.get("spec") or {})
    for c in spec.get("containers") or []:
        c.pop("name", None)
    spec.pop("restartPolicy", None)
    return json.dumps(spec, sort_keys=True)


def _check_image(template: dict, warnings: list[str], image: str | None) -> None:
    for c in ((template.get("spec") or {}).get("containers") or []):
        if image:
            c["image"] = image
        elif re.search(r"cuda|nvidia", str(c.get("image", "")), re.I):
            warnings.append(f"container {c.get('name')}: image {c.get('image')} is a CUDA image; "
                            f"it will not run on MI355X — pass --image (e.g. rocm/pytorch)")


def _restart(policy: str | None) -> str:
    return "Never" if policy == "Never" else "OnFailure"


def _finish(name: str, ns: str | None, src: str, spec: dict, warnings: list[str], pool: str | None,
            resource: str | None, labels: dict | None) -> tuple[dict, list[str]]:
    if pool:
        spec["poolRef"] = pool
    if resource:
        spec["resourceName"] = resource
    md = {"name": name, "annotations": {CONVERTED_FROM: src}}
    if ns:
        md["namespace"] = ns
    if labels:
        md["labels"] = dict(labels)
    return {"apiVersion": schema.API_VERSION, "kind": "Mi355xJob", "metadata": md,
            "spec": spec}, warnings


def from_volcano(doc: dict, pool: str | None = None, resource: str | None = None,
                 image: str | None = None) -> tuple[dict, list[str]]:
    """Volcano Job (GPU调度平台搭建.md:643-672) -> Mi355xJob."""
    warnings: list[str] = []
    md, spec = doc.get("metadata") or {}, doc.get("spec") or {}
    tasks = spec.get("tasks") or []
    if not tasks:
        raise ConvertError("Volcano Job has no spec.tasks")
    keys = {_pod_key(t.get("template") or {}) for t in tasks}
    if len(keys) > 1:
        raise ConvertError("Volcano Job tasks " + ", ".join(str(t.get("name")) for t in tasks) +
                           " have different pod templates: a Mi355xJob gang runs identical "
                           "workers — convert each task as its own job")
    replicas = sum(int(t.get("replicas", 1)) for t in tasks)
    tpl = copy.deepcopy(tasks[0].get("template") or {})
    tpl.setdefault("spec", {})
    gpus = _gpus(tpl, warnings)
    _check_image(tpl, warnings, image)
    restart = tpl["spec"].pop("restartPolicy", None)
    for pol in (spec.get("policies") or []) + [p for t in tasks for p in (t.get("policies") or [])]:
        if pol.get("action") in ("RestartJob", "RestartTask", "RestartPod"):
            restart = "OnFailure"
    out = {"replicas": replicas, "gpusPerReplica": gpus, "restartPolicy": _restart(restart),
           "template": tpl}
    if spec.get("minAvailable") is not None and int(spec["minAvailable"]) < replicas:
        out["minAvailable"] = max(1, int(spec["minAvailable"]))
    if spec.get("queue"):
        out["queue"] = spec["queue"]
    if spec.get("maxRetry") is not None:
        out["backoffLimit"] = int(spec["maxRetry"])
    if spec.get("ttlSecondsAfterFinished") is not None:
        out["ttlSecondsAfterFinished"] = int(spec["ttlSecondsAfterFinished"])
    if spec.get("schedulerName") not in (None, "volcano"):
        warnings.append(f"schedulerName {spec['schedulerName']} dropped: Mi355xJob gangs are placed "
                        f"by the gpupool job controller")
    if spec.get("priorityClassName"):
        warnings.append(f"priorityClassName {spec['priorityClassName']} not mapped: set "
                        f"spec.priority (integer) on the Mi355xJob")
    # Volcano job-level volumes: the Volcano form {mountPath, volumeClaimName} mounts in every
    # container; the plain pod-volume form (the reference's, :669-672) only declares the volume
    pod_spec = tpl["spec"]
    for i, v in enumerate(spec.get("volumes") or []):
        if "mountPath" in v:
            vname = v.get("name") or f"volcano-vol-{i}"
            claim = v.get("volumeClaimName") or (v.get("volumeClaim") or {}).get("claimName")
            if not claim:
                warnings.append(f"volume at {v['mountPath']}: only volumeClaimName is converted")
                continue
            pod_spec.setdefault("volumes", []).append(
                {"name": vname, "persistentVolumeClaim": {"claimName": claim}})
            for c in pod_spec.get("containers") or []:
                c.setdefault("volumeMounts", []).append({"name": vname, "mountPath": v["mountPath"]})
        else:
            pod_spec.setdefault("volumes", []).append(copy.deepcopy(v))
            mounted = any(m.get("name") == v.get("name") for c in pod_spec.get("containers") or []
                          for m in c.get("volumeMounts") or [])
            if not mounted:
                warnings.append(f"volume {v.get('name')} is declared but no container mounts it "
                                f"(as in the source manifest)")
    return _finish(md.get("name", "job"), md.get("namespace"), "batch.volcano.sh/v1alpha1/Job", out,
                   warnings, pool, resource, md.get("labels"))


def from_pytorchjob(doc: dict, pool: str | None = None, resource: str | None = None,
                    image: str | None = None) -> tuple[dict, list[str]]:
    """Kubeflow PyTorchJob (training-operator v1, GPU调度平台搭建.md:300-306) -> Mi355xJob. Master
    and Worker replicas become one gang (rank 0 = the master: the job controller points
    MASTER_ADDR at worker 0)."""
    warnings: list[str] = []
    md, spec = doc.get("metadata") or {}, doc.get("spec") or {}
    reps = spec.get("pytorchReplicaSpecs") or {}
    if not reps:
        raise ConvertError("PyTorchJob has no spec.pytorchReplicaSpecs")
    unknown = set(reps) - {"Master", "Worker"}
    if unknown:
        raise ConvertError(f"PyTorchJob replica types {sorted(unknown)} are not convertible")
    groups = [reps[k] for k in ("Master", "Worker") if k in reps]
    if len({_pod_key(g.get("template") or {}) for g in groups}) > 1:
        raise ConvertError("PyTorchJob Master and Worker pod templates differ: a Mi355xJob gang "
                           "runs identical workers")
    replicas = sum(int(g.get("replicas", 1)) for g in groups)
    tpl = copy.deepcopy(groups[0].get("template") or {})
    tpl.setdefault("spec", {})
    gpus = _gpus(tpl, warnings)
    _check_image(tpl, warnings, image)
    tpl["spec"].pop("restartPolicy", None)
    restart = groups[-1].get("restartPolicy")
    if restart in ("ExitCode", "Always"):
        warnings.append(f"restartPolicy {restart} mapped to OnFailure (the whole gang restarts)")
    run = spec.get("runPolicy") or {}
    sched = run.get("schedulingPolicy") or {}
    elastic = spec.get("elasticPolicy") or {}
    if not gpus and elastic.get("nProcPerNode"):
        gpus = int(elastic["nProcPerNode"])
    out = {"replicas": replicas, "gpusPerReplica": gpus, "restartPolicy": _restart(restart),
           "template": tpl}
    min_av = sched.get("minAvailable", elastic.get("minReplicas"))
    if min_av is not None and int(min_av) < replicas:
        out["minAvailable"] = max(1, int(min_av))
    if sched.get("queue"):
        out["queue"] = sched["queue"]
    for src_key, dst in (("backoffLimit", "backoffLimit"),
                         ("activeDeadlineSeconds", "activeDeadlineSeconds"),
                         ("ttlSecondsAfterFinished", "ttlSecondsAfterFinished")):
        if run.get(src_key) is not None:
            out[dst] = int(run[src_key])
    if run.get("cleanPodPolicy") in ("Running", "All", "None"):
        out["cleanPodPolicy"] = run["cleanPodPolicy"]
    if sched.get("priorityClass"):
        warnings.append(f"priorityClass {sched['priorityClass']} not mapped: set spec.priority")
    if "Master" not in reps:
        warnings.append("no Master replica: worker 0 is rank 0 (MASTER_ADDR)")
    return _finish(md.get("name", "job"), md.get("namespace"), "kubeflow.org/v1/PyTorchJob", out,
                   warnings, pool, resource, md.get("labels"))


def convert(doc: dict, pool: str | None = None, resource: str | None = None,
            image: str | None = None) -> tuple[dict, list[str]]:
    k = kind_of(doc)
    if k == VOLCANO:
        return from_volcano(doc, pool, resource, image)
    if k == PYTORCHJOB:
        return from_pytorchjob(doc, pool, resource, image)
    raise ConvertError(f"no conversion for {doc.get('apiVersion')} {doc.get('kind')}")
