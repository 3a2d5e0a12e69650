"""In-memory object store with kube-apiserver semantics (the envtest stand-in).

Semantics implemented here (all exercised by tests/unit/test_apiserver_store.py):

* one global, strictly increasing ``resourceVersion``; every write gets a fresh one;
* optimistic concurrency: an update carrying a stale ``metadata.resourceVersion`` -> 409 Conflict;
* ``metadata.generation`` starts at 1 and bumps only when the *spec* (anything outside
  ``metadata``/``status``) changes, or when ``deletionTimestamp`` is first set;
* status subresource isolation: main-resource writes ignore ``status``; ``/status`` writes
  ignore everything except ``status`` (README.md:131 ``+kubebuilder:subresource:status``);
* finalizers + ``deletionTimestamp`` two-phase delete; the object disappears (DELETED event)
  when the last finalizer is removed; new finalizers may not be added once deleting;
* graceful pod deletion: a bound pod gets ``deletionTimestamp`` and stays until the kubelet
  deletes it with grace 0; eviction subresource = graceful delete;
* CRD registration with structural-schema defaulting, pruning and validation;
* ownerReference garbage collection (background propagation);
* an event log with a compaction window: watching from a compacted RV -> 410 Gone.
"""
from __future__ import annotations

import base64
import collections
import datetime as _dt
import json
import re
import uuid as _uuid
from dataclasses import dataclass, field
from typing import Any, Callable

from ..api import openapi
from . import ssa
from ..api.smp import PatchError, strategic_merge


def clone(o):
    """Copy of a JSON-shaped value (dict / list / scalars): what the store hands out and keeps.
    5x faster than copy.deepcopy (no memo table), which was the simulator's largest CPU cost."""
    if isinstance(o, dict):
        return {k: clone(v) for k, v in o.items()}
    if isinstance(o, list):
        return [clone(v) for v in o]
    return o


class ApiError(Exception):
    def __init__(self, code: int, reason: str, message: str, details: dict | None = None):
        super().__init__(message)
        self.code = code
        self.reason = reason
        self.message = message
        self.details = details or {}

    def status(self) -> dict:
        return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
                "message": self.message, "reason": self.reason, "details": self.details,
                "code": self.code}


def now_rfc3339() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


_DNS1123_SUB = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$")


@dataclass
class ResourceType:
    group: str
    version: str
    plural: str
    kind: str
    namespaced: bool
    singular: str = ""
    short_names: list = field(default_factory=list)
    schema: dict | None = None          # openAPIV3Schema for CRs
    status_sub: bool = False
    scale_sub: dict | None = None
    printer_columns: list = field(default_factory=list)
    custom: bool = False                # served from a CRD (no strategic merge patch)

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    @property
    def key(self) -> tuple[str, str]:
        return (self.group, self.plural)


BUILTINS = [
    ResourceType("", "v1", "namespaces", "Namespace", False, "namespace", ["ns"]),
    ResourceType("", "v1", "nodes", "Node", False, "node", ["no"], status_sub=True),
    ResourceType("", "v1", "pods", "Pod", True, "pod", ["po"], status_sub=True),
    ResourceType("", "v1", "events", "Event", True, "event", ["ev"]),
    ResourceType("", "v1", "secrets", "Secret", True, "secret"),
    ResourceType("", "v1", "configmaps", "ConfigMap", True, "configmap", ["cm"]),
    ResourceType("", "v1", "resourcequotas", "ResourceQuota", True, "resourcequota", ["quota"],
                 status_sub=True),
    ResourceType("", "v1", "limitranges", "LimitRange", True, "limitrange", ["limits"]),
    ResourceType("coordination.k8s.io", "v1", "leases", "Lease", True, "lease"),
    ResourceType("policy", "v1", "poddisruptionbudgets", "PodDisruptionBudget", True,
                 "poddisruptionbudget", ["pdb"], status_sub=True),
    # stored-only kinds (no controllers behind them): lets `make deploy` manifests be applied
    # and validated against the simulator
    ResourceType("", "v1", "serviceaccounts", "ServiceAccount", True, "serviceaccount", ["sa"]),
    ResourceType("", "v1", "services", "Service", True, "service", ["svc"], status_sub=True),
    ResourceType("apps", "v1", "deployments", "Deployment", True, "deployment", ["deploy"],
                 status_sub=True),
    ResourceType("apps", "v1", "daemonsets", "DaemonSet", True, "daemonset", ["ds"],
                 status_sub=True),
    ResourceType("networking.k8s.io", "v1", "networkpolicies", "NetworkPolicy", True,
                 "networkpolicy", ["netpol"]),
    ResourceType("", "v1", "persistentvolumes", "PersistentVolume", False, "persistentvolume",
                 ["pv"], status_sub=True),
    ResourceType("", "v1", "persistentvolumeclaims", "PersistentVolumeClaim", True,
                 "persistentvolumeclaim", ["pvc"], status_sub=True),
    ResourceType("rbac.authorization.k8s.io", "v1", "clusterroles", "ClusterRole", False,
                 "clusterrole"),
    ResourceType("rbac.authorization.k8s.io", "v1", "clusterrolebindings", "ClusterRoleBinding",
                 False, "clusterrolebinding"),
    ResourceType("admissionregistration.k8s.io", "v1", "validatingadmissionpolicies",
                 "ValidatingAdmissionPolicy", False, "validatingadmissionpolicy", status_sub=True),
    ResourceType("admissionregistration.k8s.io", "v1", "validatingadmissionpolicybindings",
                 "ValidatingAdmissionPolicyBinding", False, "validatingadmissionpolicybinding"),
    ResourceType("apiextensions.k8s.io", "v1", "customresourcedefinitions",
                 "CustomResourceDefinition", False, "customresourcedefinition", ["crd", "crds"]),
]


@dataclass
class WatchEvent:
    rv: int
    rtype: tuple[str, str]
    type: str
    _obj: dict | None
    line: bytes | None = None  # the encoded watch line, built once and shared by every watcher
    # MODIFIED: the object before the write (a filtered watch turns a write that moves an object
    # out of / into its selection into DELETED / ADDED, as the apiserver's watch cache does)
    prev: dict | None = None

    @property
    def obj(self) -> dict:
        if self._obj is None:  # compacted: decoded on demand (a watch resuming from far back)
            return json.loads(self.line)["object"]
        return self._obj

    def encoded(self) -> bytes:
        if self.line is None:
            self.line = (json.dumps({"type": self.type, "object": self._obj}) + "\n").encode()
        return self.line

    def compact(self) -> None:
        """Keep only the encoded line: an old event in the log is no tree of Python objects for
        the garbage collector to walk (a full collection over the whole 50 000-event window
        stalled the event loop for ~20 ms)."""
        if self._obj is not None:
            self.encoded()
            self._obj = None
            self.prev = None


def _spec_part(obj: dict) -> dict:
    return {k: v for k, v in obj.items() if k not in ("metadata", "status", "apiVersion", "kind")}


# ------------------------------------------------------------------ selectors
def parse_label_selector(sel: str | None) -> Callable[[dict], bool]:
    if not sel:
        return lambda labels: True
    reqs = []
    # split on commas not inside parentheses
    parts, depth, cur = [], 0, ""
    for ch in sel:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    parts.append(cur)
    for p in (x.strip() for x in parts if x.strip()):
        m = re.match(r"^([^\s!=]+)\s+(in|notin)\s+\((.*)\)$", p)
        if m:
            key, op, vals = m.group(1), m.group(2), {v.strip() for v in m.group(3).split(",")}
            if op == "in":
                reqs.append(lambda l, k=key, vs=vals: l.get(k) in vs)
            else:
                reqs.append(lambda l, k=key, vs=vals: l.get(k) not in vs)
        elif "!=" in p:
            k, v = p.split("!=", 1)
            reqs.append(lambda l, k=k.strip(), v=v.strip(): l.get(k) != v)
        elif "==" in p or "=" in p:
            k, v = re.split(r"==?", p, maxsplit=1)
            reqs.append(lambda l, k=k.strip(), v=v.strip(): l.get(k) == v)
        elif p.startswith("!"):
            reqs.append(lambda l, k=p[1:].strip(): k not in l)
        else:
            reqs.append(lambda l, k=p: k in l)
    return lambda labels: all(r(labels or {}) for r in reqs)


def get_path(obj: Any, dotted: str) -> Any:
    cur = obj
    for part in dotted.split("."):
        if not part:
            continue
        if isinstance(cur, dict):
            cur = cur.get(part)
        else:
            return None
    return cur


def parse_field_selector(sel: str | None) -> Callable[[dict], bool]:
    if not sel:
        return lambda obj: True
    reqs = []
    for p in (x.strip() for x in sel.split(",") if x.strip()):
        if "!=" in p:
            k, v = p.split("!=", 1)
            reqs.append(lambda o, k=k.strip(), v=v.strip(): str(get_path(o, k) or "") != v)
        else:
            k, v = re.split(r"==?", p, maxsplit=1)
            reqs.append(lambda o, k=k.strip(), v=v.strip(): str(get_path(o, k) or "") == v)
    return lambda obj: all(r(obj) for r in reqs)


# ------------------------------------------------------------------ quantities
_QSUFFIX = {"m": 1e-3, "k": 1e3, "M": 1e6, "G": 1e9, "T": 1e12, "Ki": 1024, "Mi": 1024 ** 2,
            "Gi": 1024 ** 3, "Ti": 1024 ** 4}


def parse_quantity(v: Any) -> float:
    """A Kubernetes resource.Quantity (``2``, ``"500m"``, ``"16Gi"``) as a number."""
    if isinstance(v, (int, float)):
        return float(v)
    m = re.match(r"^\s*([0-9.]+)\s*([a-zA-Z]*)\s*$", str(v))
    if not m or (m.group(2) and m.group(2) not in _QSUFFIX):
        raise ApiError(422, "Invalid", f"quantities must match the regular expression: {v!r}")
    return float(m.group(1)) * _QSUFFIX.get(m.group(2), 1.0)


def _fmt_q(x: float) -> str:
    return str(int(x)) if float(x).is_integer() else str(x)


def _extended(name: str) -> bool:
    """Extended resources (``amd.com/gpu``): requests must equal limits, default to them."""
    return "/" in name and not name.startswith("kubernetes.io/")


def pod_usage(pod: dict) -> dict[str, float]:
    """ResourceQuota usage of one pod: ``pods`` and ``requests.<r>`` / ``limits.<r>`` per
    resource (an extended resource's request is its limit), plus the bare ``<r>`` alias quota
    accepts for extended resources."""
    use: dict[str, float] = {"pods": 1.0}
    for c in (pod.get("spec") or {}).get("containers") or []:
        res = c.get("resources") or {}
        lim, req = res.get("limits") or {}, dict(res.get("requests") or {})
        for k, v in lim.items():
            if _extended(k):
                req.setdefault(k, v)
        for k, v in req.items():
            use[f"requests.{k}"] = use.get(f"requests.{k}", 0.0) + parse_quantity(v)
            if _extended(k):
                use[k] = use.get(k, 0.0) + parse_quantity(v)
        for k, v in lim.items():
            use[f"limits.{k}"] = use.get(f"limits.{k}", 0.0) + parse_quantity(v)
    return use


# ------------------------------------------------------------------ patches
def merge_patch(target: Any, patch: Any) -> Any:
    """RFC 7386 JSON merge patch (the target is copied once, then patched in place)."""
    if not isinstance(patch, dict):
        return clone(patch)
    out = clone(target) if isinstance(target, dict) else {}
    _merge_into(out, patch)
    return out


def _merge_into(out: dict, patch: dict) -> None:
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        elif isinstance(v, dict):
            sub = out.get(k)
            if not isinstance(sub, dict):
                sub = out[k] = {}
            _merge_into(sub, v)
        else:
            out[k] = clone(v)


def _ptr_parts(path: str) -> list[str]:
    if path == "":
        return []
    return [p.replace("~1", "/").replace("~0", "~") for p in path.lstrip("/").split("/")]


def json_patch(target: Any, ops: list[dict]) -> Any:
    """RFC 6902 JSON patch (add/remove/replace/test/copy/move)."""
    doc = clone(target)

    def resolve(parts):
        cur = doc
        for p in parts[:-1]:
            cur = cur[int(p)] if isinstance(cur, list) else cur[p]
        return cur, parts[-1]

    for op in ops:
        kind, parts = op.get("op"), _ptr_parts(op.get("path", ""))
        try:
            if kind == "test":
                cur = doc
                for p in parts:
                    cur = cur[int(p)] if isinstance(cur, list) else cur[p]
                if cur != op.get("value"):
                    raise ApiError(422, "Invalid", f"test operation failed at {op['path']}")
                continue
            if kind in ("copy", "move"):
                src = _ptr_parts(op["from"])
                cur = doc
                for p in src:
                    cur = cur[int(p)] if isinstance(cur, list) else cur[p]
                val = clone(cur)
                if kind == "move":
                    parent, last = resolve(src)
                    if isinstance(parent, list):
                        parent.pop(int(last))
                    else:
                        del parent[last]
                kind, op = "add", {"value": val}
            parent, last = resolve(parts)
            if kind == "add":
                if isinstance(parent, list):
                    parent.insert(len(parent) if last == "-" else int(last), op["value"])
                else:
                    parent[last] = op["value"]
            elif kind == "replace":
                if isinstance(parent, list):
                    parent[int(last)] = op["value"]
                else:
                    if last not in parent:
                        raise KeyError(last)
                    parent[last] = op["value"]
            elif kind == "remove":
                if isinstance(parent, list):
                    parent.pop(int(last))
                else:
                    del parent[last]
            else:
                raise ApiError(422, "Invalid", f"unsupported patch op {kind!r}")
        except (KeyError, IndexError, ValueError, TypeError) as e:
            raise ApiError(422, "Invalid", f"json patch failed at {op.get('path')}: {e}") from e
    return doc


# ------------------------------------------------------------------ store
class Store:
    LIVE_EVENTS = 512  # newest watch events kept as objects; older ones only as encoded lines

    def __init__(self, window: int = 50000):
        self.rv = 0
        self.types: dict[tuple[str, str], ResourceType] = {}
        self.objects: dict[tuple[str, str], dict[tuple[str, str], dict]] = {}
        self.log: collections.deque[WatchEvent] = collections.deque(maxlen=window)
        self.listeners: list[Callable[[WatchEvent], None]] = []
        self._vschema: dict[tuple[str, str], tuple[dict, dict]] = {}  # CRD -> (schema, w/o metadata)
        self._list_keys: dict[tuple[str, str], tuple[Any, dict]] = {}  # type -> (schema, keys)
        for rt in BUILTINS:
            self.register(rt)
        self._ensure_namespace("default")

    # --------------------------------------------------------- registry
    def register(self, rt: ResourceType) -> None:
        self.types[rt.key] = rt
        self.objects.setdefault(rt.key, {})

    def unregister(self, key: tuple[str, str]) -> None:
        self.types.pop(key, None)
        self.objects.pop(key, None)

    def lookup(self, group: str, plural: str) -> ResourceType:
        rt = self.types.get((group, plural))
        if rt is None:
            raise ApiError(404, "NotFound", f"the server could not find the requested resource "
                           f"({group or 'core'}/{plural})")
        return rt

    def resolve_name(self, name: str) -> ResourceType | None:
        """kubectl-style resolution of plural/singular/kind/shortname (case-insensitive)."""
        n = name.lower()
        for rt in self.types.values():
            if n in (rt.plural, rt.singular, rt.kind.lower()) or n in rt.short_names \
                    or n == f"{rt.plural}.{rt.group}":
                return rt
        return None

    @property
    def compacted_rv(self) -> int:
        if len(self.log) < (self.log.maxlen or 0):
            return 0
        return self.log[0].rv - 1

    # --------------------------------------------------------- internals
    def _next_rv(self) -> int:
        self.rv += 1
        return self.rv

    def _emit(self, rt: ResourceType, etype: str, obj: dict, prev: dict | None = None) -> None:
        ev = WatchEvent(int(obj["metadata"]["resourceVersion"]), rt.key, etype, clone(obj),
                        prev=prev)
        self.log.append(ev)
        if len(self.log) > self.LIVE_EVENTS:  # older events: encoded bytes only
            self.log[-self.LIVE_EVENTS - 1].compact()
        for fn in list(self.listeners):
            fn(ev)
        if rt.kind == "Pod" or (rt.kind == "ResourceQuota" and etype != "DELETED"):
            self._refresh_quota_status(obj["metadata"].get("namespace", ""))

    def _ensure_namespace(self, ns: str) -> None:
        nss = self.objects[("", "namespaces")]
        if ("", ns) in nss:
            return
        rt = self.types[("", "namespaces")]
        obj = {"apiVersion": "v1", "kind": "Namespace",
               "metadata": {"name": ns}, "spec": {"finalizers": ["kubernetes"]},
               "status": {"phase": "Active"}}
        self._stamp_new(obj)
        nss[("", ns)] = obj
        self._emit(rt, "ADDED", obj)

    def _stamp_new(self, obj: dict) -> None:
        md = obj["metadata"]
        md["uid"] = str(_uuid.uuid4())
        md["creationTimestamp"] = now_rfc3339()
        md["resourceVersion"] = str(self._next_rv())
        md["generation"] = 1
        for k in ("deletionTimestamp", "deletionGracePeriodSeconds"):
            md.pop(k, None)

    def _admit_cr(self, rt: ResourceType, obj: dict, keep: str = "") -> dict:
        """Defaulting, pruning, validation for custom resources (+ secrets stringData). ``keep``:
        a top-level field taken unchanged from the stored object (status on a main-resource
        write, spec on a status write), admitted when it was written: not walked again."""
        if keep and keep in obj and rt.schema is not None and \
                keep not in (rt.schema.get("required") or []) and \
                "default" not in ((rt.schema.get("properties") or {}).get(keep) or {}):
            held = obj.pop(keep)
            obj = self._admit_cr(rt, obj)
            obj[keep] = held
            return obj
        if rt.kind == "Secret":
            sd = obj.pop("stringData", None) or {}
            data = obj.setdefault("data", {}) or {}
            for k, v in sd.items():
                data[k] = base64.b64encode(str(v).encode()).decode()
            obj["data"] = data
        if rt.schema is None:
            return obj
        obj = openapi.prune(obj, rt.schema)
        obj = openapi.apply_defaults(obj, rt.schema)
        vs = self._vschema.get(rt.key)
        if vs is None or vs[0] is not rt.schema:  # the schema minus metadata, built once per CRD
            vs = self._vschema[rt.key] = (rt.schema, {**rt.schema, "properties": {
                k: v for k, v in rt.schema.get("properties", {}).items() if k != "metadata"}})
        errs = openapi.validate({k: v for k, v in obj.items() if k != "metadata"}, vs[1])
        if errs:
            errs = [e.replace("<root>.", "") for e in errs]
            name = obj.get("metadata", {}).get("name", "")
            raise ApiError(422, "Invalid", f'{rt.kind}.{rt.group} "{name}" is invalid: '
                           + ", ".join(errs),
                           {"name": name, "kind": rt.plural,
                            "causes": [{"message": e} for e in errs]})
        return obj

    # --------------------------------------------------------- pod admission
    def _items(self, key: tuple[str, str], ns: str) -> list[dict]:
        return [o for (ons, _), o in sorted(self.objects.get(key, {}).items()) if ons == ns]

    def _admit_pod(self, ns: str, pod: dict) -> dict:
        """The LimitRanger and ResourceQuota admission plugins for pods (reference practice
        GPU调度平台搭建.md:802 "ResourceQuota + LimitRange"): LimitRange ``default`` /
        ``defaultRequest`` fill containers that name no value, ``max`` / ``min`` bound each
        container (type Container) or the pod's sum (type Pod); then every ResourceQuota of the
        namespace must still fit with this pod's usage added (403 Forbidden otherwise)."""
        name = pod["metadata"]["name"]
        containers = (pod.get("spec") or {}).get("containers") or []

        def forbid(msg: str) -> ApiError:
            return ApiError(403, "Forbidden", f'pods "{name}" is forbidden: {msg}',
                            {"name": name, "kind": "pods"})
        for lr in self._items(("", "limitranges"), ns):
            for lim in (lr.get("spec") or {}).get("limits") or []:
                typ = lim.get("type", "Container")
                if typ == "Container":
                    for c in containers:
                        res = c.setdefault("resources", {})
                        limits = res.setdefault("limits", {})
                        reqs = res.setdefault("requests", {})
                        for k, v in (lim.get("default") or {}).items():
                            limits.setdefault(k, v)
                        for k, v in (lim.get("defaultRequest") or {}).items():
                            reqs.setdefault(k, v)
                        for k, v in limits.items():
                            if _extended(k):
                                reqs.setdefault(k, v)
                        for k, v in (lim.get("max") or {}).items():
                            got = limits.get(k, reqs.get(k))
                            if got is not None and parse_quantity(got) > parse_quantity(v):
                                raise forbid(f"maximum {k} usage per Container is {v}, but limit "
                                             f"is {got}")
                        for k, v in (lim.get("min") or {}).items():
                            got = reqs.get(k, limits.get(k))
                            if got is None or parse_quantity(got) < parse_quantity(v):
                                raise forbid(f"minimum {k} usage per Container is {v}, but "
                                             f"request is {got if got is not None else 0}")
                elif typ == "Pod":
                    use = pod_usage(pod)
                    for k, v in (lim.get("max") or {}).items():
                        got = use.get(f"limits.{k}", use.get(f"requests.{k}", 0.0))
                        if got > parse_quantity(v):
                            raise forbid(f"maximum {k} usage per Pod is {v}, but limit is "
                                         f"{_fmt_q(got)}")
                    for k, v in (lim.get("min") or {}).items():
                        got = use.get(f"requests.{k}", 0.0)
                        if got < parse_quantity(v):
                            raise forbid(f"minimum {k} usage per Pod is {v}, but request is "
                                         f"{_fmt_q(got)}")
        new = pod_usage(pod)
        for q in self._items(("", "resourcequotas"), ns):
            hard = (q.get("spec") or {}).get("hard") or {}
            used = self._quota_used(ns, hard)
            over = [k for k in hard if new.get(k, 0.0) > 0 and
                    used.get(k, 0.0) + new[k] > parse_quantity(hard[k])]
            if over:
                qn = q["metadata"]["name"]
                raise forbid(f"exceeded quota: {qn}, requested: " +
                             ",".join(f"{k}={_fmt_q(new[k])}" for k in over) + ", used: " +
                             ",".join(f"{k}={_fmt_q(used.get(k, 0.0))}" for k in over) +
                             ", limited: " + ",".join(f"{k}={hard[k]}" for k in over))
        return pod

    def _quota_used(self, ns: str, hard: dict) -> dict[str, float]:
        used = {k: 0.0 for k in hard}
        for p in self._items(("", "pods"), ns):
            if (p.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
                continue  # terminal pods no longer count (quota controller semantics)
            for k, v in pod_usage(p).items():
                if k in used:
                    used[k] += v
        return used

    def _refresh_quota_status(self, ns: str) -> None:
        """ResourceQuota status.hard / status.used (the quota controller's job)."""
        rt = self.types[("", "resourcequotas")]
        for q in self._items(rt.key, ns):
            hard = (q.get("spec") or {}).get("hard") or {}
            try:
                st = {"hard": dict(hard),
                      "used": {k: _fmt_q(v) for k, v in self._quota_used(ns, hard).items()}}
            except ApiError:
                continue
            if q.get("status") != st:
                q["status"] = st
                q["metadata"]["resourceVersion"] = str(self._next_rv())
                self._emit(rt, "MODIFIED", q)

    def _check_ns(self, rt: ResourceType, ns: str | None) -> str:
        if rt.namespaced:
            if not ns:
                raise ApiError(400, "BadRequest", "namespace is required")
            return ns
        return ""

    # --------------------------------------------------------- reads
    def get(self, rt: ResourceType, ns: str | None, name: str) -> dict:
        ns = self._check_ns(rt, ns) if rt.namespaced else ""
        obj = self.objects[rt.key].get((ns, name))
        if obj is None:
            raise ApiError(404, "NotFound", f'{rt.plural}{"." + rt.group if rt.group else ""} '
                           f'"{name}" not found',
                           {"name": name, "group": rt.group, "kind": rt.plural})
        return clone(obj)

    def list(self, rt: ResourceType, ns: str | None, label_selector: str | None = None,
             field_selector: str | None = None, limit: int = 0, cont: str | None = None) -> dict:
        """A LIST; with ``limit``, one page of it. The continue token carries the first page's
        resourceVersion and the last key served: every page reports that resourceVersion (a
        watch resumes from it, as after a real paginated LIST) and only the page's objects are
        copied — an informer paging through 50 000 pods costs O(n), not O(n) per page."""
        lm = parse_label_selector(label_selector)
        fm = parse_field_selector(field_selector)
        objs = self.objects[rt.key]
        keys = sorted(k for k in objs if not rt.namespaced or not ns or k[0] == ns)
        rv0, start = str(self.rv), 0
        if cont:
            try:
                tok = json.loads(base64.urlsafe_b64decode(cont.encode()).decode())
                rv0, last = str(tok["rv"]), tuple(tok["key"])
            except (ValueError, KeyError, TypeError) as e:
                raise ApiError(400, "BadRequest", f"invalid continue token: {e}") from e
            import bisect
            start = bisect.bisect_right(keys, last)
        items, i = [], start
        while i < len(keys) and (not limit or len(items) < limit):
            o = objs[keys[i]]
            if lm(o["metadata"].get("labels")) and fm(o):
                items.append(clone(o))
            i += 1
        meta: dict[str, Any] = {"resourceVersion": rv0}
        if limit and i < len(keys):
            meta["continue"] = base64.urlsafe_b64encode(json.dumps(
                {"rv": rv0, "key": list(keys[i - 1])}).encode()).decode()
            meta["remainingItemCount"] = len(keys) - i  # an upper bound with selectors
        return {"kind": f"{rt.kind}List", "apiVersion": rt.api_version, "metadata": meta,
                "items": items}

    # --------------------------------------------------------- writes
    def create(self, rt: ResourceType, ns: str | None, obj: dict, dry_run: bool = False,
               managed: bool = False) -> dict:
        obj = clone(obj)
        ns = self._check_ns(rt, ns or obj.get("metadata", {}).get("namespace"))
        md = obj.setdefault("metadata", {})
        if not md.get("name"):
            gen = md.get("generateName")
            if not gen:
                raise ApiError(422, "Invalid", f"{rt.kind}: metadata.name: Required value")
            md["name"] = gen + _uuid.uuid4().hex[:5]
        name = md["name"]
        if len(name) > 253 or not _DNS1123_SUB.match(name):
            raise ApiError(422, "Invalid", f'{rt.kind} "{name}" is invalid: metadata.name: '
                           "Invalid value: must be a lowercase RFC 1123 subdomain")
        if md.get("namespace") and rt.namespaced and md["namespace"] != ns:
            raise ApiError(400, "BadRequest", "the namespace of the provided object does not "
                           "match the namespace sent on the request")
        if rt.namespaced:
            md["namespace"] = ns
        else:
            md.pop("namespace", None)
        obj["apiVersion"], obj["kind"] = rt.api_version, rt.kind
        if (ns, name) in self.objects[rt.key]:
            raise ApiError(409, "AlreadyExists", f'{rt.plural}{"." + rt.group if rt.group else ""}'
                           f' "{name}" already exists',
                           {"name": name, "group": rt.group, "kind": rt.plural})
        if not managed:
            md.pop("managedFields", None)  # only server-side apply records ownership (ssa.py)
        if rt.status_sub and rt.schema is not None:
            obj.pop("status", None)  # CR status is not settable on create
        obj = self._admit_cr(rt, obj)
        if rt.kind == "Pod":
            obj.setdefault("status", {}).setdefault("phase", "Pending")
            obj["spec"].setdefault("terminationGracePeriodSeconds", 30)
            obj = self._admit_pod(ns, obj)
        if dry_run:
            return obj
        if rt.namespaced:
            self._ensure_namespace(ns)
        self._stamp_new(obj)
        self.objects[rt.key][(ns, name)] = obj
        if rt.kind == "CustomResourceDefinition":
            self._register_crd(obj)
        self._emit(rt, "ADDED", obj)
        return clone(obj)

    def update(self, rt: ResourceType, ns: str | None, name: str, obj: dict,
               subresource: str = "", dry_run: bool = False, owned: bool = False,
               copy_out: bool = True, manager: str = "unknown", applied: bool = False) -> dict:
        """``owned``: ``obj`` is the caller's private copy (a freshly decoded request body, a
        patch result) and is stored as is. ``copy_out=False``: the stored object itself is
        returned, for a caller that only serialises it before yielding (the HTTP front-end):
        two full-object copies less per write, ~0.1 ms for an 8-GPU pool's status."""
        ns = self._check_ns(rt, ns) if rt.namespaced else ""
        cur = self.objects[rt.key].get((ns, name))
        if cur is None:
            raise ApiError(404, "NotFound", f'{rt.plural} "{name}" not found',
                           {"name": name, "kind": rt.plural})
        new = obj if owned else clone(obj)  # ``owned``: a private copy already (patch)
        nmd = new.setdefault("metadata", {})
        if nmd.get("name", name) != name:
            raise ApiError(400, "BadRequest", "the name of the object does not match the URL")
        rv = nmd.get("resourceVersion")
        if rv and rv != cur["metadata"]["resourceVersion"]:
            raise ApiError(409, "Conflict",
                           f'Operation cannot be fulfilled on {rt.plural}'
                           f'{"." + rt.group if rt.group else ""} "{name}": the object has been '
                           "modified; please apply your changes to the latest version and try "
                           "again", {"name": name, "group": rt.group, "kind": rt.plural})
        cmd = cur["metadata"]
        keep = ""
        if subresource == "status":
            merged = {k: clone(v) for k, v in cur.items() if k != "status"}  # status: replaced
            if "status" in new:
                merged["status"] = new["status"]
            else:
                merged.pop("status", None)
            if applied:  # the apply's own ownership record
                merged["metadata"]["managedFields"] = nmd.get("managedFields") or []
            new = merged
            keep = "spec"
        else:
            # immutable / server-owned metadata
            for k in ("uid", "creationTimestamp", "deletionTimestamp",
                      "deletionGracePeriodSeconds", "generation", "namespace"):
                if k in cmd:
                    nmd[k] = cmd[k]
                else:
                    nmd.pop(k, None)
            nmd["name"] = name
            if rt.status_sub:
                if "status" in cur:
                    if not (owned and new.get("status") == cur["status"]):  # a patch's own copy
                        new["status"] = clone(cur["status"])
                    keep = "status"
                else:
                    new.pop("status", None)
            if cmd.get("deletionTimestamp"):
                added = set(nmd.get("finalizers") or []) - set(cmd.get("finalizers") or [])
                if added:
                    raise ApiError(422, "Forbidden", f"no new finalizers can be added if the "
                                   f"object is being deleted, found new finalizers {sorted(added)}")
        new["apiVersion"], new["kind"] = rt.api_version, rt.kind
        new = self._admit_cr(rt, new, keep)
        new["metadata"]["resourceVersion"] = cmd["resourceVersion"]
        if not applied:  # field ownership of a non-apply write (objects someone applied)
            if cmd.get("managedFields"):
                ssa.record_update(cur, new, manager, self.list_keys(rt), rt.status_sub,
                                  subresource, rt.api_version, now_rfc3339())
            else:
                new["metadata"].pop("managedFields", None)
        if dry_run:
            return new
        if new == cur:  # no-op update: no new resourceVersion, no event (apiserver behaviour)
            return clone(cur) if copy_out else cur
        nmd = new["metadata"]
        if _spec_part(new) != _spec_part(cur):
            nmd["generation"] = int(cmd.get("generation", 1)) + 1
        else:
            nmd["generation"] = cmd.get("generation", 1)
        nmd["resourceVersion"] = str(self._next_rv())
        if nmd.get("deletionTimestamp") and not nmd.get("finalizers") and rt.kind != "Pod":
            self._remove(rt, ns, name, new)
            return clone(new) if copy_out else new
        self.objects[rt.key][(ns, name)] = new
        if rt.kind == "CustomResourceDefinition":
            self._register_crd(new)
        self._emit(rt, "MODIFIED", new, prev=cur)  # ``cur`` is replaced, never mutated
        return clone(new) if copy_out else new

    def list_keys(self, rt: ResourceType) -> dict:
        """List strategies for field ownership (ssa.list_keys), once per type and schema."""
        got = self._list_keys.get(rt.key)
        if got is None or got[0] is not rt.schema:
            got = self._list_keys[rt.key] = (rt.schema, ssa.list_keys(rt.kind, rt.schema))
        return got[1]

    def apply(self, rt: ResourceType, ns: str | None, name: str, cfg: Any, manager: str,
              force: bool = False, subresource: str = "", dry_run: bool = False) -> dict:
        """Server-side apply (ssa.py): creates the object when it does not exist."""
        if not manager:
            raise ApiError(400, "BadRequest", "PATCH requests with an apply patch require a "
                           "fieldManager query parameter")
        if not isinstance(cfg, dict):
            raise ApiError(400, "BadRequest", "an apply patch must be an object")
        if cfg.get("kind") and cfg["kind"] != rt.kind or \
                cfg.get("apiVersion") and cfg["apiVersion"] != rt.api_version:
            raise ApiError(400, "BadRequest", f"the apply patch is a {cfg.get('apiVersion')} "
                           f"{cfg.get('kind')}, the request is for {rt.api_version} {rt.kind}")
        md = cfg.get("metadata") or {}
        if md.get("name", name) != name:
            raise ApiError(400, "BadRequest", "the name of the object does not match the URL")
        nsk = self._check_ns(rt, ns) if rt.namespaced else ""
        cur = self.objects[rt.key].get((nsk, name))
        cfg = {**cfg, "metadata": {**md, "name": name}}
        try:
            new = ssa.apply(cur, cfg, manager, force, self.list_keys(rt), rt.status_sub,
                            subresource, rt.api_version, now_rfc3339())
        except ssa.Conflict as e:
            n = len(e.conflicts)
            raise ApiError(409, "Conflict", f"Apply failed with {n} conflict{'s' * (n > 1)}: " +
                           "; ".join(f'conflict with "{m}": .{f}' for m, f in e.conflicts),
                           {"name": name, "group": rt.group, "kind": rt.plural, "causes": [
                               {"reason": "FieldManagerConflict",
                                "message": f'conflict with "{m}"', "field": "." + f}
                               for m, f in e.conflicts]}) from e
        if cur is None:
            if subresource:
                self.get(rt, ns, name)  # raises the NotFound
            return self.create(rt, ns, new, dry_run, managed=True)
        new["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
        return self.update(rt, ns, name, new, subresource, dry_run, owned=True, applied=True)

    def patch(self, rt: ResourceType, ns: str | None, name: str, patch: Any, ptype: str,
              subresource: str = "", dry_run: bool = False, copy_out: bool = True,
              manager: str = "unknown", force: bool = False) -> dict:
        if ptype == "apply":
            return self.apply(rt, ns, name, patch, manager, force, subresource, dry_run)
        nsk = self._check_ns(rt, ns) if rt.namespaced else ""
        cur = self.objects[rt.key].get((nsk, name))
        if cur is None:
            self.get(rt, ns, name)  # raises the NotFound
        # both patch forms copy ``cur`` first: the stored object is never touched
        if ptype == "json":
            new = json_patch(cur, patch)
        elif ptype == "strategic":
            if rt.custom:  # apiserver: SMP needs Go struct tags, which a CRD does not have
                raise ApiError(415, "UnsupportedMediaType",
                               "strategic merge patch is not supported for custom resources; "
                               "use a JSON merge patch or a JSON patch")
            try:
                new = strategic_merge(cur, patch, rt.kind)
            except PatchError as e:
                raise ApiError(422, "Invalid", str(e)) from e
        else:
            new = merge_patch(cur, patch)
        if not (isinstance(patch, dict) and patch.get("metadata", {}).get("resourceVersion")):
            new.setdefault("metadata", {})["resourceVersion"] = cur["metadata"]["resourceVersion"]
        return self.update(rt, ns, name, new, subresource, dry_run, owned=True, copy_out=copy_out,
                           manager=manager)

    def delete(self, rt: ResourceType, ns: str | None, name: str, grace: int | None = None,
               preconditions: dict | None = None, dry_run: bool = False) -> dict:
        ns = self._check_ns(rt, ns) if rt.namespaced else ""
        cur = self.objects[rt.key].get((ns, name))
        if cur is None:
            raise ApiError(404, "NotFound", f'{rt.plural}{"." + rt.group if rt.group else ""} '
                           f'"{name}" not found', {"name": name, "kind": rt.plural})
        md = cur["metadata"]
        pre = preconditions or {}
        if pre.get("uid") and pre["uid"] != md["uid"]:
            raise ApiError(409, "Conflict", "Precondition failed: UID in precondition: "
                           f"{pre['uid']}, UID in object meta: {md['uid']}")
        if pre.get("resourceVersion") and pre["resourceVersion"] != md["resourceVersion"]:
            raise ApiError(409, "Conflict", "Precondition failed: resourceVersion mismatch")
        if dry_run:
            return clone(cur)
        graceful = False
        if rt.kind == "Pod" and cur.get("spec", {}).get("nodeName") \
                and cur.get("status", {}).get("phase") not in ("Succeeded", "Failed"):
            g = grace if grace is not None else cur["spec"].get("terminationGracePeriodSeconds", 30)
            graceful = g > 0
            if graceful:
                md["deletionGracePeriodSeconds"] = int(g)
        if graceful or md.get("finalizers"):
            if not md.get("deletionTimestamp"):
                md["deletionTimestamp"] = now_rfc3339()
                md["generation"] = int(md.get("generation", 1)) + 1
                md["resourceVersion"] = str(self._next_rv())
                self._emit(rt, "MODIFIED", cur)
            elif rt.kind == "Pod" and grace == 0 and not md.get("finalizers"):
                self._remove(rt, ns, name, cur)
            return clone(cur)
        self._remove(rt, ns, name, cur)
        return clone(cur)

    def _remove(self, rt: ResourceType, ns: str, name: str, obj: dict) -> None:
        self.objects[rt.key].pop((ns, name), None)
        obj["metadata"]["resourceVersion"] = str(self._next_rv())
        self._emit(rt, "DELETED", obj)
        if rt.kind == "CustomResourceDefinition":
            spec = obj["spec"]
            key = (spec["group"], spec["names"]["plural"])
            for (ons, oname), o in list(self.objects.get(key, {}).items()):
                self.objects[key].pop((ons, oname), None)
                o["metadata"]["resourceVersion"] = str(self._next_rv())
                self._emit(self.types[key], "DELETED", o)
            self.unregister(key)
        if rt.kind == "Namespace":
            for key, objs in list(self.objects.items()):
                t = self.types.get(key)
                if t and t.namespaced:
                    for (ons, oname) in [k for k in objs if k[0] == name]:
                        o = objs.pop((ons, oname))
                        o["metadata"]["resourceVersion"] = str(self._next_rv())
                        self._emit(t, "DELETED", o)
        self._gc(obj["metadata"]["uid"])

    def _gc(self, owner_uid: str) -> None:
        """Background-propagation garbage collection of dependents."""
        for key, objs in list(self.objects.items()):
            rt = self.types.get(key)
            if rt is None:
                continue
            for (ons, oname), o in list(objs.items()):
                refs = o["metadata"].get("ownerReferences") or []
                if any(r.get("uid") == owner_uid for r in refs):
                    remaining = [r for r in refs if r.get("uid") != owner_uid]
                    if remaining:
                        o["metadata"]["ownerReferences"] = remaining
                        o["metadata"]["resourceVersion"] = str(self._next_rv())
                        self._emit(rt, "MODIFIED", o)
                    else:
                        try:
                            self.delete(rt, ons or None, oname, grace=0)
                        except ApiError:
                            pass

    def _pdb_blocks(self, pod: dict) -> str | None:
        """Eviction API semantics: refuse (429) when evicting ``pod`` would take a matching
        PodDisruptionBudget below minAvailable / above maxUnavailable. Returns the PDB name."""
        ns = pod["metadata"].get("namespace")
        labels = pod["metadata"].get("labels") or {}
        pods_rt = self.types[("", "pods")]
        pdb_rt = self.types.get(("policy", "poddisruptionbudgets"))
        if pdb_rt is None:
            return None
        for pdb in self.list(pdb_rt, ns)["items"]:
            sel = ((pdb.get("spec") or {}).get("selector") or {}).get("matchLabels") or {}
            if not sel or any(labels.get(k) != v for k, v in sel.items()):
                continue
            matching = [p for p in self.list(pods_rt, ns)["items"]
                        if all((p["metadata"].get("labels") or {}).get(k) == v for k, v in sel.items())
                        and not p["metadata"].get("deletionTimestamp")]
            healthy = sum(1 for p in matching if (p.get("status") or {}).get("phase") == "Running")
            expected = len(matching)

            def resolve(v):
                if isinstance(v, str) and v.endswith("%"):
                    import math
                    return math.ceil(expected * int(v[:-1]) / 100)
                return int(v)
            spec = pdb.get("spec") or {}
            if "minAvailable" in spec and healthy - 1 < resolve(spec["minAvailable"]):
                return pdb["metadata"]["name"]
            if "maxUnavailable" in spec and expected - (healthy - 1) > resolve(spec["maxUnavailable"]):
                return pdb["metadata"]["name"]
        return None

    def evict(self, ns: str, name: str, body: dict | None) -> dict:
        rt = self.types[("", "pods")]
        pod = self.get(rt, ns, name)
        if not pod["metadata"].get("deletionTimestamp"):
            blocker = self._pdb_blocks(pod)
            if blocker:
                raise ApiError(429, "TooManyRequests",
                               "Cannot evict pod as it would violate the pod's disruption budget.",
                               details={"causes": [{"reason": "DisruptionBudget",
                                                    "message": f"The disruption budget {blocker} "
                                                               "needs more healthy pods"}]})
        opts = (body or {}).get("deleteOptions") or {}
        self.delete(rt, ns, name, grace=opts.get("gracePeriodSeconds"),
                    preconditions=opts.get("preconditions"))
        return {"kind": "Status", "apiVersion": "v1", "status": "Success", "code": 201,
                "metadata": {}}

    # --------------------------------------------------------- scale subresource
    def get_scale(self, rt: ResourceType, ns: str, name: str) -> dict:
        if not rt.scale_sub:
            raise ApiError(404, "NotFound", f"{rt.plural} has no scale subresource")
        obj = self.get(rt, ns, name)
        spec_path = rt.scale_sub.get("specReplicasPath", ".spec.replicas")
        st_path = rt.scale_sub.get("statusReplicasPath", ".status.replicas")
        return {"kind": "Scale", "apiVersion": "autoscaling/v1",
                "metadata": {"name": name, "namespace": ns, "uid": obj["metadata"]["uid"],
                             "resourceVersion": obj["metadata"]["resourceVersion"],
                             "creationTimestamp": obj["metadata"]["creationTimestamp"]},
                "spec": {"replicas": get_path(obj, spec_path) or 0},
                "status": {"replicas": get_path(obj, st_path) or 0}}

    def update_scale(self, rt: ResourceType, ns: str, name: str, scale: dict,
                     manager: str = "unknown") -> dict:
        obj = self.get(rt, ns, name)
        rv = scale.get("metadata", {}).get("resourceVersion")
        if rv and rv != obj["metadata"]["resourceVersion"]:
            raise ApiError(409, "Conflict", f'Operation cannot be fulfilled on {rt.plural} '
                           f'"{name}": the object has been modified')
        path = rt.scale_sub.get("specReplicasPath", ".spec.replicas").lstrip(".").split(".")
        cur = obj
        for p in path[:-1]:
            cur = cur.setdefault(p, {})
        cur[path[-1]] = int(scale.get("spec", {}).get("replicas", 0))
        self.update(rt, ns, name, obj, manager=manager)
        return self.get_scale(rt, ns, name)

    # --------------------------------------------------------- CRDs
    def _register_crd(self, crd: dict) -> None:
        spec = crd["spec"]
        ver = next((v for v in spec["versions"] if v.get("storage")), spec["versions"][0])
        subs = ver.get("subresources") or {}
        names = spec["names"]
        self.register(ResourceType(
            group=spec["group"], version=ver["name"], plural=names["plural"], kind=names["kind"],
            namespaced=spec.get("scope", "Namespaced") == "Namespaced",
            singular=names.get("singular", names["kind"].lower()),
            short_names=list(names.get("shortNames") or []),
            schema=(ver.get("schema") or {}).get("openAPIV3Schema"),
            status_sub="status" in subs, scale_sub=subs.get("scale"),
            printer_columns=list(ver.get("additionalPrinterColumns") or []), custom=True))
        crd.setdefault("status", {})["conditions"] = [
            {"type": "Established", "status": "True", "reason": "InitialNamesAccepted",
             "message": "the initial names have been accepted",
             "lastTransitionTime": now_rfc3339()}]
        crd["status"]["acceptedNames"] = names

    # --------------------------------------------------------- watch support
    def events_since(self, rt: ResourceType, rv: int) -> list[WatchEvent]:
        if rv < self.compacted_rv:
            raise ApiError(410, "Expired", f"too old resource version: {rv} "
                           f"({self.compacted_rv + 1})")
        # the log is in resourceVersion order: walk back from the newest event only as far as rv
        # (a resuming watch is usually a few events behind; scanning the whole 50 000-event window
        # per watch (re)connect cost ~0.4 ms on the event loop)
        out = []
        for e in reversed(self.log):
            if e.rv <= rv:
                break
            if e.rtype == rt.key:
                out.append(e)
        out.reverse()
        return out

