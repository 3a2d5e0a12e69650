"""aiohttp front-end of the apiserver simulator: the k8s REST shape over HTTP/1.1 JSON.

Routes:
  /api, /api/v1, /apis, /apis/{g}/{v}                         discovery
  /api/v1/{plural}[/{name}[/{sub}]]                           cluster-scoped core
  /api/v1/namespaces/{ns}/{plural}[/{name}[/{sub}]]           namespaced core
  /apis/{g}/{v}/{plural}[/{name}[/{sub}]]                     cluster-scoped group
  /apis/{g}/{v}/namespaces/{ns}/{plural}[/{name}[/{sub}]]     namespaced group
  sub in {status, scale, eviction}
  ?watch=1&resourceVersion=&allowWatchBookmarks=&timeoutSeconds=   chunked watch stream
  Accept: application/json;as=Table                           server-side printing (kubectl get)
  /healthz /readyz /livez /version /metrics
"""
from __future__ import annotations

import asyncio
import datetime as _dt
import json
import logging
import os
import re
import time
from typing import Any

import yaml
from aiohttp import web

from .store import ApiError, ResourceType, Store, WatchEvent, get_path, parse_field_selector, \
    parse_label_selector

log = logging.getLogger("apiserver-sim")


# ------------------------------------------------------------------ printing (Table)
def _age(ts: str | None) -> str:
    if not ts:
        return "<unknown>"
    try:
        t = _dt.datetime.strptime(ts, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=_dt.timezone.utc)
    except ValueError:
        return "<invalid>"
    s = int((_dt.datetime.now(_dt.timezone.utc) - t).total_seconds())
    if s < 120:
        return f"{s}s"
    if s < 7200:
        return f"{s // 60}m"
    if s < 172800:
        return f"{s // 3600}h"
    return f"{s // 86400}d"


_FILTER = re.compile(r"^(.*?)\[\?\(@\.(\w+)==\"([^\"]*)\"\)\](.*)$")


def jsonpath(obj: Any, path: str) -> Any:
    """Subset of kubectl JSONPath: ``.a.b`` and ``.a[?(@.k=="v")].c``."""
    m = _FILTER.match(path)
    if m:
        lst = get_path(obj, m.group(1)) or []
        for x in lst:
            if isinstance(x, dict) and str(x.get(m.group(2))) == m.group(3):
                return get_path(x, m.group(4)) if m.group(4) else x
        return None
    return get_path(obj, path)


def _cell(v: Any, typ: str) -> Any:
    if typ == "date":
        return _age(v)
    if v is None:
        return "" if typ == "string" else None
    return v


def builtin_columns(rt: ResourceType) -> list[tuple[str, str, Any]]:
    if rt.kind == "Pod":
        def ready(o):
            cs = o.get("status", {}).get("containerStatuses") or []
            return f"{sum(1 for c in cs if c.get('ready'))}/{len(o.get('spec', {}).get('containers', []))}"

        def status(o):
            if o["metadata"].get("deletionTimestamp"):
                return "Terminating"
            return o.get("status", {}).get("phase", "")
        return [("Ready", "string", ready), ("Status", "string", status),
                ("Node", "string", lambda o: o.get("spec", {}).get("nodeName", "")),
                ("Age", "date", lambda o: o["metadata"].get("creationTimestamp"))]
    if rt.kind == "Node":
        def nstatus(o):
            for c in o.get("status", {}).get("conditions") or []:
                if c.get("type") == "Ready":
                    return "Ready" if c.get("status") == "True" else "NotReady"
            return "Unknown"

        def gpus(o):
            alloc = o.get("status", {}).get("allocatable") or {}
            return ",".join(f"{k}={v}" for k, v in sorted(alloc.items()) if k.startswith("amd.com/"))
        return [("Status", "string", nstatus), ("GPUs", "string", gpus),
                ("Age", "date", lambda o: o["metadata"].get("creationTimestamp"))]
    if rt.kind == "Event":
        return [("Type", "string", lambda o: o.get("type", "")),
                ("Reason", "string", lambda o: o.get("reason", "")),
                ("Object", "string", lambda o: "{}/{}".format(
                    (o.get("involvedObject") or {}).get("kind", "").lower(),
                    (o.get("involvedObject") or {}).get("name", ""))),
                ("Message", "string", lambda o: o.get("message", ""))]
    if rt.kind == "ResourceQuota":  # kubectl's columns: "<resource>: used/hard" per kind
        def usage(limits: bool):
            def f(o):
                hard = (o.get("status") or {}).get("hard") or (o.get("spec") or {}).get("hard") or {}
                used = (o.get("status") or {}).get("used") or {}
                return ", ".join(f"{k}: {used.get(k, '0')}/{v}" for k, v in sorted(hard.items())
                                 if k.startswith("limits.") == limits)
            return f
        return [("Age", "date", lambda o: o["metadata"].get("creationTimestamp")),
                ("Request", "string", usage(False)), ("Limit", "string", usage(True))]
    return [("Age", "date", lambda o: o["metadata"].get("creationTimestamp"))]


def to_table(rt: ResourceType, items: list[dict], rv: str) -> dict:
    cols = [{"name": "Name", "type": "string", "format": "name"}]
    getters = []
    if rt.printer_columns:
        for pc in rt.printer_columns:
            cols.append({"name": pc["name"], "type": pc.get("type", "string")})
            getters.append(lambda o, p=pc: _cell(jsonpath(o, p["jsonPath"]), p.get("type", "string")))
    else:
        for name, typ, fn in builtin_columns(rt):
            cols.append({"name": name, "type": "string" if typ == "date" else typ})
            getters.append(lambda o, f=fn, t=typ: _cell(f(o), t))
    rows = [{"cells": [o["metadata"]["name"]] + [g(o) for g in getters],
             "object": {"kind": "PartialObjectMetadata", "apiVersion": "meta.k8s.io/v1",
                        "metadata": o["metadata"]}} for o in items]
    return {"kind": "Table", "apiVersion": "meta.k8s.io/v1", "metadata": {"resourceVersion": rv},
            "columnDefinitions": cols, "rows": rows}


def agent_node_policy_violation(user: dict, old: dict, new: dict, own: list[str],
                                prefixes: list[str]) -> str:
    """The message of the first rule of schema.agent_node_policy that ``old -> new`` breaks, or
    "" when the agent's Node write is admissible."""
    claim = ((user.get("extra") or {}).get("authentication.kubernetes.io/node-name") or [""])[0]
    if claim != new["metadata"]["name"]:
        return "the gpupool agent may only write the Node it runs on"
    if new.get("spec") != old.get("spec"):
        return "the gpupool agent may not change Node spec"
    ost, nst = old.get("status") or {}, new.get("status") or {}
    others = [[c for c in (st.get("conditions") or []) if c.get("type") not in own]
              for st in (ost, nst)]
    if ost.get("capacity") != nst.get("capacity") or \
            ost.get("allocatable") != nst.get("allocatable") or others[0] != others[1]:
        return f"the gpupool agent may only write its own Node conditions ({', '.join(own)})"
    for f in ("labels", "annotations"):
        a, b = old["metadata"].get(f) or {}, new["metadata"].get(f) or {}
        mine = lambda k: any(k.startswith(p) for p in prefixes)  # noqa: E731
        if {k: v for k, v in a.items() if not mine(k)} != {k: v for k, v in b.items()
                                                            if not mine(k)}:
            return f"the gpupool agent may only write labels/annotations under {', '.join(prefixes)}"
    return ""


USER_KEY = web.RequestKey("user", dict) if hasattr(web, "RequestKey") else "user"


# ------------------------------------------------------------------ server
class ApiServerSim:
    def __init__(self, token: str | None = None, bookmark_interval: float = 5.0,
                 window: int = 50000, watch_delay: float = 0.0):
        self.store = Store(window=window)
        # a lagging watch cache (as a loaded kube-apiserver has): every watch event is delivered
        # ``watch_delay`` seconds after the write, so informers see stale objects meanwhile
        self.watch_delay = watch_delay
        self.token = token
        # bearer tokens beside the admin ``token``: token -> {"username", "groups", "extra",
        # "expiresAt" (unix s, optional)}. An expired token answers 401, as a bound ServiceAccount
        # token past its expiry does; POST /debug/tokens replaces the set (rotation tests)
        self.users: dict[str, dict] = {}
        self.auth_failures = 0
        self.bookmark_interval = bookmark_interval
        # watch queues per resource type (a kube-apiserver's watch cache is per resource too): a
        # write wakes only the watchers of its own type, not every informer of every kind
        self.watchers: dict[tuple[str, str], set[asyncio.Queue]] = {}
        self.store.listeners.append(self._fanout)
        self.requests_total: dict[tuple[str, int], int] = {}
        # LIST / WATCH requests per resource (what informers and uncached readers cost the server)
        self.lists: dict[str, int] = {}
        self.watches: dict[str, int] = {}
        # fault injection (tests): resource plural -> LIST/WATCH requests still to fail with 503
        # (-1: until cleared); set at start (--fail-list) or through POST /debug/faults
        self.fail_list: dict[str, int] = {}
        self.started = time.time()
        self.app = web.Application(middlewares=[self._mw], client_max_size=64 << 20)
        r = self.app.router
        r.add_get("/healthz", self._ok)
        r.add_get("/readyz", self._ok)
        r.add_get("/livez", self._ok)
        r.add_get("/version", self._version)
        r.add_get("/metrics", self._metrics)
        r.add_post("/debug/faults", self._set_faults)
        r.add_post("/debug/tokens", self._set_tokens)
        r.add_get("/api", self._api_versions)
        r.add_get("/apis", self._api_groups)
        r.add_get("/api/{version}", self._resource_list_core)
        r.add_get("/apis/{group}/{version}", self._resource_list_group)
        r.add_route("*", "/api/{version}/{rest:.*}", self._dispatch_core)
        r.add_route("*", "/apis/{group}/{version}/{rest:.*}", self._dispatch_group)

    # -------------------------------------------------------------- plumbing
    @web.middleware
    async def _mw(self, request: web.Request, handler):
        if (self.token or self.users) and request.path not in ("/healthz", "/readyz", "/livez"):
            user = self.authenticate(request.headers.get("Authorization", ""))
            if user is None:
                self.auth_failures += 1
                return self._err(ApiError(401, "Unauthorized", "Unauthorized"))
            request[USER_KEY] = user
        try:
            resp = await handler(request)
        except ApiError as e:
            resp = self._err(e)
        except web.HTTPException:
            raise
        except json.JSONDecodeError as e:
            resp = self._err(ApiError(400, "BadRequest", f"invalid JSON body: {e}"))
        except Exception as e:  # pragma: no cover - surfaced as 500
            log.exception("internal error")
            resp = self._err(ApiError(500, "InternalError", repr(e)))
        key = (request.method, resp.status)
        self.requests_total[key] = self.requests_total.get(key, 0) + 1
        return resp

    @staticmethod
    def _err(e: ApiError) -> web.Response:
        return web.json_response(e.status(), status=e.code)

    async def _ok(self, request):
        return web.Response(text="ok")

    async def _version(self, request):
        return web.json_response({"major": "1", "minor": "30", "gitVersion": "v1.30.0-gpupool-sim",
                                  "platform": "linux/amd64"})

    async def _metrics(self, request):
        lines = ["# TYPE apiserver_request_total counter"]
        for (m, c), n in sorted(self.requests_total.items()):
            lines.append(f'apiserver_request_total{{verb="{m}",code="{c}"}} {n}')
        lines.append("# TYPE apiserver_watchers gauge")
        lines.append(f"apiserver_watchers {sum(len(v) for v in self.watchers.values())}")
        lines.append(f"apiserver_authentication_failures_total {self.auth_failures}")
        for r, n in sorted(self.lists.items()):
            lines.append(f'apiserver_list_total{{resource="{r}"}} {n}')
        for r, n in sorted(self.watches.items()):
            lines.append(f'apiserver_watch_total{{resource="{r}"}} {n}')
        lines.append("# TYPE etcd_resource_version gauge")
        lines.append(f"etcd_resource_version {self.store.rv}")
        return web.Response(text="\n".join(lines) + "\n", content_type="text/plain")

    ADMIN = {"username": "system:admin", "groups": ["system:masters"], "extra": {}}

    def authenticate(self, header: str) -> dict | None:
        if not header.startswith("Bearer "):
            return None
        tok = header[7:].strip()
        if self.token and tok == self.token:
            return self.ADMIN
        u = self.users.get(tok)
        if u is None or (u.get("expiresAt") and time.time() >= float(u["expiresAt"])):
            return None
        return u

    async def _set_tokens(self, request):
        """{"tokens": {token: {"username", "groups", "extra", "expiresAt"}}, "merge": bool}."""
        if request.get(USER_KEY) not in (None, self.ADMIN):
            raise ApiError(403, "Forbidden", "debug endpoints are admin-only")
        body = await request.json()
        toks = {str(k): dict(v or {}) for k, v in (body.get("tokens") or {}).items()}
        self.users = {**self.users, **toks} if body.get("merge") else toks
        return web.json_response({"tokens": len(self.users)})

    async def _set_faults(self, request):
        """{"failList": {"resourcequotas": -1}}: LIST and WATCH of those resources answer 503
        (the count: how many more; -1 until cleared). {} clears."""
        body = await request.json()
        self.fail_list = {str(k): int(v) for k, v in (body.get("failList") or {}).items()}
        return web.json_response({"failList": self.fail_list})

    def _inject_list_fault(self, rt) -> None:
        n = self.fail_list.get(rt.plural)
        if n is None or n == 0:
            return
        if n > 0:
            self.fail_list[rt.plural] = n - 1
        raise ApiError(503, "ServiceUnavailable", f"injected: {rt.plural} cannot be listed")

    def _fanout(self, ev: WatchEvent) -> None:
        qs = self.watchers.get(ev.rtype)
        if qs:
            t = time.monotonic()
            for q in list(qs):
                q.put_nowait((t, ev))

    # -------------------------------------------------------------- discovery
    def _resources_for(self, group: str, version: str) -> list[dict]:
        out = []
        for rt in self.store.types.values():
            if rt.group != group or rt.version != version:
                continue
            verbs = ["create", "delete", "deletecollection", "get", "list", "patch", "update",
                     "watch"]
            out.append({"name": rt.plural, "singularName": rt.singular, "namespaced": rt.namespaced,
                        "kind": rt.kind, "verbs": verbs, "shortNames": rt.short_names})
            if rt.status_sub:
                out.append({"name": rt.plural + "/status", "namespaced": rt.namespaced,
                            "kind": rt.kind, "verbs": ["get", "patch", "update"]})
            if rt.scale_sub:
                out.append({"name": rt.plural + "/scale", "namespaced": rt.namespaced,
                            "kind": "Scale", "group": "autoscaling", "version": "v1",
                            "verbs": ["get", "patch", "update"]})
            if rt.kind == "Pod":
                out.append({"name": "pods/eviction", "namespaced": True, "kind": "Eviction",
                            "group": "policy", "version": "v1", "verbs": ["create"]})
        return out

    async def _api_versions(self, request):
        return web.json_response({"kind": "APIVersions", "versions": ["v1"]})

    async def _api_groups(self, request):
        groups = {}
        for rt in self.store.types.values():
            if rt.group:
                groups.setdefault(rt.group, set()).add(rt.version)
        return web.json_response({"kind": "APIGroupList", "apiVersion": "v1", "groups": [
            {"name": g, "versions": [{"groupVersion": f"{g}/{v}", "version": v} for v in sorted(vs)],
             "preferredVersion": {"groupVersion": f"{g}/{sorted(vs)[-1]}",
                                  "version": sorted(vs)[-1]}}
            for g, vs in sorted(groups.items())]})

    async def _resource_list_core(self, request):
        return web.json_response({"kind": "APIResourceList", "groupVersion": "v1",
                                  "resources": self._resources_for("", request.match_info["version"])})

    async def _resource_list_group(self, request):
        g, v = request.match_info["group"], request.match_info["version"]
        res = self._resources_for(g, v)
        if not res:
            raise ApiError(404, "NotFound", f"the server could not find {g}/{v}")
        return web.json_response({"kind": "APIResourceList", "groupVersion": f"{g}/{v}",
                                  "resources": res})

    # -------------------------------------------------------------- dispatch
    async def _dispatch_core(self, request):
        return await self._dispatch(request, "", request.match_info["version"],
                                    request.match_info["rest"])

    async def _dispatch_group(self, request):
        return await self._dispatch(request, request.match_info["group"],
                                    request.match_info["version"], request.match_info["rest"])

    async def _dispatch(self, request: web.Request, group: str, version: str, rest: str):
        parts = [p for p in rest.split("/") if p]
        ns = None
        # /namespaces/{ns}/{plural}/... vs /namespaces/{name}
        if parts and parts[0] == "namespaces" and len(parts) >= 3:
            ns, parts = parts[1], parts[2:]
        if not parts:
            raise ApiError(404, "NotFound", "not found")
        rt = self.store.lookup(group, parts[0])
        if rt.version != version:
            raise ApiError(404, "NotFound", f"{group}/{version} {parts[0]} is not served")
        name = parts[1] if len(parts) > 1 else None
        sub = parts[2] if len(parts) > 2 else ""
        if rt.namespaced and ns is None and name is not None:
            raise ApiError(404, "NotFound", f"{rt.plural} is namespaced")
        q = request.query
        dry = q.get("dryRun") == "All"
        m = request.method
        if name is None:
            if m == "GET":
                self._inject_list_fault(rt)
                if q.get("watch") in ("1", "true"):
                    self.watches[rt.plural] = self.watches.get(rt.plural, 0) + 1
                    return await self._watch(request, rt, ns)
                self.lists[rt.plural] = self.lists.get(rt.plural, 0) + 1
                lst = self.store.list(rt, ns, q.get("labelSelector"), q.get("fieldSelector"),
                                      int(q.get("limit", 0) or 0), q.get("continue"))
                if "as=Table" in request.headers.get("Accept", ""):
                    return web.json_response(to_table(rt, lst["items"],
                                                      lst["metadata"]["resourceVersion"]))
                return web.json_response(lst)
            if m == "POST":
                body = await request.json()
                out = self.store.create(rt, ns, body, dry_run=dry)
                return web.json_response(out, status=201)
            if m == "DELETE":
                lst = self.store.list(rt, ns, q.get("labelSelector"), q.get("fieldSelector"))
                for o in lst["items"]:
                    try:
                        self.store.delete(rt, o["metadata"].get("namespace"), o["metadata"]["name"])
                    except ApiError:
                        pass
                return web.json_response(lst)
            raise ApiError(405, "MethodNotAllowed", f"{m} not allowed on collection")
        if sub == "status":
            return await self._object(request, rt, ns, name, "status", dry)
        if sub == "scale":
            if m == "GET":
                return web.json_response(self.store.get_scale(rt, ns, name))
            if m == "PUT":
                return web.json_response(self.store.update_scale(rt, ns, name, await request.json(),
                                                                 self._manager(request)))
            if m == "PATCH":
                body = await request.json()
                cur = self.store.get_scale(rt, ns, name)
                cur["spec"]["replicas"] = body.get("spec", {}).get("replicas", cur["spec"]["replicas"])
                cur["metadata"].pop("resourceVersion", None)
                return web.json_response(self.store.update_scale(rt, ns, name, cur,
                                                                 self._manager(request)))
            raise ApiError(405, "MethodNotAllowed", f"{m} not allowed on scale")
        if sub == "log":
            if rt.kind != "Pod" or m != "GET":
                raise ApiError(405, "MethodNotAllowed", "log is GET on pods only")
            return await self._pod_log(request, ns, name)
        if sub == "eviction":
            if rt.kind != "Pod" or m != "POST":
                raise ApiError(405, "MethodNotAllowed", "eviction is POST on pods only")
            body = await request.json() if request.can_read_body else {}
            return web.json_response(self.store.evict(ns, name, body), status=201)
        if sub:
            raise ApiError(404, "NotFound", f"unknown subresource {sub}")
        return await self._object(request, rt, ns, name, "", dry)

    async def _pod_log(self, request, ns: str, name: str):
        """``pods/{name}/log``: what the kubelet proxies on a cluster; here the test kubelet's log
        file (the pod's ``gpupool.amd.com/log-path`` annotation). ``tailLines``, ``limitBytes``
        and ``follow`` (streams until the pod ends or the client goes)."""
        q = request.query
        pods = self.store.lookup("", "pods")
        pod = self.store.get(pods, ns, name)
        path = (pod["metadata"].get("annotations") or {}).get("gpupool.amd.com/log-path")
        if not path or not os.path.exists(path):
            if pod.get("status", {}).get("phase") == "Pending":
                raise ApiError(400, "BadRequest", f'container in pod "{name}" is waiting to start')
            return web.Response(text="", content_type="text/plain")

        def read(off: int) -> bytes:
            with open(path, "rb") as f:
                f.seek(off)
                return f.read()
        data = read(0)
        if q.get("tailLines"):
            n = int(q["tailLines"])
            lines = data.splitlines(keepends=True)
            data = b"".join(lines[-n:]) if n > 0 else b""
        if q.get("limitBytes"):
            data = data[:int(q["limitBytes"])]
        if q.get("follow") not in ("true", "1"):
            return web.Response(body=data, content_type="text/plain")
        resp = web.StreamResponse(headers={"Content-Type": "text/plain"})
        await resp.prepare(request)
        await resp.write(data)
        off = os.path.getsize(path)
        while True:
            await asyncio.sleep(0.1)
            try:
                more = read(off)
            except OSError:
                break
            if more:
                off += len(more)
                await resp.write(more)
            cur = self.store.objects[pods.key].get((ns, name))
            if cur is None or cur.get("status", {}).get("phase") in ("Succeeded", "Failed"):
                tail = read(off)
                if tail:
                    await resp.write(tail)
                break
        await resp.write_eof()
        return resp

    PATCH_TYPES = {"application/json-patch+json": "json",
                   "application/merge-patch+json": "merge",
                   "application/strategic-merge-patch+json": "strategic",
                   "application/apply-patch+yaml": "apply"}

    @staticmethod
    def _manager(request) -> str:
        """The field manager of a write: ``fieldManager``, else the User-Agent's product."""
        m = request.query.get("fieldManager")
        if m:
            return m
        ua = request.headers.get("User-Agent", "").split("/", 1)[0].strip()
        return ua or "unknown"

    @classmethod
    def _patch_type(cls, ctype: str) -> str:
        base = ctype.split(";", 1)[0].strip().lower()
        if base in cls.PATCH_TYPES:
            return cls.PATCH_TYPES[base]
        raise ApiError(415, "UnsupportedMediaType",
                       f"the body of the request was in an unknown format - accepted media types "
                       f"include: {', '.join(cls.PATCH_TYPES)}")

    def _admit_node_write(self, request, name: str, new: dict) -> None:
        """The agent's ValidatingAdmissionPolicy (schema.agent_node_policy), evaluated natively
        when that policy object is installed: no CEL engine here, the same four rules in Python.
        ``new`` is the write's dry-run result; the decision happens before the real write, with
        no await in between."""
        from ..api import schema
        user = request.get(USER_KEY)
        if not user or user.get("username") != schema.AGENT_SA_USER:
            return
        vap = self.store.types.get(("admissionregistration.k8s.io",
                                    "validatingadmissionpolicies"))
        if vap is None or ("", "gpupool-agent-own-node") not in self.store.objects[vap.key]:
            return
        old = self.store.get(self.store.lookup("", "nodes"), None, name)
        why = agent_node_policy_violation(user, old, new, schema.AGENT_OWN_CONDITIONS,
                                          schema.AGENT_LABEL_PREFIXES)
        if why:
            raise ApiError(403, "Forbidden", f'nodes "{name}" is forbidden: '
                           f"ValidatingAdmissionPolicy 'gpupool-agent-own-node' denied request: "
                           f"{why}")

    async def _object(self, request, rt, ns, name, sub, dry):
        m = request.method
        if m == "GET":
            obj = self.store.get(rt, ns, name)
            if "as=Table" in request.headers.get("Accept", ""):
                return web.json_response(to_table(rt, [obj], obj["metadata"]["resourceVersion"]))
            return web.json_response(obj)
        if m == "PUT":
            body = await request.json()
            mgr = self._manager(request)
            if rt.kind == "Node":
                self._admit_node_write(request, name, self.store.update(
                    rt, ns, name, body, sub, True, manager=mgr))
            # the decoded body is this request's own; the reply only serialises the result
            return web.json_response(self.store.update(rt, ns, name, body, sub, dry,
                                                       owned=True, copy_out=False, manager=mgr))
        if m == "PATCH":
            ptype = self._patch_type(request.headers.get("Content-Type", ""))
            if ptype == "apply":  # YAML (JSON is YAML too)
                try:
                    body = yaml.safe_load(await request.text())
                except yaml.YAMLError as e:
                    raise ApiError(400, "BadRequest", f"invalid apply patch: {e}") from e
                mgr = request.query.get("fieldManager", "")
            else:
                body = await request.json()
                mgr = self._manager(request)
            force = request.query.get("force") in ("true", "1")
            if rt.kind == "Node":
                self._admit_node_write(request, name, self.store.patch(
                    rt, ns, name, body, ptype, sub, True, manager=mgr, force=force))
            created = ptype == "apply" and \
                ((ns or "") if rt.namespaced else "", name) not in self.store.objects[rt.key]
            out = self.store.patch(rt, ns, name, body, ptype, sub, dry, copy_out=False,
                                   manager=mgr, force=force)
            return web.json_response(out, status=201 if created else 200)
        if m == "DELETE" and not sub:
            body = {}
            if request.can_read_body:
                try:
                    body = await request.json()
                except json.JSONDecodeError:
                    body = {}
            grace = request.query.get("gracePeriodSeconds", body.get("gracePeriodSeconds"))
            out = self.store.delete(rt, ns, name, None if grace is None else int(grace),
                                    body.get("preconditions"), dry)
            return web.json_response(out)
        raise ApiError(405, "MethodNotAllowed", f"{m} not allowed")

    # -------------------------------------------------------------- watch
    async def _watch(self, request: web.Request, rt: ResourceType, ns: str | None):
        q = request.query
        lm = parse_label_selector(q.get("labelSelector"))
        fm = parse_field_selector(q.get("fieldSelector"))
        bookmarks = q.get("allowWatchBookmarks") in ("1", "true")
        timeout = float(q.get("timeoutSeconds") or 0) or None
        rv_s = q.get("resourceVersion", "")

        def match(ev_obj: dict) -> bool:
            md = ev_obj["metadata"]
            if rt.namespaced and ns and md.get("namespace") != ns:
                return False
            return lm(md.get("labels")) and fm(ev_obj)
        filtered = bool(q.get("labelSelector") or q.get("fieldSelector"))

        queue: asyncio.Queue = asyncio.Queue()
        resp: web.StreamResponse | None = None
        # Register before computing the backlog so nothing falls between the two.
        self.watchers.setdefault(rt.key, set()).add(queue)
        try:
            initial: list[tuple[str, dict]] = []
            if rv_s in ("", "0"):
                start_rv = self.store.rv
                for o in self.store.list(rt, ns)["items"]:
                    if match(o):
                        initial.append(("ADDED", o))
            else:
                start_rv = int(rv_s)
                try:
                    for ev in self.store.events_since(rt, start_rv):
                        if match(ev.obj):
                            initial.append((ev.type, ev.obj))
                except ApiError as e:
                    resp = web.StreamResponse(headers={"Content-Type": "application/json"})
                    resp.enable_chunked_encoding()
                    await resp.prepare(request)
                    await resp.write((json.dumps({"type": "ERROR", "object": e.status()}) +
                                      "\n").encode())
                    await resp.write_eof()
                    return resp
            last_rv = max([start_rv] + [int(o["metadata"]["resourceVersion"]) for _, o in initial])
            resp = web.StreamResponse(headers={"Content-Type": "application/json",
                                               "Transfer-Encoding": "chunked"})
            resp.enable_chunked_encoding()
            await resp.prepare(request)
            for etype, o in initial:
                await resp.write((json.dumps({"type": etype, "object": o}) + "\n").encode())
            deadline = time.monotonic() + timeout if timeout else None
            next_bm = time.monotonic() + self.bookmark_interval
            while True:
                now = time.monotonic()
                wait = next_bm - now
                if deadline is not None:
                    wait = min(wait, deadline - now)
                    if wait <= 0:
                        break
                try:
                    t_ev, ev = await asyncio.wait_for(queue.get(), timeout=max(wait, 0.001))
                except asyncio.TimeoutError:
                    if bookmarks and time.monotonic() >= next_bm:
                        bm = {"type": "BOOKMARK", "object": {
                            "kind": rt.kind, "apiVersion": rt.api_version,
                            "metadata": {"resourceVersion": str(self.store.rv)}}}
                        await resp.write((json.dumps(bm) + "\n").encode())
                    if time.monotonic() >= next_bm:
                        next_bm = time.monotonic() + self.bookmark_interval
                    continue
                if ev.rtype != rt.key or ev.rv <= last_rv:
                    continue
                line = None
                if filtered and ev.type == "MODIFIED" and ev.prev is not None:
                    now_in, was_in = match(ev.obj), match(ev.prev)
                    if now_in != was_in:  # left / entered the selection
                        line = (json.dumps({"type": "ADDED" if now_in else "DELETED",
                                            "object": ev.obj}) + "\n").encode()
                    elif not now_in:
                        continue
                elif not match(ev.obj):
                    continue
                last_rv = ev.rv
                if self.watch_delay > 0:
                    lag = t_ev + self.watch_delay - time.monotonic()
                    if lag > 0:
                        await asyncio.sleep(lag)
                await resp.write(line or ev.encoded())
            await resp.write_eof()
            return resp
        except ConnectionResetError:
            # the client went away mid-stream (a watch it stopped, a process that exited): the
            # stream just ends, as the apiserver's does
            return resp if resp is not None else web.Response(status=499)
        finally:
            self.watchers.get(rt.key, set()).discard(queue)


async def serve(host: str, port: int, sim: ApiServerSim, port_file: str | None = None,
                crd_dir: str | None = None, unix: str | None = None,
                tls_cert: str | None = None, tls_key: str | None = None,
                client_ca: str | None = None) -> None:
    """Serve the simulator. With ``tls_cert``/``tls_key`` the TCP listener is HTTPS (TLS >= 1.2);
    with ``client_ca`` it additionally requires a client certificate signed by that CA."""
    if crd_dir:
        load_crd_dir(sim.store, crd_dir)
    runner = web.AppRunner(sim.app, access_log=None)
    await runner.setup()
    ssl_ctx = None
    if tls_cert:
        import ssl
        ssl_ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ssl_ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        ssl_ctx.load_cert_chain(tls_cert, tls_key)
        if client_ca:
            ssl_ctx.load_verify_locations(client_ca)
            ssl_ctx.verify_mode = ssl.CERT_REQUIRED
    site = web.TCPSite(runner, host, port, reuse_address=True, ssl_context=ssl_ctx)
    await site.start()
    bound = site._server.sockets[0].getsockname()[1]  # type: ignore[union-attr]
    if unix:
        await web.UnixSite(runner, unix).start()
    if port_file:
        import os
        tmp = port_file + ".tmp"
        with open(tmp, "w") as f:
            f.write(str(bound))
        os.replace(tmp, port_file)
    log.info("apiserver-sim listening on %s:%d", host, bound)
    print(f"apiserver-sim listening on {'https' if ssl_ctx else 'http'}://{host}:{bound}", flush=True)
    # start-up state (aiohttp, the parsed CRDs and their compiled schemas) lives for the whole
    # run: out of the collector's generations, so a full collection walks only request garbage
    import gc
    gc.collect()
    gc.freeze()
    while True:
        await asyncio.sleep(3600)


def load_crd_dir(store: Store, crd_dir: str) -> None:
    import glob
    import os

    import yaml
    rt = store.types[("apiextensions.k8s.io", "customresourcedefinitions")]
    for path in sorted(glob.glob(os.path.join(crd_dir, "*.yaml"))):
        with open(path) as f:
            for doc in yaml.safe_load_all(f):
                if doc and doc.get("kind") == "CustomResourceDefinition":
                    try:
                        store.create(rt, None, doc)
                    except ApiError as e:
                        if e.code != 409:
                            raise
