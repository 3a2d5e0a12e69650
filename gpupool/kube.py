"""Minimal, dependency-free Kubernetes REST client (stdlib ``http.client``).

Used by gpuctl, the node agent, the fake kubelet, the bench and the tests. Thread-safe: each
call opens its own connection unless a per-thread keep-alive connection is available.
Transports: http, https (CA file or in-memory PEM, optional client certificate) and unix
sockets; configuration from flags, the in-cluster ServiceAccount, or a kubeconfig.
"""
from __future__ import annotations

import http.client
import json
import os
import socket
import threading
import time
import urllib.parse
from dataclasses import dataclass
from typing import Any, Iterator

from .api import schema


class KubeError(Exception):
    def __init__(self, code: int, body: Any):
        self.code = code
        self.body = body
        msg = body.get("message") if isinstance(body, dict) else str(body)
        self.reason = body.get("reason", "") if isinstance(body, dict) else ""
        super().__init__(f"HTTP {code}: {msg}")


@dataclass(frozen=True)
class Res:
    """A resource type: group ('' = core), version, plural, namespaced."""
    group: str
    version: str
    plural: str
    namespaced: bool = True

    def path(self, ns: str | None = None, name: str | None = None, sub: str | None = None) -> str:
        base = f"/apis/{self.group}/{self.version}" if self.group else f"/api/{self.version}"
        if self.namespaced and ns:
            base += f"/namespaces/{ns}"
        base += f"/{self.plural}"
        if name:
            base += f"/{name}"
        if sub:
            base += f"/{sub}"
        return base


PODS = Res("", "v1", "pods")
NODES = Res("", "v1", "nodes", namespaced=False)
EVENTS = Res("", "v1", "events")
SECRETS = Res("", "v1", "secrets")
CONFIGMAPS = Res("", "v1", "configmaps")
NAMESPACES = Res("", "v1", "namespaces", namespaced=False)
LEASES = Res("coordination.k8s.io", "v1", "leases")
CRDS = Res("apiextensions.k8s.io", "v1", "customresourcedefinitions", namespaced=False)
MI355XPOOLS = Res(schema.GROUP, schema.VERSION, "mi355xpools")
AZUREVMPOOLS = Res(schema.GROUP, schema.VERSION, "azurevmpools")
MI355XJOBS = Res(schema.GROUP, schema.VERSION, "mi355xjobs")
MI355XQUEUES = Res(schema.GROUP, schema.VERSION, "mi355xqueues", namespaced=False)

BY_KIND = {
    "Pod": PODS, "Node": NODES, "Event": EVENTS, "Secret": SECRETS, "ConfigMap": CONFIGMAPS,
    "Namespace": NAMESPACES, "Lease": LEASES, "CustomResourceDefinition": CRDS,
    "Mi355xPool": MI355XPOOLS, "AzureVmPool": AZUREVMPOOLS, "Mi355xJob": MI355XJOBS,
    "Mi355xQueue": MI355XQUEUES,
    "ClusterRole": Res("rbac.authorization.k8s.io", "v1", "clusterroles", namespaced=False),
    "ClusterRoleBinding": Res("rbac.authorization.k8s.io", "v1", "clusterrolebindings",
                              namespaced=False),
    "ResourceQuota": Res("", "v1", "resourcequotas"),
    "ServiceAccount": Res("", "v1", "serviceaccounts"),
    "Service": Res("", "v1", "services"),
    "Deployment": Res("apps", "v1", "deployments"),
    "DaemonSet": Res("apps", "v1", "daemonsets"),
    "PodDisruptionBudget": Res("policy", "v1", "poddisruptionbudgets"),
    "NetworkPolicy": Res("networking.k8s.io", "v1", "networkpolicies"),
    "PersistentVolume": Res("", "v1", "persistentvolumes", namespaced=False),
    "PersistentVolumeClaim": Res("", "v1", "persistentvolumeclaims"),
    "ValidatingAdmissionPolicy": Res("admissionregistration.k8s.io", "v1",
                                     "validatingadmissionpolicies", namespaced=False),
    "ValidatingAdmissionPolicyBinding": Res("admissionregistration.k8s.io", "v1",
                                            "validatingadmissionpolicybindings", namespaced=False),
}


def load_kubeconfig(path: str | None = None, context: str | None = None) -> dict:
    """Resolve a kubeconfig context (clientcmd semantics; same subset as the C++
    ``load_kubeconfig``): path defaults to the first ``$KUBECONFIG`` entry, else ~/.kube/config;
    context to ``current-context``. Returns {server, token, namespace, context, ca_file, ca_data,
    cert_file, key_file, cert_data, key_data, insecure} (``*_data`` already base64-decoded)."""
    import base64

    import yaml
    if not path:
        env = os.environ.get("KUBECONFIG", "")
        path = env.split(os.pathsep)[0] if env else os.path.expanduser("~/.kube/config")
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    base = os.path.dirname(os.path.abspath(path))

    def named(kind: str, name: str) -> dict:
        for e in cfg.get(kind) or []:
            if e.get("name") == name:
                return e
        raise ValueError(f"kubeconfig {path}: no {kind[:-1]} named {name!r}")

    def rel(p: str | None) -> str | None:
        return p if not p or os.path.isabs(p) else os.path.join(base, p)

    def b64(v: str | None) -> str | None:
        return base64.b64decode(v).decode() if v else None

    ctx_name = context or cfg.get("current-context")
    if not ctx_name:
        raise ValueError(f"kubeconfig {path}: no current-context")
    ctx = named("contexts", ctx_name).get("context") or {}
    cl = named("clusters", ctx.get("cluster", "")).get("cluster") or {}
    out = {"server": cl.get("server"), "context": ctx_name, "namespace": ctx.get("namespace"),
           "insecure": bool(cl.get("insecure-skip-tls-verify")),
           "ca_file": rel(cl.get("certificate-authority")),
           "ca_data": b64(cl.get("certificate-authority-data")), "token": None,
           "cert_file": None, "key_file": None, "cert_data": None, "key_data": None}
    if ctx.get("user"):
        u = named("users", ctx["user"]).get("user") or {}
        if "exec" in u or "auth-provider" in u:
            raise ValueError(f"kubeconfig {path}: user {ctx['user']!r} uses an exec/auth-provider "
                             "plugin; use a token or client certificate")
        out["token"] = u.get("token")
        if not out["token"] and u.get("tokenFile"):
            with open(rel(u["tokenFile"])) as f:
                out["token"] = f.read().strip()
        out["cert_file"], out["key_file"] = rel(u.get("client-certificate")), rel(u.get("client-key"))
        out["cert_data"], out["key_data"] = b64(u.get("client-certificate-data")), \
            b64(u.get("client-key-data"))
    if not out["server"]:
        raise ValueError(f"kubeconfig {path}: cluster has no server")
    return out


class Client:
    def __init__(self, server: str, token: str | None = None, timeout: float = 30.0,
                 ca_file: str | None = None, insecure: bool = False,
                 client_cert: str | None = None, client_key: str | None = None,
                 token_file: str | None = None):
        u = urllib.parse.urlparse(server if "://" in server else "http://" + server)
        self.scheme = u.scheme
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or (443 if u.scheme == "https" else 80)
        self.unix = u.path if u.scheme == "unix" else None
        self.server = server
        self.token = token
        # a rotating credential (projected ServiceAccount token, Workload Identity): re-read at
        # most TOKEN_RELOAD_S after the last read and at once after a 401, as client-go does
        self.token_file = token_file
        self._token_read = -1e9
        self._token_mu = threading.Lock()
        self.token_reloads = 0
        if token_file:
            self._reload_token(force=True)
        self.timeout = timeout
        # "<product>/<version>": the apiserver names a writer's field manager after it
        self.user_agent = "gpupool-client/0.1"
        self.namespace: str | None = None  # kubeconfig context namespace, if any
        self._local = threading.local()
        self._ssl = None
        if self.scheme == "https":
            import ssl
            ca_data = None
            if ca_file and ca_file.startswith("-----BEGIN"):  # in-memory PEM (kubeconfig *-data)
                ca_data, ca_file = ca_file, None
            ctx = ssl.create_default_context(cafile=ca_file or os.environ.get("GPUPOOL_CA_FILE") or None,
                                             cadata=ca_data)
            ctx.minimum_version = ssl.TLSVersion.TLSv1_2
            if insecure:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
            if client_cert:
                ctx.load_cert_chain(client_cert, client_key)
            self._ssl = ctx

    SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"
    TOKEN_RELOAD_S = 60.0

    def _reload_token(self, force: bool = False) -> bool:
        """Re-read ``token_file`` when due (or ``force``). True when the token changed."""
        if not self.token_file:
            return False
        with self._token_mu:
            now = time.monotonic()
            if not force and now - self._token_read < self.TOKEN_RELOAD_S:
                return False
            self._token_read = now
            try:
                with open(self.token_file) as f:
                    tok = f.read().strip()
            except OSError:
                return False  # mid-rotation (the kubelet swaps a symlink): keep the last one
            if not tok or tok == self.token:
                return False
            self.token = tok
            self.token_reloads += 1
            return True

    @classmethod
    def from_env(cls) -> "Client":
        """``GPUPOOL_APISERVER``/``GPUPOOL_TOKEN``/``GPUPOOL_CA_FILE`` if set, else the in-cluster
        ServiceAccount config, else the local simulator default."""
        server = os.environ.get("GPUPOOL_APISERVER")
        if not server or server == "in-cluster":
            c = cls.in_cluster()
            if c is not None:
                return c
        return cls(server or "http://127.0.0.1:6443", os.environ.get("GPUPOOL_TOKEN") or None,
                   ca_file=os.environ.get("GPUPOOL_CA_FILE") or None)

    @classmethod
    def in_cluster(cls, sa_dir: str | None = None) -> "Client | None":
        """ServiceAccount config: https://$KUBERNETES_SERVICE_HOST:$KUBERNETES_SERVICE_PORT with the
        mounted token and CA. None when not running in a pod."""
        sa_dir = sa_dir or cls.SA_DIR
        host = os.environ.get("KUBERNETES_SERVICE_HOST")
        if not host or not os.path.exists(os.path.join(sa_dir, "token")):
            return None
        if ":" in host:
            host = f"[{host}]"
        return cls(f"https://{host}:{os.environ.get('KUBERNETES_SERVICE_PORT', '443')}", None,
                   ca_file=os.path.join(sa_dir, "ca.crt"), token_file=os.path.join(sa_dir, "token"))

    @classmethod
    def from_kubeconfig(cls, path: str | None = None, context: str | None = None,
                        timeout: float = 30.0) -> "Client":
        kc = load_kubeconfig(path, context)
        cert, key = kc["cert_file"], kc["key_file"]
        if kc["cert_data"]:  # ssl.load_cert_chain needs files: a private temp dir
            import tempfile
            d = tempfile.mkdtemp(prefix="gpuctl-kc-")
            cert, key = os.path.join(d, "client.crt"), os.path.join(d, "client.key")
            for pth, data in ((cert, kc["cert_data"]), (key, kc["key_data"] or kc["cert_data"])):
                fd = os.open(pth, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
                with os.fdopen(fd, "w") as f:
                    f.write(data)
        c = cls(kc["server"], kc["token"], timeout=timeout, ca_file=kc["ca_data"] or kc["ca_file"],
                insecure=kc["insecure"], client_cert=cert, client_key=key)
        c.namespace = kc["namespace"]
        return c

    @classmethod
    def connect(cls, server: str, token: str | None = None,
                token_file: str | None = None) -> "Client":
        """``server == "in-cluster"`` selects the ServiceAccount config, anything else is a URL.
        ``token_file`` (re-read as it rotates) wins over a fixed ``token``."""
        if server == "in-cluster":
            c = cls.in_cluster()
            if c is None:
                raise RuntimeError("--apiserver in-cluster but no ServiceAccount / KUBERNETES_SERVICE_HOST")
            return c
        return cls(server, token, token_file=token_file)

    # ------------------------------------------------------------ transport
    def _conn(self, timeout: float | None = None) -> http.client.HTTPConnection:
        if self.unix:
            return _UnixHTTPConnection(self.unix, timeout=timeout or self.timeout)
        if self.scheme == "https":
            return http.client.HTTPSConnection(self.host, self.port, timeout=timeout or self.timeout,
                                               context=self._ssl)
        return http.client.HTTPConnection(self.host, self.port, timeout=timeout or self.timeout)

    def _headers(self, ctype: str = "application/json", accept: str = "application/json") -> dict:
        self._reload_token()
        h = {"Content-Type": ctype, "Accept": accept, "User-Agent": self.user_agent}
        if self.token:
            h["Authorization"] = f"Bearer {self.token}"
        return h

    def request(self, method: str, path: str, body: Any = None, query: dict | None = None,
                ctype: str = "application/json", accept: str = "application/json",
                extra_headers: dict | None = None) -> Any:
        if query:
            q = {k: v for k, v in query.items() if v is not None}
            if q:
                path += "?" + urllib.parse.urlencode(q)
        data = None if body is None else json.dumps(body).encode()
        used = self.token
        resp, raw = self._roundtrip(method, path, data, ctype, accept, extra_headers)
        if resp.status == 401 and self.token_file:  # rotated under us: re-read, once more
            self._reload_token(force=True)
            if self.token != used:  # (or another thread's 401 already re-read it)
                resp, raw = self._roundtrip(method, path, data, ctype, accept, extra_headers)
        try:
            out = json.loads(raw) if raw else None
        except json.JSONDecodeError:
            out = raw.decode(errors="replace")
        if resp.status >= 400:
            raise KubeError(resp.status, out)
        return out

    def _roundtrip(self, method: str, path: str, data: bytes | None, ctype: str, accept: str,
                   extra_headers: dict | None = None):
        for attempt in range(2):
            conn = getattr(self._local, "conn", None)
            fresh = conn is None
            if conn is None:
                conn = self._local.conn = self._conn()
            try:
                conn.request(method, path, body=data,
                             headers={**self._headers(ctype, accept), **(extra_headers or {})})
                resp = conn.getresponse()
                raw = resp.read()
                break
            except (http.client.HTTPException, ConnectionError, OSError):
                self._local.conn = None
                try:
                    conn.close()
                except Exception:
                    pass
                if fresh or attempt == 1:
                    raise
        return resp, raw

    # ------------------------------------------------------------ verbs
    def get(self, res: Res, name: str, ns: str | None = None, sub: str | None = None) -> dict:
        return self.request("GET", res.path(ns, name, sub))

    def list(self, res: Res, ns: str | None = None, label_selector: str | None = None,
             field_selector: str | None = None) -> dict:
        return self.request("GET", res.path(ns), query={"labelSelector": label_selector,
                                                        "fieldSelector": field_selector})

    def table(self, res: Res, ns: str | None = None, name: str | None = None,
              label_selector: str | None = None) -> dict:
        return self.request("GET", res.path(ns, name), query={"labelSelector": label_selector},
                            accept="application/json;as=Table;v=v1;g=meta.k8s.io")

    def create(self, res: Res, obj: dict, ns: str | None = None, dry_run: bool = False) -> dict:
        return self.request("POST", res.path(ns), obj, query={"dryRun": "All" if dry_run else None})

    def update(self, res: Res, obj: dict, ns: str | None = None, sub: str | None = None,
               dry_run: bool = False) -> dict:
        return self.request("PUT", res.path(ns, obj["metadata"]["name"], sub), obj,
                            query={"dryRun": "All" if dry_run else None})

    def patch(self, res: Res, name: str, patch: Any, ns: str | None = None, sub: str | None = None,
              ptype: str = "merge", dry_run: bool = False) -> dict:
        ctype = {"merge": "application/merge-patch+json", "json": "application/json-patch+json",
                 "strategic": "application/strategic-merge-patch+json"}[ptype]
        return self.request("PATCH", res.path(ns, name, sub), patch, ctype=ctype,
                            query={"dryRun": "All" if dry_run else None})

    def delete(self, res: Res, name: str, ns: str | None = None, grace: int | None = None,
               preconditions: dict | None = None) -> dict:
        body: dict[str, Any] = {"kind": "DeleteOptions", "apiVersion": "v1"}
        if grace is not None:
            body["gracePeriodSeconds"] = grace
        if preconditions:
            body["preconditions"] = preconditions
        return self.request("DELETE", res.path(ns, name), body)

    def evict(self, ns: str, name: str, grace: int | None = None) -> dict:
        body = {"apiVersion": "policy/v1", "kind": "Eviction",
                "metadata": {"name": name, "namespace": ns}}
        if grace is not None:
            body["deleteOptions"] = {"gracePeriodSeconds": grace}
        return self.request("POST", PODS.path(ns, name, "eviction"), body)

    LAST_APPLIED = "kubectl.kubernetes.io/last-applied-configuration"

    def apply(self, obj: dict, ns: str | None = None, dry_run: bool = False,
              server_side: bool = False, field_manager: str = "gpuctl",
              force: bool = False) -> tuple[str, dict]:
        """``kubectl apply``. Client-side (the default): create, or patch with the three-way
        diff of the last applied configuration (kept in the ``last-applied-configuration``
        annotation), this manifest and the live object — fields others set (a ``scale``, a
        controller, a label someone added) survive, fields dropped from the manifest go; a
        strategic merge patch for built-in kinds, a JSON merge patch for custom resources.
        ``server_side``: server-side apply as ``field_manager`` (conflicts are the server's
        409 unless ``force``)."""
        from .api.smp import three_way
        res = res_for(obj)
        ns = (obj.get("metadata", {}).get("namespace") or ns or "default") if res.namespaced else None
        name = obj["metadata"]["name"]
        if server_side:
            existed = True
            try:
                self.get(res, name, ns)
            except KubeError as e:
                if e.code != 404:
                    raise
                existed = False
            out = self.request("PATCH", res.path(ns, name), obj, ctype="application/apply-patch+yaml",
                               query={"fieldManager": field_manager, "force": "true" if force else None,
                                      "dryRun": "All" if dry_run else None})
            return ("serverside-applied" if existed else "created"), out
        cfg = json.loads(json.dumps(obj))
        ann = cfg.setdefault("metadata", {}).get("annotations") or {}
        ann.pop(self.LAST_APPLIED, None)
        if not ann:
            cfg["metadata"].pop("annotations", None)
        modified = json.loads(json.dumps(cfg))
        modified["metadata"].setdefault("annotations", {})[self.LAST_APPLIED] = \
            json.dumps(cfg, sort_keys=True, separators=(",", ":"))
        try:
            cur = self.get(res, name, ns)
        except KubeError as e:
            if e.code != 404:
                raise
            return "created", self.create(res, modified, ns, dry_run)
        try:
            original = json.loads((cur["metadata"].get("annotations") or {})
                                  .get(self.LAST_APPLIED) or "null")
        except json.JSONDecodeError:
            original = None
        builtin = res.group in ("", "apps", "batch", "policy", "autoscaling") or \
            res.group.endswith(".k8s.io")
        for kind in ((obj.get("kind"), None) if builtin else (None,)):
            patch = three_way(original, modified, cur, kind)
            patch.pop("status", None)  # apply never writes status through the main resource
            if not patch:
                return "unchanged", cur
            try:
                out = self.patch(res, name, patch, ns, ptype="strategic" if kind else "merge",
                                 dry_run=dry_run)
            except KubeError as e:
                if e.code == 415 and kind:  # no strategic merge for this type: merge patch
                    continue
                raise
            changed = out["metadata"]["resourceVersion"] != cur["metadata"]["resourceVersion"]
            return ("configured" if changed else "unchanged"), out
        raise KubeError(415, {"message": "apply: no patch type accepted"})

    # ------------------------------------------------------------ watch
    def watch(self, res: Res, ns: str | None = None, resource_version: str | None = None,
              label_selector: str | None = None, field_selector: str | None = None,
              timeout_seconds: int | None = None, bookmarks: bool = True,
              stop: threading.Event | None = None) -> Iterator[dict]:
        """Yield watch events (dicts with ``type`` and ``object``) from one HTTP stream."""
        q = {"watch": "1", "resourceVersion": resource_version, "labelSelector": label_selector,
             "fieldSelector": field_selector, "allowWatchBookmarks": "true" if bookmarks else None,
             "timeoutSeconds": timeout_seconds}
        path = res.path(ns) + "?" + urllib.parse.urlencode({k: v for k, v in q.items() if v})
        # Reads block (a quiet watch may see nothing for minutes). The socket timeout only catches
        # a dead connection: after a timeout a response reader is unusable ("cannot read from
        # timed out object"), so ``stop`` is honoured by shutting the socket down from a helper
        # thread instead of polling with short timeouts — which broke every watch idle for 1 s,
        # and a relist in that gap missed DELETED events.
        conn = self._conn(timeout=(timeout_seconds or 3600) + 30)
        hdrs = self._headers()
        used = self.token
        conn.request("GET", path, headers=hdrs)
        resp = conn.getresponse()
        if resp.status == 401 and self.token_file and \
                (self._reload_token(force=True) or self.token != used):
            resp.read()
            conn.close()
            conn = self._conn(timeout=(timeout_seconds or 3600) + 30)
            conn.request("GET", path, headers=self._headers())
            resp = conn.getresponse()
        if resp.status >= 400:
            raw = resp.read()
            conn.close()
            raise KubeError(resp.status, json.loads(raw) if raw else None)
        done = threading.Event()
        if stop is not None:
            sock = conn.sock

            def _stopper() -> None:
                while not done.wait(0.2):
                    if stop.is_set():
                        try:
                            sock.shutdown(socket.SHUT_RDWR)
                        except OSError:
                            pass
                        return
            threading.Thread(target=_stopper, daemon=True, name="watch-stop").start()
        buf = b""
        try:
            while True:
                if stop is not None and stop.is_set():
                    return
                try:
                    chunk = resp.read1(65536) if hasattr(resp, "read1") else resp.read(1)
                except (OSError, ValueError, http.client.HTTPException):
                    if stop is not None and stop.is_set():  # our own shutdown of the socket
                        return
                    raise
                if not chunk:
                    return
                buf += chunk
                while b"\n" in buf:
                    line, buf = buf.split(b"\n", 1)
                    if line.strip():
                        yield json.loads(line)
        finally:
            done.set()
            conn.close()

    def wait_for(self, res: Res, name: str, ns: str | None, pred, timeout: float = 30.0,
                 poll: float | None = None) -> dict:
        """Block until ``pred(obj)`` is true (watch-driven); returns the object."""
        deadline = time.monotonic() + timeout
        while True:
            try:
                obj = self.get(res, name, ns)
                if pred(obj):
                    return obj
                rv = obj["metadata"]["resourceVersion"]
            except KubeError as e:
                if e.code != 404:
                    raise
                obj, rv = None, None
                if pred(None):
                    return None  # type: ignore[return-value]
            remaining = deadline - time.monotonic()
            if remaining <= 0:
                raise TimeoutError(f"timed out waiting for {res.plural}/{name}: last={obj}")
            if poll:
                time.sleep(min(poll, remaining))
                continue
            try:
                for ev in self.watch(res, ns, rv, field_selector=f"metadata.name={name}",
                                     timeout_seconds=max(1, int(remaining) + 1)):
                    if ev["type"] == "ERROR":
                        break
                    if ev["type"] == "BOOKMARK":
                        continue
                    o = None if ev["type"] == "DELETED" else ev["object"]
                    if pred(o):
                        return o  # type: ignore[return-value]
                    if time.monotonic() > deadline:
                        break
            except (OSError, http.client.HTTPException):
                time.sleep(0.05)


class _UnixHTTPConnection(http.client.HTTPConnection):
    def __init__(self, path: str, timeout: float = 30.0):
        super().__init__("localhost", timeout=timeout)
        self._path = path

    def connect(self) -> None:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.settimeout(self.timeout)
        s.connect(self._path)
        self.sock = s


def res_for(obj: dict) -> Res:
    kind = obj.get("kind")
    if kind in BY_KIND:
        return BY_KIND[kind]
    api = obj.get("apiVersion", "v1")
    g, v = api.split("/", 1) if "/" in api else ("", api)
    return Res(g, v, kind.lower() + "s")
