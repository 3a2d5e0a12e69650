"""Local control plane launcher: apiserver-sim + gpupool-manager + N node agents (+ fake kubelets).

The envtest/kind stand-in used by the integration tests, ``bench.py`` and ``make run``. Every
component runs as its own process (own session, so teardown kills whole process groups); logs go
to ``<workdir>/*.log``.
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time
from dataclasses import dataclass, field

from ..kube import Client

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "node_8x_mi355x.json")


def native_bin(name: str) -> str:
    d = os.environ.get("GPUPOOL_NATIVE_DIR") or os.path.join(ROOT, "build", "native")
    p = os.path.join(d, name)
    if not os.path.exists(p):
        raise FileNotFoundError(f"{p} missing: run `make native`")
    return p


def make_test_pki(workdir: str, name: str = "apiserver") -> tuple[str, str, str]:
    """Throw-away CA + server certificate (SAN IP:127.0.0.1, DNS:localhost) via the openssl CLI.
    Returns (ca.crt, server.crt, server.key)."""
    d = os.path.join(workdir, "pki")
    os.makedirs(d, exist_ok=True)
    ca_key, ca_crt = os.path.join(d, "ca.key"), os.path.join(d, "ca.crt")
    key, csr, crt = (os.path.join(d, f"{name}.{ext}") for ext in ("key", "csr", "crt"))
    ext = os.path.join(d, f"{name}.ext")
    with open(ext, "w") as f:
        f.write("subjectAltName=IP:127.0.0.1,DNS:localhost\nbasicConstraints=CA:FALSE\n"
                "keyUsage=digitalSignature,keyEncipherment\nextendedKeyUsage=serverAuth,clientAuth\n")
    run = lambda *a: subprocess.run(["openssl", *a], check=True, capture_output=True)  # noqa: E731
    run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", ca_key, "-out", ca_crt,
        "-days", "2", "-subj", f"/CN=gpupool-test-ca-{os.urandom(4).hex()}")
    run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", csr, "-subj", f"/CN={name}")
    run("x509", "-req", "-in", csr, "-CA", ca_crt, "-CAkey", ca_key, "-CAcreateserial", "-out", crt,
        "-days", "2", "-extfile", ext)
    return ca_crt, crt, key


def issue_client_cert(workdir: str, cn: str = "gpupool-admin") -> tuple[str, str]:
    """Client certificate (CN=user) signed by the CA ``make_test_pki(workdir)`` created.
    Returns (client.crt, client.key)."""
    d = os.path.join(workdir, "pki")
    key, csr, crt = (os.path.join(d, f"client-{cn}.{ext}") for ext in ("key", "csr", "crt"))
    ext = os.path.join(d, "client.ext")
    with open(ext, "w") as f:
        f.write("basicConstraints=CA:FALSE\nkeyUsage=digitalSignature,keyEncipherment\n"
                "extendedKeyUsage=clientAuth\n")
    run = lambda *a: subprocess.run(["openssl", *a], check=True, capture_output=True)  # noqa: E731
    run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", csr, "-subj", f"/CN={cn}")
    run("x509", "-req", "-in", csr, "-CA", os.path.join(d, "ca.crt"), "-CAkey",
        os.path.join(d, "ca.key"), "-CAcreateserial", "-out", crt, "-days", "2", "-extfile", ext)
    return crt, key


def make_signing_key(workdir: str, name: str = "agent-signing") -> tuple[str, str]:
    """An Ed25519 key pair (openssl CLI): (private key PEM path, public key PEM path)."""
    d = os.path.join(workdir, "pki")
    os.makedirs(d, exist_ok=True)
    key, pub = os.path.join(d, f"{name}.key"), os.path.join(d, f"{name}.pub")
    subprocess.run(["openssl", "genpkey", "-algorithm", "ed25519", "-out", key], check=True,
                   capture_output=True)
    os.chmod(key, 0o600)
    subprocess.run(["openssl", "pkey", "-in", key, "-pubout", "-out", pub], check=True,
                   capture_output=True)
    return key, pub


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _wait_file(path: str, timeout: float, proc: subprocess.Popen | None = None,
               logpath: str | None = None) -> str:
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if os.path.exists(path):
            with open(path) as f:
                data = f.read()
            if data:
                return data
        if proc is not None and proc.poll() is not None:
            tail = open(logpath).read()[-3000:] if logpath and os.path.exists(logpath) else ""
            raise RuntimeError(f"process exited ({proc.returncode}) before {path}:\n{tail}")
        time.sleep(0.02)
    tail = open(logpath).read()[-3000:] if logpath and os.path.exists(logpath) else ""
    raise TimeoutError(f"timed out waiting for {path}\n{tail}")


@dataclass
class NodeSpec:
    name: str
    backend: str = "fake"
    fixture: str = FIXTURE
    count: int = -1
    probe: str = ""               # "" -> agent default (simulated for fake, inproc for real)
    kubelet: bool = True
    extra_args: list[str] = field(default_factory=list)
    kubelet_args: list[str] = field(default_factory=list)
    # strict mounts (default): the fake kubelet fails a pod whose Allocate mounts or device
    # nodes lie outside what the agent DaemonSet shares with the host — the agent's state dir
    # (hostPath /var/lib/gpupool) and the GPU device nodes
    strict_mounts: bool = True


class Cluster:
    def __init__(self, workdir: str, nodes: list[NodeSpec] | None = None,
                 manager_args: list[str] | None = None, manager: bool = True,
                 python: str = sys.executable, env: dict | None = None,
                 sample_interval: float = 0.5, kinds: str = "mi355x,azure,job",
                 manager_bin: str | None = None, tls: bool = False, token: str | None = None,
                 fsync: bool = False, apiserver_args: list[str] | None = None,
                 agent_auth: str = "both", discovery: str = "annotation"):
        self.workdir = os.path.abspath(workdir)
        self.tls = tls
        self.token = token
        os.makedirs(self.workdir, exist_ok=True)
        # unix socket paths are limited to 107 bytes: keep every socket under a short /tmp dir
        import tempfile
        self.sockdir = tempfile.mkdtemp(prefix="gp", dir="/tmp")
        self.nodes = nodes if nodes is not None else [NodeSpec("mi355x-node-0")]
        self.manager_args = manager_args or []
        self.apiserver_args = apiserver_args or []
        self.want_manager = manager
        self.python = python
        self.env = dict(os.environ)
        self.env.setdefault("PYTHONPATH", ROOT)
        self.env["PYTHONPATH"] = ROOT + os.pathsep + self.env.get("PYTHONPATH", "")
        self.env.update(env or {})
        # every daemon started here exits once this process is gone (a runner killed at a
        # timeout skips the teardown): gpupool/utils/parent_watch.py
        self.env["GPUPOOL_EXIT_WITH_PARENT"] = str(os.getpid())
        self.sample_interval = sample_interval
        self.fsync = fsync  # agents' ledger fsync (the production default; tests skip it for speed)
        self.kinds = kinds
        self.manager_bin = manager_bin
        self.procs: dict[str, subprocess.Popen] = {}
        # the agents' RPC requires a shared secret (as deployed: the gpupool-agent-token Secret)
        self.agent_token = os.urandom(16).hex()
        self.agent_token_file = os.path.join(self.workdir, "agent-token")
        with open(self.agent_token_file, "w") as f:
            f.write(self.agent_token + "\n")
        os.chmod(self.agent_token_file, 0o600)
        self.env["GPUPOOL_AGENT_TOKEN"] = self.agent_token
        # manager -> agent credentials: "signature" (the deployed default: Ed25519 per request,
        # agentauth.h / edsig.py), "token" (the shared bearer) or "both" (agents accept either;
        # the manager then signs and sends no bearer)
        self.agent_auth = agent_auth
        self.signing_key = self.pubkeys = ""
        if agent_auth in ("signature", "both"):
            self.signing_key, self.pubkeys = make_signing_key(self.workdir)
        # "annotation": agents on unix sockets, found through the Node annotation; "pod": agents
        # on TCP at distinct loopback addresses, found through mirror Pods of the agent DaemonSet
        self.discovery = discovery
        self.agent_port = _free_port() if discovery == "pod" else 0
        self.agent_ips: dict[str, str] = {}
        self.url = ""
        self.client: Client | None = None

    # ------------------------------------------------------------ process helpers
    def _spawn(self, key: str, argv: list[str]) -> subprocess.Popen:
        logpath = os.path.join(self.workdir, f"{key}.log")
        logf = open(logpath, "ab")
        p = subprocess.Popen(argv, cwd=ROOT, env=self.env, stdout=logf, stderr=subprocess.STDOUT,
                             start_new_session=True)
        logf.close()
        self.procs[key] = p
        return p

    def _kill(self, key: str, sig=signal.SIGTERM, timeout: float = 10.0) -> None:
        p = self.procs.pop(key, None)
        if p is None or p.poll() is not None:
            return
        try:
            os.killpg(p.pid, sig)
        except ProcessLookupError:
            return
        try:
            p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait(timeout=5)

    def log(self, key: str) -> str:
        p = os.path.join(self.workdir, f"{key}.log")
        return open(p).read() if os.path.exists(p) else ""

    # ------------------------------------------------------------ components
    def start_apiserver(self) -> None:
        pf = os.path.join(self.workdir, "apiserver.port")
        if os.path.exists(pf):
            os.remove(pf)
        argv = [self.python, "-m", "gpupool.apiserver_sim", "--port", "0", "--port-file", pf,
                "--crd-dir", os.path.join(ROOT, "config", "crd"), "--bookmark-interval", "2"]
        argv += self.apiserver_args
        if self.token:
            argv += ["--token", self.token]
            self.env["GPUPOOL_TOKEN"] = self.token
        if self.tls:
            self.ca_file, cert, key = make_test_pki(self.workdir)
            argv += ["--tls-cert", cert, "--tls-key", key]
            self.env["GPUPOOL_CA_FILE"] = self.ca_file
        p = self._spawn("apiserver", argv)
        port = int(_wait_file(pf, 60, p, os.path.join(self.workdir, "apiserver.log")))
        self.url = f"{'https' if self.tls else 'http'}://127.0.0.1:{port}"
        self.client = Client(self.url, self.token, ca_file=self.ca_file if self.tls else None)

    def kubelet_root(self, node: NodeSpec) -> str:
        return os.path.join(self.sockdir, f"k-{node.name}")

    def start_kubelet(self, node: NodeSpec) -> None:
        root = self.kubelet_root(node)
        rf = os.path.join(self.workdir, f"kubelet-{node.name}.ready")
        if os.path.exists(rf):
            os.remove(rf)
        argv = [self.python, "-m", "gpupool.kubelet_fake", "--node", node.name,
                "--apiserver", self.url, "--root", root, "--workdir", ROOT, "--ready-file", rf]
        if node.strict_mounts:
            for hp in (self.state_dir(node.name), "/dev/kfd", "/dev/dri"):
                argv += ["--host-path", hp]
        argv += node.kubelet_args
        p = self._spawn(f"kubelet-{node.name}", argv)
        _wait_file(rf, 60, p, os.path.join(self.workdir, f"kubelet-{node.name}.log"))

    def faults_path(self, node: str) -> str:
        return os.path.join(self.workdir, f"faults-{node}.json")

    def state_dir(self, node: str) -> str:
        return os.path.join(self.workdir, f"state-{node}")

    def agent_socket(self, node: str) -> str:
        return os.path.join(self.sockdir, f"a-{node}.sock")

    def start_agent(self, node: NodeSpec) -> None:
        rf = os.path.join(self.workdir, f"agent-{node.name}.ready")
        if os.path.exists(rf):
            os.remove(rf)
        argv = [self.python, "-m", "gpupool.agent", "--node", node.name, "--backend", node.backend,
                "--state-dir", self.state_dir(node.name),
                "--socket", self.agent_socket(node.name), "--apiserver", self.url,
                "--faults", self.faults_path(node.name), "--ready-file", rf,
                "--sample-interval", str(self.sample_interval)] + \
            ([] if self.fsync else ["--no-fsync"])
        if self.agent_auth in ("token", "both"):
            argv += ["--auth-token-file", self.agent_token_file]
        if self.pubkeys:
            argv += ["--manager-pubkeys", self.pubkeys]
        if self.discovery == "pod":
            ip = self.agent_ips.setdefault(node.name, f"127.0.0.{10 + len(self.agent_ips)}")
            argv += ["--listen", f"{ip}:{self.agent_port}",
                     "--endpoint", f"http://{ip}:{self.agent_port}"]
        if node.backend == "fake":
            argv += ["--fixture", node.fixture]
        if node.count >= 0:
            argv += ["--count", str(node.count)]
        if node.probe:
            argv += ["--probe", node.probe]
        if node.kubelet:
            root = self.kubelet_root(node)
            argv += ["--plugin-dir", os.path.join(root, "device-plugins"),
                     "--pod-resources", os.path.join(root, "pod-resources", "kubelet.sock")]
        argv += node.extra_args
        wrap = os.environ.get("GPUPOOL_AGENT_WRAP", "")  # e.g. "rocprofv3 --kernel-trace --stats -d D --"
        if wrap:
            import shlex
            argv = shlex.split(wrap) + argv
        p = self._spawn(f"agent-{node.name}", argv)
        _wait_file(rf, 300, p, os.path.join(self.workdir, f"agent-{node.name}.log"))
        if self.discovery == "pod":
            self.publish_agent_pod(node.name)

    AGENT_NS = "gpupool-system"

    def publish_agent_pod(self, node: str, ip: str | None = None, ready: bool = True,
                          name: str | None = None) -> None:
        """The agent's Pod as the DaemonSet controller + kubelet would show it: bound to the node,
        Running, with the pod IP the CNI gave it (a mirror pod: the fake kubelet does not run it)."""
        from ..kube import PODS, KubeError
        name = name or f"gpupool-agent-{node}"
        pod = {"apiVersion": "v1", "kind": "Pod",
               "metadata": {"name": name, "namespace": self.AGENT_NS,
                            "labels": {"app.kubernetes.io/name": "gpupool-agent"},
                            "annotations": {"kubernetes.io/config.mirror": "gpupool-testing"}},
               "spec": {"nodeName": node, "containers": [{"name": "agent", "image": "gpupool"}]}}
        try:
            self.client.create(PODS, pod, self.AGENT_NS)
        except KubeError as e:
            if e.code != 409:
                raise
        self.client.patch(PODS, name, {"status": {
            "phase": "Running", "podIP": ip or self.agent_ips[node],
            "conditions": [{"type": "Ready", "status": "True" if ready else "False"}]}},
            self.AGENT_NS, sub="status")

    def start_manager(self) -> None:
        pf = os.path.join(self.workdir, "manager.port")
        if os.path.exists(pf):
            os.remove(pf)
        argv = [self.manager_bin or native_bin("gpupool-manager"), "--apiserver", self.url, "--port-file", pf,
                "--kinds", self.kinds, "--progress-poll", "100ms"]
        if self.agent_auth in ("token", "both"):
            argv += ["--agent-token-file", self.agent_token_file]
        if self.signing_key:
            argv += ["--agent-signing-key", self.signing_key]
        if self.discovery == "pod":
            argv += ["--agent-discovery", "pod", "--agent-scheme", "http",
                     "--agent-port", str(self.agent_port), "--agent-namespace", self.AGENT_NS]
        if self.tls:
            argv += ["--ca-file", self.ca_file]
        if self.token:
            tf = os.path.join(self.workdir, "token")
            with open(tf, "w") as f:
                f.write(self.token + "\n")
            argv += ["--token-file", tf]
        argv += self.manager_args
        p = self._spawn("manager", argv)
        self.metrics_port = int(_wait_file(pf, 60, p, os.path.join(self.workdir, "manager.log")))

    def start(self) -> "Cluster":
        self.start_apiserver()
        for n in self.nodes:
            if n.kubelet:
                self.start_kubelet(n)
            self.start_agent(n)
        if self.want_manager:
            self.start_manager()
        return self

    def stop(self) -> None:
        for key in [k for k in self.procs if k == "manager"] + \
                   [k for k in self.procs if k.startswith("agent")] + \
                   [k for k in self.procs if k.startswith("kubelet")] + list(self.procs):
            self._kill(key)
        import shutil
        shutil.rmtree(self.sockdir, ignore_errors=True)

    def __enter__(self) -> "Cluster":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()

    # ------------------------------------------------------------ fault injection
    def set_faults(self, node: str, faults: dict, sample: bool = True, notify: bool = True) -> None:
        """Write the node's fault overlay. ``sample`` forces an agent sample over the RPC;
        ``notify=False`` marks the write as not-an-event, so only the agent's periodic sample sees
        it (the detection path of a real ECC counter change, which amdsmi does not signal)."""
        path = self.faults_path(node)
        with open(path + ".tmp", "w") as f:
            json.dump(faults if notify else {**faults, "notify": False}, f)
        os.replace(path + ".tmp", path)
        # make sure the mtime changes even within one filesystem tick
        st = os.stat(path)
        os.utime(path, ns=(st.st_atime_ns, st.st_mtime_ns + 1000))
        if sample:
            self.agent_request(node, "POST", "/v1/sample", {})

    def agent_request(self, node: str, method: str, path: str, body: dict | None = None) -> dict:
        """An admin call on the node's agent (its unix socket), with the manager's credentials:
        the shared token if agents take one, else a signature for that node."""
        if self.agent_auth in ("token", "both"):
            c = Client("unix://" + self.agent_socket(node), self.agent_token)
            return c.request(method, path, body)
        from ..utils import edsig
        c = Client("unix://" + self.agent_socket(node))
        signer = edsig.Signer(self.signing_key)
        data = b"" if body is None else json.dumps(body).encode()
        hdr = signer.header(method, path, node, data)
        return c.request(method, path, body, extra_headers={"X-Gpupool-Signature": hdr})

    def manager_metrics(self) -> str:
        import urllib.request
        with urllib.request.urlopen(f"http://127.0.0.1:{self.metrics_port}/metrics", timeout=5) as r:
            return r.read().decode()

    def manager_traces(self, key: str = "", n: int = 64) -> list:
        """Recent reconcile traces from the manager's /debug/traces (newest first)."""
        import urllib.parse
        import urllib.request
        q = urllib.parse.urlencode({"n": n, **({"key": key} if key else {})})
        with urllib.request.urlopen(f"http://127.0.0.1:{self.metrics_port}/debug/traces?{q}",
                                    timeout=5) as r:
            return json.loads(r.read())
