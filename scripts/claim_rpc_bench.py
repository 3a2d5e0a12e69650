#!/usr/bin/env python3
"""Claim-RPC overhead micro-benchmark: one node agent (fake backend, simulated 1 ms probe, fsync on)
with a device-plugin consumer standing in for the kubelet (Registration + a ListAndWatch stream
read on its own thread, as the kubelet does), driven over its unix socket with the manager's
claim / cordon / release calls. Prints per-phase p50s and the overhead the manager sees over the
probe: client round trip − probe. Used to cut the claim path."""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import http.client
import json
import os
import socket
import statistics
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import grpc  # noqa: E402

from gpupool.agent.deviceplugin.proto import DP, Stub, service_handler, unix_target  # noqa: E402


class Kubelet:
    """Registration service; every registered plugin gets a ListAndWatch reader thread."""

    def __init__(self, plugin_dir: str):
        self.dir = plugin_dir
        self.updates = 0
        self.server = grpc.server(cf.ThreadPoolExecutor(4))
        self.server.add_generic_rpc_handlers((service_handler("v1beta1.Registration",
                                                              {"Register": self.Register}),))
        os.makedirs(plugin_dir, exist_ok=True)
        self.server.add_insecure_port(unix_target(os.path.join(plugin_dir, "kubelet.sock")))
        self.server.start()

    def Register(self, req, ctx):
        threading.Thread(target=self._watch, args=(req.endpoint,), daemon=True).start()
        return DP.Empty()

    def _watch(self, endpoint: str) -> None:
        time.sleep(0.05)
        ch = grpc.insecure_channel(unix_target(os.path.join(self.dir, endpoint)))
        try:
            for _ in Stub(ch, "v1beta1.DevicePlugin").ListAndWatch(DP.Empty()):
                self.updates += 1
        except grpc.RpcError:
            pass  # the agent stopped


class UnixHTTP(http.client.HTTPConnection):
    def __init__(self, path: str):
        super().__init__("localhost")
        self.path = path

    def connect(self):
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.connect(self.path)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--count", type=int, default=1)
    ap.add_argument("--gap", type=float, default=0.05, help="idle seconds between cycles")
    ap.add_argument("--auth", choices=["none", "v1", "v2"], default="none",
                    help="sign the calls as the manager does: v1 Ed25519, v2 the per-node MAC")
    args = ap.parse_args()
    d = tempfile.mkdtemp(prefix="claimbench", dir="/tmp")
    auth_args: list[str] = []
    signer = None
    if args.auth != "none":
        from gpupool.utils import edsig
        seed = os.urandom(32)
        pub = edsig.public_from_private(seed)
        with open(os.path.join(d, "manager.pem"), "w") as f:
            f.write(edsig.public_pem(pub))
        auth_args = ["--manager-pubkeys", os.path.join(d, "manager.pem")]

        def signer(method: str, path: str, body: bytes) -> dict:
            if args.auth == "v1":
                return {"X-Gpupool-Signature": edsig.sign_header(seed, method, path, "n0", body,
                                                                 pub=pub)}
            kx = edsig.AgentKx(os.path.join(d, "state", "agent-kx.key"))  # the agent's, read once
            if not hasattr(signer, "key"):
                xm_priv = edsig.x25519_private_from_ed25519_seed(seed)
                xm = edsig.x25519_public(xm_priv)
                signer.key = edsig.mac_key(edsig.x25519(xm_priv, kx.public), "n0", xm, kx.public)
                signer.kx = kx.public
            return {"X-Gpupool-Signature": edsig.mac_header(signer.key, edsig.key_id(pub),
                                                            signer.kx, method, path, "n0", body)}
    # the kubelet is its own process (as on a node): its stream reader must not share this
    # client's GIL
    kubelet = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--kubelet",
                                os.path.join(d, "dp")], cwd=ROOT)
    deadline = time.monotonic() + 30
    while not os.path.exists(os.path.join(d, "dp", "kubelet.sock")) and \
            time.monotonic() < deadline:
        time.sleep(0.02)
    sock = os.path.join(d, "agent.sock")
    ready = os.path.join(d, "ready")
    agent = subprocess.Popen(
        [sys.executable, "-m", "gpupool.agent", "--node", "n0", "--backend", "fake",
         "--fixture", os.path.join(ROOT, "tests", "fixtures", "node_8x_mi355x.json"),
         "--state-dir", os.path.join(d, "state"), "--socket", sock,
         "--plugin-dir", os.path.join(d, "dp"), "--probe", "simulated", "--probe-sim-ms", "1",
         "--scrub-interval", "0", "--ready-file", ready, *auth_args],
        cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT), stderr=open("/tmp/agent_claimbench.err", "w"))
    try:
        deadline = time.monotonic() + 60
        while not os.path.exists(ready) and time.monotonic() < deadline:
            time.sleep(0.05)
        conn = UnixHTTP(sock)

        def hdrs(path: str, b: bytes) -> dict:
            return {"Content-Type": "application/json", **(signer("POST", path, b) if signer else {})}

        def call(path: str, body: dict) -> dict:
            b = json.dumps(body).encode()
            conn.request("POST", path, b, hdrs(path, b))
            r = conn.getresponse()
            return json.loads(r.read())

        req = {"poolUID": "uid-1", "pool": "default/p", "count": args.count,
               "resourceName": "amd.com/gpu", "policy": {}, "topologyPolicy": "xgmi-packed",
               "probe": {"enabled": True}}
        rows = []
        for i in range(args.warmup + args.iters):
            b = json.dumps(req).encode()
            h = hdrs("/v1/claims", b)  # signed outside the timed window (the manager's C++ cost)
            t0 = time.perf_counter()
            conn.request("POST", "/v1/claims", b, h)
            raw = conn.getresponse().read()
            rt = (time.perf_counter() - t0) * 1e3
            out = json.loads(raw)
            assert out.get("ok"), out
            uu = [x["uuid"] for x in out["devices"]]
            if i >= args.warmup:
                rows.append({"rt": rt, **out["timingsMs"]})
                reply_bytes = len(raw)
            call("/v1/cordon", {"poolUID": "uid-1", "uuids": uu})
            rel = call("/v1/release", {"poolUID": "uid-1", "uuids": uu})
            assert rel.get("ok"), rel
            time.sleep(args.gap)  # the bench's cycles are apart: let the agent settle
        hz = []
        for _ in range(200):
            t0 = time.perf_counter()
            conn.request("GET", "/healthz")
            conn.getresponse().read()
            hz.append((time.perf_counter() - t0) * 1e3)
        conn.request("GET", "/metrics")
        met = conn.getresponse().read().decode()
        server = {}
        for line in met.splitlines():
            if 'path="/v1/claims"' in line:
                server[line.split("{")[0]] = float(line.rsplit(" ", 1)[1])
        server_avg = 1e3 * server["gpupool_agent_rpc_seconds_sum"] / \
            server["gpupool_agent_rpc_requests_total"]
        keys = sorted({k for r in rows for k in r})
        p50 = {k: round(statistics.median(r.get(k, 0.0) for r in rows), 3) for k in keys}
        spans = sum(v for k, v in p50.items() if k not in ("rt", "probe"))
        un = [r["rt"] - sum(v for k, v in r.items() if k != "rt") for r in rows]
        p90 = {k: round(sorted(r.get(k, 0.0) for r in rows)[int(0.9 * len(rows))], 3)
               for k in keys}
        print(json.dumps({"iters": args.iters, "p50_ms": p50,
                          "overhead_over_probe_ms": round(p50["rt"] - p50["probe"], 3),
                          "spans_sum_ms": round(spans, 3),
                          "unspanned_ms": round(p50["rt"] - p50["probe"] - spans, 3),
                          "unspanned_per_call_p50_ms": round(statistics.median(un), 3),
                          "p90_ms": p90,
                          "server_avg_ms_incl_warmup": round(server_avg, 3),
                          "reply_bytes": reply_bytes,
                          "healthz_rt_p50_ms": round(statistics.median(hz), 3),
                          }))
        return 0
    finally:
        agent.terminate()
        try:
            agent.wait(timeout=10)
        except subprocess.TimeoutExpired:
            agent.kill()
        kubelet.terminate()
        kubelet.wait(timeout=10)


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--kubelet":
        Kubelet(sys.argv[2])
        threading.Event().wait()
    sys.exit(main())
