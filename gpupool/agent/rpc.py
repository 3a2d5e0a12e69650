"""The node agent's RPC server: HTTP/1.1 + JSON over a unix socket and/or TCP (optionally TLS),
one thread per connection.

The manager keeps a few persistent connections per agent (its workers' claim / observe / release
calls and one long-poll on /v1/events). Serving each connection on its own thread lets a handler
run where the request arrived: a claim runs on its connection's thread from request to reply — no
event-loop hop into an executor and back, which on the claim path cost two GIL hand-offs and a
loop wake-up (profiles/r2am claim spans: executorIn + executorOut + aiohttp framing ~ 1 ms) — and
the event long-poll simply waits on a condition variable. Request framing is minimal on purpose:
Content-Length bodies (no chunked requests), keep-alive by default, ``Connection: close`` honoured.

Exposure bounds (the TCP listener is reachable from the node network): at most ``max_conns``
connections are served at once (more are closed on accept); a connection must finish its TLS
handshake and its first request within ``first_request_timeout`` seconds, and stays bounded by it
until a request is answered with something other than 401 — only then may it idle as a pooled
keep-alive connection; a request refused for its token closes the connection.
"""
from __future__ import annotations

import hmac
import json
import logging
import os
import socket
import ssl
import threading
import time
import urllib.parse
from typing import Callable

log = logging.getLogger("gpupool.agent.rpc")

# handler(query, body) -> (status, content_type, payload bytes, after_send or None)
Handler = Callable[[dict, bytes], tuple]
OPEN_PATHS = {"/healthz", "/metrics"}
_REASONS = {200: "OK", 400: "Bad Request", 401: "Unauthorized", 404: "Not Found",
            405: "Method Not Allowed", 409: "Conflict", 413: "Payload Too Large",
            500: "Internal Server Error"}
MAX_BODY = 16 << 20


def json_reply(obj, status: int = 200, after: Callable[[], None] | None = None) -> tuple:
    return status, "application/json", json.dumps(obj).encode(), after


def text_reply(text: str, status: int = 200) -> tuple:
    return status, "text/plain", text.encode(), None


class RpcServer:
    def __init__(self, routes: dict[tuple[str, str], Handler], token: str = "",
                 max_conns: int = 512, first_request_timeout: float = 10.0):
        self.routes = routes
        self.max_conns = max_conns
        self.first_request_timeout = first_request_timeout
        self._conns = 0
        self.refused_conns = 0
        self._conns_mu = threading.Lock()
        self._auth = ("Bearer " + token).encode() if token else b""
        self._listeners: list[socket.socket] = []
        self._stop = threading.Event()
        self.requests = 0
        self.stats: dict[str, list] = {}  # path -> [count, seconds]
        self._stats_mu = threading.Lock()

    # ------------------------------------------------------------ listeners
    def listen_unix(self, path: str) -> None:
        try:
            os.unlink(path)
        except FileNotFoundError:
            pass
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.bind(path)
        s.listen(64)
        self._start(s, None)

    def listen_tcp(self, host: str, port: int, ssl_ctx: ssl.SSLContext | None = None) -> None:
        s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind((host or "0.0.0.0", port))
        s.listen(64)
        self._start(s, ssl_ctx)

    def _start(self, s: socket.socket, ssl_ctx) -> None:
        self._listeners.append(s)
        threading.Thread(target=self._accept, args=(s, ssl_ctx), daemon=True,
                         name="rpc-accept").start()

    def close(self) -> None:
        self._stop.set()
        for s in self._listeners:
            try:
                s.close()
            except OSError:
                pass

    def _accept(self, s: socket.socket, ssl_ctx) -> None:
        while not self._stop.is_set():
            try:
                conn, _ = s.accept()
            except OSError:
                return
            with self._conns_mu:
                full = self._conns >= self.max_conns
                if full:
                    self.refused_conns += 1
                else:
                    self._conns += 1
            if full:
                try:
                    conn.close()
                except OSError:
                    pass
                continue
            try:
                threading.Thread(target=self._serve_conn, args=(conn, ssl_ctx), daemon=True,
                                 name="rpc-conn").start()
            except RuntimeError:  # no thread to be had: drop this connection, keep accepting
                with self._conns_mu:
                    self._conns -= 1
                    self.refused_conns += 1
                try:
                    conn.close()
                except OSError:
                    pass

    @property
    def open_conns(self) -> int:
        with self._conns_mu:
            return self._conns

    # ------------------------------------------------------------ one connection
    def _serve_conn(self, conn: socket.socket, ssl_ctx) -> None:
        trusted = False  # until a request is answered with something other than 401
        try:
            conn.settimeout(self.first_request_timeout or None)  # handshake + first request
            if conn.family != socket.AF_UNIX:
                conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            if ssl_ctx is not None:
                conn = ssl_ctx.wrap_socket(conn, server_side=True)
            rf = conn.makefile("rb", buffering=65536)
            while not self._stop.is_set():
                line = rf.readline(65537)
                if not line:
                    return
                if line in (b"\r\n", b"\n"):
                    continue
                try:
                    method, target, version = line.decode("latin-1").split(None, 2)
                except ValueError:
                    return
                headers: dict[str, str] = {}
                while True:
                    h = rf.readline(65537)
                    if h in (b"\r\n", b"\n", b""):
                        break
                    k, _, v = h.decode("latin-1").partition(":")
                    headers[k.strip().lower()] = v.strip()
                n = int(headers.get("content-length") or 0)
                if n > MAX_BODY:
                    self._send(conn, (413, "text/plain", b"body too large\n", None), False)
                    return
                body = rf.read(n) if n else b""
                keep = headers.get("connection", "").lower() != "close" and \
                    not version.strip().upper().endswith("1.0")
                t0 = time.perf_counter()
                reply = self._dispatch(method.upper(), target, headers, body)
                if reply[0] == 401:
                    keep = False  # no second guess on this connection
                elif not trusted:
                    trusted = True
                    conn.settimeout(None)  # a pooled keep-alive connection may idle from here
                self._send(conn, reply, keep)
                self._account(target.partition("?")[0], time.perf_counter() - t0)
                if reply[3] is not None:
                    try:
                        reply[3]()
                    except Exception:
                        log.exception("post-reply hook failed")
                if not keep:
                    return
        except (OSError, ssl.SSLError, ValueError):
            return
        finally:
            try:
                conn.close()
            except OSError:
                pass
            with self._conns_mu:
                self._conns -= 1

    def _account(self, path: str, seconds: float) -> None:
        with self._stats_mu:
            st = self.stats.setdefault(path, [0, 0.0])
            st[0] += 1
            st[1] += seconds

    def metrics_lines(self) -> list[str]:
        """Server-side time per RPC path, request parsed -> reply written (``rpc_seconds``); the
        manager's span for the same call minus this is transport + framing."""
        with self._stats_mu:
            items = sorted(self.stats.items())
        out = [f"gpupool_agent_rpc_open_connections {self.open_conns}",
               f"gpupool_agent_rpc_refused_connections_total {self.refused_conns}"]
        for path, (n, sec) in items:
            out.append(f'gpupool_agent_rpc_requests_total{{path="{path}"}} {n}')
            out.append(f'gpupool_agent_rpc_seconds_sum{{path="{path}"}} {sec:.6f}')
        return out

    def _dispatch(self, method: str, target: str, headers: dict, body: bytes) -> tuple:
        path, _, qs = target.partition("?")
        self.requests += 1
        if self._auth and path not in OPEN_PATHS and \
                not hmac.compare_digest(headers.get("authorization", "").encode(), self._auth):
            return json_reply({"reason": "Unauthorized",
                               "message": "agent RPC requires the manager's token"}, 401)
        h = self.routes.get((method, path))
        if h is None:
            known = any(p == path for _, p in self.routes)
            return json_reply({"reason": "MethodNotAllowed" if known else "NotFound",
                               "message": f"{method} {path}"}, 405 if known else 404)
        query = {k: v[-1] for k, v in urllib.parse.parse_qs(qs).items()}
        try:
            return h(query, body)
        except (ValueError, KeyError, TypeError) as e:
            return json_reply({"reason": "BadRequest", "message": str(e)}, 400)
        except Exception as e:  # a handler bug must not kill the connection thread silently
            log.exception("RPC %s %s failed", method, path)
            return json_reply({"reason": "InternalError", "message": repr(e)}, 500)

    @staticmethod
    def _send(conn: socket.socket, reply: tuple, keep: bool) -> None:
        status, ctype, payload = reply[0], reply[1], reply[2]
        head = (f"HTTP/1.1 {status} {_REASONS.get(status, 'OK')}\r\n"
                f"Content-Type: {ctype}\r\nContent-Length: {len(payload)}\r\n"
                f"Connection: {'keep-alive' if keep else 'close'}\r\n\r\n").encode()
        conn.sendall(head + payload)
