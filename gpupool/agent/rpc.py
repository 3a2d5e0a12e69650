"""The node agent's RPC server: HTTP/1.1 + JSON over a unix socket and/or TCP (optionally TLS),
one thread per connection.

The manager keeps a few persistent connections per agent (its workers' claim / observe / release
calls and one long-poll on /v1/events). Serving each connection on its own thread lets a handler
run where the request arrived: a claim runs on its connection's thread from request to reply — no
event-loop hop into an executor and back, which on the claim path cost two GIL hand-offs and a
loop wake-up (profiles/r2am claim spans: executorIn + executorOut + aiohttp framing ~ 1 ms) — and
the event long-poll simply waits on a condition variable. Request framing is minimal on purpose:
Content-Length bodies (no chunked requests), keep-alive by default, ``Connection: close`` honoured.

Exposure bounds (the TCP listener is reachable from the node network):
  * at most ``max_conns`` connections are served at once (more are closed on accept);
  * an absolute deadline: a connection must finish its TLS handshake and its first request within
    ``first_request_timeout`` seconds of its accept, however slowly its bytes trickle in — every
    read waits only for what is left of it, and a reaper thread shuts down a connection still
    untrusted at its deadline (which also bounds a stalled TLS handshake). The deadline covers
    receiving the request, not handling it: once an authorised request has been read whole it is
    lifted, so a long handler (a scrub that maps the free HBM of a GPU whose VRAM the driver is
    still clearing, a claim probing 8 GPUs) still gets its reply out. Only a request that carried
    valid credentials makes the connection trusted (with none configured: any request): it may
    then idle as a pooled keep-alive connection. An unauthenticated request to an open path
    (/healthz, /metrics) is answered with ``Connection: close`` — one keep-alive GET /healthz per
    connection must not pin the ``max_conns`` slots the manager's claims need;
  * a trusted connection may idle between requests, but once the first byte of a request head
    arrives, the head and its body must be in within ``first_request_timeout``: a trusted peer
    cannot drip a request either;
  * credentials (auth.py: the manager's per-request signature and/or a rotating bearer token) are
    checked right after the headers, before any body byte is read, and the signed body digest
    once the body is in; a request refused for them closes the connection;
  * at most ``MAX_HEADERS`` header lines of ``MAX_HEADER_BYTES`` in total; a body-carrying method
    (POST/PUT/PATCH) needs a decimal Content-Length (missing, negative or non-numeric -> 400,
    nothing read), at most ``MAX_BODY``.
"""
from __future__ import annotations

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
            431: "Request Header Fields Too Large", 500: "Internal Server Error"}
MAX_BODY = 16 << 20
MAX_HEADERS = 64
MAX_HEADER_BYTES = 16 << 10
MAX_LINE = 8 << 10
BODY_METHODS = {"POST", "PUT", "PATCH"}


class _Closed(Exception):
    """The peer went away, or the connection's deadline passed."""


class _Reader:
    """Buffered reads from a socket under an optional absolute deadline (``time.monotonic``):
    each recv waits only for the time left, so a peer dripping one byte at a time cannot stretch
    the bound the way a per-recv socket timeout lets it."""

    def __init__(self, conn):
        self.conn = conn
        self.buf = bytearray()
        self.deadline: float | None = None
        self._timed = False
        self.total = 0  # bytes received on this connection

    def _fill(self) -> None:
        if self.deadline is not None:
            left = self.deadline - time.monotonic()
            if left <= 0:
                raise _Closed("deadline")
            self.conn.settimeout(left)
            self._timed = True
        elif self._timed:
            self.conn.settimeout(None)
            self._timed = False
        try:
            data = self.conn.recv(65536)
        except socket.timeout:
            raise _Closed("deadline") from None
        if not data:
            raise _Closed("eof")
        self.total += len(data)
        self.buf += data

    def readline(self, limit: int) -> bytes:
        """One line including its newline; ValueError past ``limit`` bytes without one."""
        start = 0
        while True:
            i = self.buf.find(b"\n", start)
            if i >= 0:
                if i + 1 > limit:
                    raise ValueError("line too long")
                line = bytes(self.buf[:i + 1])
                del self.buf[:i + 1]
                return line
            if len(self.buf) >= limit:
                raise ValueError("line too long")
            start = len(self.buf)
            self._fill()

    def read_head(self, limit: int) -> bytes | None:
        """Everything up to and including the blank line that ends a request head; None past
        ``limit`` bytes without one. One scan per received chunk, not one per header line."""
        start = 0
        while True:
            i = self.buf.find(b"\r\n\r\n", start)
            if i >= 0:
                head = bytes(self.buf[:i + 4])
                del self.buf[:i + 4]
                return head
            if len(self.buf) > limit:
                return None
            start = max(0, len(self.buf) - 3)
            self._fill()

    def read(self, n: int) -> bytes:
        while len(self.buf) < n:
            self._fill()
        out = bytes(self.buf[:n])
        del self.buf[:n]
        return out


def json_reply(obj, status: int = 200, after: Callable[[], None] | None = None) -> tuple:
    return status, "application/json", json.dumps(obj).encode(), after


def text_reply(text: str, status: int = 200) -> tuple:
    return status, "text/plain", text.encode(), None


class RpcServer:
    def __init__(self, routes: dict[tuple[str, str], Handler], token: str = "",
                 max_conns: int = 512, first_request_timeout: float = 10.0,
                 guard: Callable[[str, str, dict], tuple | None] | None = None,
                 auth=None):
        self.routes = routes
        # guard(method, path, headers) -> a reply refusing the request, or None: runs after the
        # token check and before the handler (the agent's leader fencing, StaleLeader)
        self.guard = guard
        self.max_conns = max_conns
        self.first_request_timeout = first_request_timeout
        self._conns = 0
        self.refused_conns = 0
        self._conns_mu = threading.Lock()
        # who may call (auth.AgentAuth): request signatures and/or a rotating bearer token;
        # ``token`` alone is the fixed shared secret of tests and older deployments
        if auth is None:
            from .auth import AgentAuth, TokenAuth
            auth = AgentAuth(token=TokenAuth(token) if token else None)
        self.auth = auth
        self._listeners: list[socket.socket] = []
        self._stop = threading.Event()
        self.requests = 0
        self.stats: dict[str, list] = {}  # path -> [count, seconds]
        self._stats_mu = threading.Lock()
        # untrusted connections -> their absolute deadline; the reaper shuts down the late ones
        self._pending: dict[socket.socket, float] = {}
        self._pending_cv = threading.Condition()
        self.reaped = 0
        self.rejected_requests = 0
        self.open_path_closes = 0  # unauthenticated /healthz, /metrics answered and closed
        self.request_deadline_closes = 0  # trusted connections cut mid-request at the deadline
        self.bytes_read = 0  # over all finished connections (tests: what a rejected peer cost)
        threading.Thread(target=self._reaper, daemon=True, name="rpc-reaper").start()

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
        with self._pending_cv:
            self._pending_cv.notify()
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

    # ------------------------------------------------------------ deadlines
    def _reaper(self) -> None:
        """Shuts down connections still untrusted at their deadline: a blocked recv (plain or in
        a TLS handshake) then returns, and the connection's thread closes it."""
        with self._pending_cv:
            while not self._stop.is_set():
                now = time.monotonic()
                late = [c for c, d in self._pending.items() if d <= now]
                for c in late:
                    del self._pending[c]
                    self.reaped += 1
                    try:
                        c.shutdown(socket.SHUT_RDWR)
                    except OSError:
                        pass
                nxt = min(self._pending.values(), default=None)
                self._pending_cv.wait(None if nxt is None else max(0.01, nxt - now))

    def _watch(self, conn: socket.socket, deadline: float) -> None:
        with self._pending_cv:
            self._pending[conn] = deadline
            self._pending_cv.notify()

    def _unwatch(self, conn: socket.socket) -> None:
        with self._pending_cv:
            self._pending.pop(conn, None)

    # ------------------------------------------------------------ one connection
    LINGER_BYTES = 64 << 10  # at most this much of a refused request is ever read, in total
    LINGER_S = 0.5

    def _reject(self, conn, status: int, reason: str, message: str, rf: "_Reader | None" = None) -> None:
        """Answer a refused request and close without reading its body — gracefully: the reply is
        followed by a FIN, then whatever the client still sends is discarded for a moment
        (bounded by LINGER_BYTES over the whole connection and LINGER_S), so the client reads the
        status instead of a reset. Closing with unread bytes in the receive buffer makes TCP send
        an RST, and the client's body write then fails with EPIPE before it sees the 401."""
        self.rejected_requests += 1
        try:
            self._send(conn, json_reply({"reason": reason, "message": message}, status), False)
            conn.shutdown(socket.SHUT_WR)
        except OSError:
            return
        budget = self.LINGER_BYTES - (rf.total if rf is not None else 0)
        end = time.monotonic() + self.LINGER_S
        while budget > 0:
            left = end - time.monotonic()
            if left <= 0:
                break
            try:
                conn.settimeout(left)
                data = conn.recv(min(65536, budget))
            except (OSError, ValueError):
                break
            if not data:
                break
            budget -= len(data)
            if rf is not None:
                rf.total += len(data)

    def _serve_conn(self, conn: socket.socket, ssl_ctx) -> None:
        trusted = False  # until a request carrying the token (or any, without one) is answered
        raw = conn
        rf = None
        deadline = time.monotonic() + self.first_request_timeout if self.first_request_timeout \
            else None
        if deadline is not None:
            self._watch(raw, deadline)
        try:
            if conn.family != socket.AF_UNIX:
                conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            if ssl_ctx is not None:
                # the wrapper takes over the fd (the plain socket object is detached): watch the
                # wrapper from here, then handshake — bounded by the reaper like any read
                conn.settimeout(self.first_request_timeout or None)
                conn = ssl_ctx.wrap_socket(conn, server_side=True, do_handshake_on_connect=False)
                if deadline is not None:
                    self._unwatch(raw)
                    self._watch(conn, deadline)
                raw = conn
                conn.do_handshake()
            rf = _Reader(conn)
            rf.deadline = deadline
            while not self._stop.is_set():
                try:
                    if trusted and self.first_request_timeout:
                        # idle keep-alive: no bound until the next request starts; from its first
                        # byte, head and body share one absolute deadline
                        rf.deadline = None
                        if not rf.buf:
                            rf._fill()
                        rf.deadline = time.monotonic() + self.first_request_timeout
                    head = rf.read_head(MAX_LINE + MAX_HEADER_BYTES)
                except _Closed as e:
                    if trusted and str(e) == "deadline":
                        self.request_deadline_closes += 1
                    return
                if head is None:
                    self._reject(conn, 431, "HeadersTooLarge",
                                 f"request head over {MAX_LINE + MAX_HEADER_BYTES} bytes", rf)
                    return
                lines = head.split(b"\r\n")
                while lines and not lines[0]:  # blank lines before a request line are allowed
                    lines.pop(0)
                if not lines:
                    continue
                if len(lines[0]) > MAX_LINE:
                    return
                try:
                    method, target, version = lines[0].decode("latin-1").split(None, 2)
                except ValueError:
                    return
                method = method.upper()
                fields = [h for h in lines[1:] if h]
                if len(fields) > MAX_HEADERS or len(head) - len(lines[0]) > MAX_HEADER_BYTES:
                    self._reject(conn, 431, "HeadersTooLarge",
                                 f"at most {MAX_HEADERS} header lines / {MAX_HEADER_BYTES} bytes", rf)
                    return
                headers: dict[str, str] = {}
                for h in fields:
                    k, _, v = h.decode("latin-1").partition(":")
                    headers[k.strip().lower()] = v.strip()
                path = target.partition("?")[0]
                # credentials before the body: an unauthenticated peer never gets a byte buffered.
                # An open path asked without credentials (a Prometheus scrape, a probe) is served
                # untrusted and not counted as a refused credential
                if path in OPEN_PATHS and not self.auth.presented(headers):
                    why = "NoCredentials" if self.auth.required else None
                else:
                    try:
                        why = self.auth.check_head(method, target, headers)
                    except Exception:  # a broken key file or verifier: refuse, never drop the thread
                        log.exception("agent RPC credential check failed")
                        why = "AuthError"
                authed = why is None
                if not authed and path not in OPEN_PATHS:
                    self._reject(conn, 401, why or "Unauthorized",
                                 "agent RPC requires the manager's signature or token", rf)
                    return
                cl = headers.get("content-length")
                if cl is None:
                    if method in BODY_METHODS:
                        self._reject(conn, 400, "BadRequest", "Content-Length required", rf)
                        return
                    n = 0
                elif not cl.isdigit() or not cl.isascii():  # no sign, no spaces, no hex
                    self._reject(conn, 400, "BadRequest", f"bad Content-Length {cl[:32]!r}", rf)
                    return
                else:
                    n = int(cl)
                if n > MAX_BODY:
                    self._reject(conn, 413, "PayloadTooLarge", f"body over {MAX_BODY} bytes", rf)
                    return
                try:
                    body = rf.read(n) if n else b""
                except _Closed as e:
                    if trusted and str(e) == "deadline":
                        self.request_deadline_closes += 1
                    return
                try:
                    bad_body = authed and self.auth.check_body(headers, body)
                except Exception:
                    log.exception("agent RPC body check failed")
                    bad_body = "AuthError"
                if bad_body:  # signed digest != body
                    self._reject(conn, 401, "BodyMismatch", "request body does not match its "
                                 "signature", rf)
                    return
                rf.deadline = None  # the request is in: its handling is not bounded
                keep = headers.get("connection", "").lower() != "close" and \
                    not version.strip().upper().endswith("1.0")
                if not trusted:
                    self._unwatch(raw)
                t0 = time.perf_counter()
                reply = self._dispatch(method, target, headers, body)
                if reply[0] == 401:
                    keep = False  # no second guess on this connection
                elif not authed:
                    # an open path answered without the token: it never earns a pooled slot
                    keep = False
                    self.open_path_closes += 1
                elif not trusted:
                    trusted = True  # a pooled keep-alive connection may idle from here
                try:
                    self._send(conn, reply, keep)
                    self._account(path, time.perf_counter() - t0)
                finally:
                    # the hook runs even when the peer is gone (e.g. a claim whose caller timed
                    # out): it ends the claim's event hold, which must never stay raised
                    if reply[3] is not None:
                        try:
                            reply[3]()
                        except Exception:
                            log.exception("post-reply hook failed")
                if not keep:
                    return
        except (OSError, ssl.SSLError, ValueError, _Closed):
            return
        finally:
            self._unwatch(raw)
            try:
                conn.close()
            except OSError:
                pass
            with self._conns_mu:
                self._conns -= 1
                self.bytes_read += rf.total if rf is not None else 0

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
               f"gpupool_agent_rpc_refused_connections_total {self.refused_conns}",
               f"gpupool_agent_rpc_deadline_closed_connections_total {self.reaped}",
               f"gpupool_agent_rpc_rejected_requests_total {self.rejected_requests}",
               f"gpupool_agent_rpc_open_path_closed_connections_total {self.open_path_closes}",
               f"gpupool_agent_rpc_request_deadline_closed_connections_total "
               f"{self.request_deadline_closes}"]
        out += self.auth.metrics_lines()
        for path, (n, sec) in items:
            out.append(f'gpupool_agent_rpc_requests_total{{path="{path}"}} {n}')
            out.append(f'gpupool_agent_rpc_seconds_sum{{path="{path}"}} {sec:.6f}')
        return out

    def _dispatch(self, method: str, target: str, headers: dict, body: bytes) -> tuple:
        path, _, qs = target.partition("?")
        self.requests += 1  # the token was checked in _serve_conn, before the body was read
        h = self.routes.get((method, path))
        if h is not None and self.guard is not None:
            refused = self.guard(method, path, headers)
            if refused is not None:
                return refused
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
