"""The agent RPC server's exposure bounds (gpupool/agent/rpc.py): connection cap, first-request
timeout for connections that never send (or never finish a TLS handshake), a 401 closes the
connection, and a trusted keep-alive connection may idle past the first-request timeout."""
from __future__ import annotations

import socket
import time

import pytest

from gpupool.agent.rpc import RpcServer, json_reply


def _server(**kw) -> tuple[RpcServer, int]:
    srv = RpcServer({("GET", "/v1/ping"): lambda q, b: json_reply({"ok": True})}, **kw)
    srv.listen_tcp("127.0.0.1", 0)
    port = srv._listeners[-1].getsockname()[1]
    return srv, port


def _get(sock: socket.socket, path: str, token: str = "") -> bytes:
    auth = f"Authorization: Bearer {token}\r\n" if token else ""
    sock.sendall(f"GET {path} HTTP/1.1\r\nHost: x\r\n{auth}\r\n".encode())
    buf = b""
    while b"\r\n\r\n" not in buf:
        chunk = sock.recv(4096)
        if not chunk:
            break
        buf += chunk
    head, _, rest = buf.partition(b"\r\n\r\n")
    n = int([ln.split(b":")[1] for ln in head.split(b"\r\n") if ln.lower().startswith(b"content-length")][0])
    while len(rest) < n:
        rest += sock.recv(4096)
    return head.split(b"\r\n")[0] + b" " + rest


def _closed(sock: socket.socket, within: float) -> bool:
    sock.settimeout(within)
    try:
        return sock.recv(1) == b""
    except socket.timeout:
        return False
    except OSError:
        return True


def _wait(pred, timeout: float = 3.0) -> bool:
    end = time.time() + timeout
    while time.time() < end:
        if pred():
            return True
        time.sleep(0.01)
    return pred()


def test_silent_connection_is_dropped_after_the_first_request_timeout():
    srv, port = _server(first_request_timeout=0.3)
    try:
        s = socket.create_connection(("127.0.0.1", port))
        assert _closed(s, 3.0)  # never sent a request line
        assert _wait(lambda: srv.open_conns == 0)
    finally:
        srv.close()


def test_trusted_keep_alive_connection_may_idle():
    srv, port = _server(first_request_timeout=0.3)
    try:
        s = socket.create_connection(("127.0.0.1", port))
        assert b"200" in _get(s, "/v1/ping")
        time.sleep(0.8)  # idle well past the first-request timeout
        assert b"200" in _get(s, "/v1/ping")
        s.close()
    finally:
        srv.close()


def test_unauthorized_request_closes_the_connection():
    srv, port = _server(token="secret")
    try:
        s = socket.create_connection(("127.0.0.1", port))
        assert b"401" in _get(s, "/v1/ping", token="wrong")
        assert _closed(s, 3.0)
        s2 = socket.create_connection(("127.0.0.1", port))
        assert b"200" in _get(s2, "/v1/ping", token="secret")
        s2.close()
    finally:
        srv.close()


def test_connection_cap_refuses_extra_connections():
    srv, port = _server(max_conns=2, first_request_timeout=5.0)
    held = []
    try:
        held = [socket.create_connection(("127.0.0.1", port)) for _ in range(2)]
        assert _wait(lambda: srv.open_conns == 2)
        extra = socket.create_connection(("127.0.0.1", port))
        assert _closed(extra, 3.0)
        assert srv.refused_conns == 1
        assert any("gpupool_agent_rpc_refused_connections_total 1" == ln
                   for ln in srv.metrics_lines())
        for s in held:
            s.close()
        assert _wait(lambda: srv.open_conns == 0)
        s = socket.create_connection(("127.0.0.1", port))  # capacity is back
        assert b"200" in _get(s, "/v1/ping")
        s.close()
    finally:
        for s in held:
            s.close()
        srv.close()


@pytest.mark.parametrize("max_conns", [512])
def test_defaults(max_conns):
    srv = RpcServer({})
    assert srv.max_conns == max_conns and srv.first_request_timeout == 10.0
