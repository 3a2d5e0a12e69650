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


def test_a_handler_slower_than_the_first_request_timeout_still_replies():
    """The deadline bounds receiving the first request, not handling it: an explicit scrub that
    maps a GPU's free HBM while the driver still clears its VRAM ran past 10 s on MI355X and the
    reaper cut its reply off (RemoteDisconnected, profiles/r4y_pytest_gpu_scrub_rpc_cut.txt)."""
    srv = RpcServer({("GET", "/v1/slow"): lambda q, b: (time.sleep(0.8), json_reply({"ok": True}))[1]},
                    first_request_timeout=0.3)
    srv.listen_tcp("127.0.0.1", 0)
    port = srv._listeners[-1].getsockname()[1]
    try:
        s = socket.create_connection(("127.0.0.1", port))
        s.settimeout(5.0)
        assert b"200" in _get(s, "/v1/slow")  # 0.8 s of handling on a fresh connection
        assert b"200" in _get(s, "/v1/slow")  # and the connection stays usable
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


def _raw(port: int) -> socket.socket:
    s = socket.create_connection(("127.0.0.1", port))
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    return s


def _status(sock: socket.socket, timeout: float = 5.0) -> bytes:
    sock.settimeout(timeout)
    buf = b""
    try:
        while b"\r\n" not in buf:
            chunk = sock.recv(4096)
            if not chunk:
                break
            buf += chunk
    except OSError:
        pass
    return buf.split(b"\r\n")[0]


def test_negative_content_length_from_an_unauthenticated_peer_reads_nothing():
    """Content-Length: -1 then 64 MiB from a client without the token: the server answers (401:
    the token is checked before the body) having read no more than 64 KiB, and closes."""
    import threading
    srv, port = _server(token="secret")
    try:
        s = _raw(port)
        s.sendall(b"POST /v1/claims HTTP/1.1\r\nHost: x\r\nContent-Length: -1\r\n\r\n")
        sent = [0]

        def flood():
            chunk = b"x" * (1 << 20)
            try:
                for _ in range(64):
                    s.sendall(chunk)
                    sent[0] += len(chunk)
            except OSError:
                pass
        t = threading.Thread(target=flood, daemon=True)
        t.start()
        assert _status(s).split(b" ")[1] in (b"400", b"401")
        t.join(timeout=10)
        assert _wait(lambda: srv.open_conns == 0)
        assert srv.bytes_read <= 64 << 10, srv.bytes_read
        s.close()
    finally:
        srv.close()


@pytest.mark.parametrize("cl", ["-1", "abc", "+5", "0x10", " 12 3"])
def test_bad_content_length_is_400_before_any_body(cl):
    srv, port = _server(token="secret")
    try:
        s = _raw(port)
        s.sendall(f"POST /v1/ping HTTP/1.1\r\nAuthorization: Bearer secret\r\n"
                  f"Content-Length: {cl}\r\n\r\n".encode() + b"y" * 4096)
        assert b"400" in _status(s)
        assert _closed(s, 3.0)
        s2 = _raw(port)  # a body-carrying method without Content-Length is refused too
        s2.sendall(b"POST /v1/ping HTTP/1.1\r\nAuthorization: Bearer secret\r\n\r\n")
        assert b"400" in _status(s2)
        s.close()
        s2.close()
    finally:
        srv.close()


def test_header_drip_is_closed_at_the_absolute_deadline():
    """One header byte every 1.5 s kept a per-recv timeout alive forever; the deadline is absolute:
    the connection closes first_request_timeout (2.0 s) after accept, +-0.5 s, and its slot is
    freed."""
    import threading
    srv, port = _server(first_request_timeout=2.0)
    try:
        s = _raw(port)
        t0 = time.monotonic()
        stop = threading.Event()

        def drip():
            for ch in b"GET /v1/ping HTTP/1.1\r\nX-Slow: " + b"a" * 64:
                try:
                    s.sendall(bytes([ch]))
                except OSError:
                    return
                if stop.wait(1.5):
                    return
        threading.Thread(target=drip, daemon=True).start()
        s.settimeout(6.0)
        try:
            got = s.recv(1)
        except OSError:
            got = b""
        elapsed = time.monotonic() - t0
        stop.set()
        assert got == b"", got
        assert 1.5 <= elapsed <= 2.5, elapsed
        assert _wait(lambda: srv.open_conns == 0)
        assert any(ln == "gpupool_agent_rpc_deadline_closed_connections_total 1" or
                   ln.startswith("gpupool_agent_rpc_deadline_closed_connections_total")
                   for ln in srv.metrics_lines())
        s.close()
    finally:
        srv.close()


def test_too_many_headers_are_refused():
    srv, port = _server()
    try:
        s = _raw(port)
        s.sendall(b"GET /v1/ping HTTP/1.1\r\n" + b"".join(f"X-{i}: v\r\n".encode() for i in range(200))
                  + b"\r\n")
        assert b"431" in _status(s)
        assert _closed(s, 3.0)
        s.close()
    finally:
        srv.close()


def test_post_reply_hook_runs_when_the_peer_is_gone():
    """A claim's reply hook ends its event hold (release_events): it must run even when writing the
    reply fails because the manager gave up and reset the connection."""
    import struct
    import threading
    ran = threading.Event()

    def slow(q, b):
        time.sleep(0.3)
        return json_reply({"ok": True}, after=ran.set)
    srv = RpcServer({("POST", "/v1/claims"): slow})
    srv.listen_tcp("127.0.0.1", 0)
    port = srv._listeners[-1].getsockname()[1]
    try:
        s = _raw(port)
        s.sendall(b"POST /v1/claims HTTP/1.1\r\nContent-Length: 2\r\n\r\n{}")
        s.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))
        s.close()  # RST: the server's write of the reply fails
        assert ran.wait(5.0)
        assert _wait(lambda: srv.open_conns == 0)
    finally:
        srv.close()


def _open_path_server(**kw) -> tuple[RpcServer, int]:
    from gpupool.agent.rpc import text_reply
    srv = RpcServer({("GET", "/v1/ping"): lambda q, b: json_reply({"ok": True}),
                     ("GET", "/healthz"): lambda q, b: text_reply("ok\n")}, **kw)
    srv.listen_tcp("127.0.0.1", 0)
    return srv, srv._listeners[-1].getsockname()[1]


def test_unauthenticated_open_path_requests_cannot_pin_connection_slots():
    """five unauthenticated clients each send a keep-alive GET /healthz and
    idle. Before, the 200 made each connection trusted and lifted its deadline (open_conns stayed
    5, reaped 0). Now an open path answered without the token closes its connection, so all are
    gone well within first_request_timeout + 0.5 s."""
    srv, port = _open_path_server(token="secret", first_request_timeout=1.0)
    socks = []
    try:
        t0 = time.monotonic()
        for _ in range(5):
            s = _raw(port)
            assert b"200" in _get(s, "/healthz")
            socks.append(s)
        assert all(_closed(s, 1.5) for s in socks)
        assert _wait(lambda: srv.open_conns == 0, 1.5)
        assert time.monotonic() - t0 <= 1.0 + 0.5 + 1.0  # 5 requests + the bound
        assert srv.open_path_closes == 5
        assert "gpupool_agent_rpc_open_path_closed_connections_total 5" in srv.metrics_lines()
    finally:
        for s in socks:
            s.close()
        srv.close()


def test_a_head_dripped_after_an_open_path_request_is_cut():
    """The second half of the repro: after GET /healthz the peer drips a second request head at
    1 byte per 0.1 s. The connection is closed after the first reply, so nothing it drips is read
    and its slot is free at once."""
    import threading
    srv, port = _open_path_server(token="secret", first_request_timeout=1.0)
    try:
        s = _raw(port)
        assert b"200" in _get(s, "/healthz")
        stop = threading.Event()

        def drip():
            for ch in b"GET /healthz HTTP/1.1\r\nX-Slow: " + b"a" * 200:
                try:
                    s.sendall(bytes([ch]))
                except OSError:
                    return
                if stop.wait(0.1):
                    return
        threading.Thread(target=drip, daemon=True).start()
        t0 = time.monotonic()
        assert _closed(s, 2.0)
        assert time.monotonic() - t0 <= 1.5
        stop.set()
        assert _wait(lambda: srv.open_conns == 0, 1.5)
    finally:
        srv.close()


def test_a_trusted_connection_cannot_drip_a_later_request():
    """After trust a connection may idle, but a request head that starts arriving must be in
    within first_request_timeout: a bearer-authenticated peer dripping its second head is cut."""
    import threading
    srv, port = _open_path_server(token="secret", first_request_timeout=1.0)
    try:
        s = _raw(port)
        assert b"200" in _get(s, "/v1/ping", token="secret")
        time.sleep(1.3)  # idling past the bound is fine
        stop = threading.Event()

        def drip():
            for ch in b"GET /v1/ping HTTP/1.1\r\nAuthorization: Bearer secret\r\nX-Slow: " + b"a" * 200:
                try:
                    s.sendall(bytes([ch]))
                except OSError:
                    return
                if stop.wait(0.1):
                    return
        threading.Thread(target=drip, daemon=True).start()
        t0 = time.monotonic()
        assert _closed(s, 3.0)
        assert 0.8 <= time.monotonic() - t0 <= 1.6
        stop.set()
        assert _wait(lambda: srv.open_conns == 0, 1.5)
        assert srv.request_deadline_closes == 1
    finally:
        srv.close()


def test_authenticated_open_path_request_keeps_the_connection():
    srv, port = _open_path_server(token="secret", first_request_timeout=0.3)
    try:
        s = _raw(port)
        assert b"200" in _get(s, "/healthz", token="secret")
        time.sleep(0.6)
        assert b"200" in _get(s, "/v1/ping", token="secret")
        s.close()
    finally:
        srv.close()
