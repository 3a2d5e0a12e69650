"""Manager -> agent request signatures (gpupool/utils/edsig.py; the C++ signer in
native/src/runtime/agentauth.cc): a signature is good for one request to one node, once, within
the skew window; key rotation through the agents' public-key bundle; the RPC server refuses
unsigned / wrong-node / replayed / tampered requests before reading their bodies."""
from __future__ import annotations

import json
import os
import subprocess
import time

import pytest

from gpupool.agent.auth import AgentAuth, TokenAuth
from gpupool.agent.rpc import RpcServer, json_reply
from gpupool.kube import Client, KubeError
from gpupool.testing.cluster import make_signing_key
from gpupool.utils import edsig


@pytest.fixture
def keys(tmp_path):
    k1, p1 = make_signing_key(str(tmp_path), "k1")
    k2, p2 = make_signing_key(str(tmp_path), "k2")
    return {"k1": k1, "p1": p1, "k2": k2, "p2": p2, "dir": tmp_path}


def hdr(signer, method, target, node, body=b""):
    return {edsig.HEADER: signer.header(method, target, node, body)}


def test_signature_is_bound_to_request_node_and_time(keys):
    s = edsig.Signer(keys["k1"])
    v_b = edsig.Verifier(keys["p1"], "node-b")
    v_a = edsig.Verifier(keys["p1"], "node-a")
    h = hdr(s, "POST", "/v1/claims", "node-b", b'{"count":1}')
    assert v_a.check_head("POST", "/v1/claims", dict(h)) == "WrongNode"   # another agent
    assert v_b.check_head("POST", "/v1/release", dict(h)) == "BadSignature"  # another request
    assert v_b.check_head("POST", "/v1/claims", dict(h)) is None
    assert v_b.check_body(h, b'{"count":8}') == "BodyMismatch"          # tampered body
    assert v_b.check_body(h, b'{"count":1}') is None
    assert v_b.check_head("POST", "/v1/claims", dict(h)) == "Replay"      # once only
    old = {edsig.HEADER: edsig.sign_header(s.seed, "GET", "/v1/node", "node-b",
                                           ts_ms=int(time.time() * 1000) - 120_000)}
    assert v_b.check_head("GET", "/v1/node", old) == "StaleSignature"
    other = edsig.Signer(keys["k2"])
    assert v_b.check_head("GET", "/v1/node", hdr(other, "GET", "/v1/node", "node-b")) == "UnknownKey"
    assert v_b.check_head("GET", "/v1/node", {}) == "NoSignature"


def test_nonce_cache_under_a_burst_inside_the_skew_window(keys):
    """More live nonces than the prune threshold: every fresh request passes, every replay of
    one still inside the window is refused, and the sweep is not repeated on each request."""
    s = edsig.Signer(keys["k1"])
    v = edsig.Verifier(keys["p1"], "node-b")
    v._nonce_prune_at = 64  # the production threshold (4096) scaled down for the test's speed
    sent = [hdr(s, "GET", f"/v1/node?i={i}", "node-b") for i in range(300)]
    assert all(v.check_head("GET", f"/v1/node?i={i}", dict(h)) is None for i, h in enumerate(sent))
    assert v._nonce_prune_at >= 2 * 64  # all 300 alive: the threshold moved out
    assert len(v._nonces) == 300
    assert all(v.check_head("GET", f"/v1/node?i={i}", dict(sent[i])) == "Replay"
               for i in (0, 63, 64, 299))


def test_key_rotation_through_the_bundle(keys):
    bundle = keys["dir"] / "bundle"
    bundle.mkdir()
    (bundle / "a.pem").write_text(open(keys["p1"]).read())
    v = edsig.Verifier(str(bundle), "n", reload_s=0)
    s1, s2 = edsig.Signer(keys["k1"]), edsig.Signer(keys["k2"])
    assert v.check_head("GET", "/v1/node", hdr(s1, "GET", "/v1/node", "n")) is None
    assert v.check_head("GET", "/v1/node", hdr(s2, "GET", "/v1/node", "n")) == "UnknownKey"
    (bundle / "b.pem").write_text(open(keys["p2"]).read())   # 1. agents learn the new key
    assert v.check_head("GET", "/v1/node", hdr(s2, "GET", "/v1/node", "n")) is None
    assert v.check_head("GET", "/v1/node", hdr(s1, "GET", "/v1/node", "n")) is None
    os.unlink(bundle / "a.pem")                               # 3. the old key retires
    assert v.check_head("GET", "/v1/node", hdr(s1, "GET", "/v1/node", "n")) == "UnknownKey"
    # the manager side re-reads its key file when it changes (2. the swap)
    live = keys["dir"] / "live.key"
    live.write_text(open(keys["k1"]).read())
    s = edsig.Signer(str(live), reload_s=0)
    kid1 = edsig.key_id(s.pub)
    time.sleep(0.01)
    live.write_text(open(keys["k2"]).read())
    os.utime(live, ns=(time.time_ns(), time.time_ns() + 10_000_000))
    s.header("GET", "/", "n")
    assert edsig.key_id(s.pub) != kid1


def test_cpp_signer_matches_python_verifier(keys, native_built):
    """The manager's C++ AgentSigner and the agent's Python verifier agree byte for byte
    (gpupool_tests prints one signature for fixed inputs)."""
    exe = os.path.join(native_built, "gpupool_tests")
    out = subprocess.run([exe, "--sign", keys["k1"], "POST", "/v1/claims?x=1", "node-b",
                          '{"a":1}'], capture_output=True, text=True, timeout=30)
    assert out.returncode == 0, out.stderr
    line = out.stdout.strip()
    assert line.startswith("X-Gpupool-Signature: v1 ")
    h = {edsig.HEADER: line.split(": ", 1)[1]}
    v = edsig.Verifier(keys["p1"], "node-b")
    assert v.check_head("POST", "/v1/claims?x=1", dict(h)) is None
    assert v.check_body(h, b'{"a":1}') is None


def test_cpp_mac_matches_python_verifier(keys, native_built, tmp_path):
    """v2: the C++ signer derives the same per-node MAC key from the agent's X25519 key as the
    agent does from the manager's Ed25519 public key (one point on two curves); a MAC for
    another node, another agent key or a tampered request is refused."""
    exe = os.path.join(native_built, "gpupool_tests")
    kx = edsig.AgentKx(str(tmp_path / "agent-kx.key"))
    out = subprocess.run([exe, "--sign", keys["k1"], "POST", "/v1/claims?x=1", "node-b",
                          '{"a":1}', kx.annotation()], capture_output=True, text=True, timeout=30)
    assert out.returncode == 0, out.stderr
    line = out.stdout.strip()
    assert line.startswith("X-Gpupool-Signature: v2 ") and f"kx={kx.id}" in line
    h = {edsig.HEADER: line.split(": ", 1)[1]}
    v = edsig.Verifier(keys["p1"], "node-b", kx=kx)
    assert v.check_head("POST", "/v1/claims?x=1", dict(h)) is None
    assert v.check_body(h, b'{"a":1}') is None
    assert v.by_version == {"v2": 1}
    assert v.check_head("POST", "/v1/claims?x=1", dict(h)) == "Replay"
    assert edsig.Verifier(keys["p1"], "node-b", kx=edsig.AgentKx(str(tmp_path / "o.key"))) \
        .check_head("POST", "/v1/claims?x=1", dict(h)) == "StaleAgentKey"
    assert edsig.Verifier(keys["p1"], "node-b").check_head("POST", "/v1/claims?x=1", dict(h)) \
        == "NoAgentKey"
    out = subprocess.run([exe, "--sign", keys["k1"], "POST", "/v1/release", "node-b", "{}",
                          kx.annotation()], capture_output=True, text=True, timeout=30)
    h2 = {edsig.HEADER: out.stdout.strip().split(": ", 1)[1]}
    assert v.check_head("POST", "/v1/claims", dict(h2)) == "BadSignature"  # another target
    # the Ed25519 -> X25519 map: the manager's X25519 public key from its seed and the agent's
    # from the Ed25519 public key it trusts are the same bytes
    seed = edsig.load_private_key(open(keys["k1"]).read())
    assert edsig.x25519_public(edsig.x25519_private_from_ed25519_seed(seed)) == \
        edsig.x25519_from_ed25519_public(edsig.public_from_private(seed))


def _server(auth):
    routes = {("POST", "/v1/claims"): lambda q, b: json_reply({"ok": True, "n": len(b)}),
              ("GET", "/v1/node"): lambda q, b: json_reply({"node": "node-b"})}
    srv = RpcServer(routes, auth=auth)
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv.listen_tcp("127.0.0.1", port)
    return srv, f"http://127.0.0.1:{port}"


def test_rpc_server_with_signatures_and_rotating_token(keys):
    tok = keys["dir"] / "token"
    tok.write_text("t1\n")
    auth = AgentAuth(edsig.Verifier(keys["p1"], "node-b"), TokenAuth(path=str(tok), grace_s=60,
                                                                     reload_s=0))
    srv, url = _server(auth)
    try:
        s = edsig.Signer(keys["k1"])
        c = Client(url)
        body = {"count": 1}
        raw = json.dumps(body).encode()
        assert c.request("POST", "/v1/claims", body, extra_headers={
            "X-Gpupool-Signature": s.header("POST", "/v1/claims", "node-b", raw)})["ok"]
        for bad in ({"X-Gpupool-Signature": s.header("POST", "/v1/claims", "node-a", raw)},
                    {"X-Gpupool-Signature": s.header("POST", "/v1/claims", "node-b", b"{}")}, {}):
            with pytest.raises(KubeError) as ei:
                c.request("POST", "/v1/claims", body, extra_headers=bad)
            assert ei.value.code == 401
        # the shared token rotates: the old one keeps working for the grace period
        assert Client(url, "t1").request("GET", "/v1/node")["node"] == "node-b"
        time.sleep(0.01)
        tok.write_text("t2\n")
        os.utime(tok, ns=(time.time_ns(), time.time_ns() + 10_000_000))
        assert Client(url, "t2").request("GET", "/v1/node")["node"] == "node-b"
        assert Client(url, "t1").request("GET", "/v1/node")["node"] == "node-b"
        auth.token.previous = [(t, 0.0) for t, _ in auth.token.previous]  # grace over
        with pytest.raises(KubeError):
            Client(url, "t1").request("GET", "/v1/node")
        m = "\n".join(srv.metrics_lines())
        assert 'result="signature"' in m and 'result="rejected_WrongNode"' in m
    finally:
        srv.close()


def test_a_credential_check_that_raises_is_a_refusal_not_a_dropped_connection(keys):
    """A verifier that throws (a corrupt key bundle, a bug) answers 401 AuthError: the caller
    learns why, and the connection thread does not die with the exception."""
    class Broken(AgentAuth):
        def check_head(self, method, target, headers):
            raise AttributeError("verifier state")

    srv, url = _server(Broken(edsig.Verifier(keys["p1"], "node-b")))
    try:
        with pytest.raises(KubeError) as ei:
            Client(url).request("POST", "/v1/claims", {"count": 1}, extra_headers={
                "X-Gpupool-Signature": "v1 keyId=x node=node-b ts=1 nonce=n body=b sig=s"})
        assert ei.value.code == 401 and ei.value.reason == "AuthError"
    finally:
        srv.close()
