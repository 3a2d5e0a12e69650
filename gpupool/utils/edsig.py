"""Ed25519 request signatures for the manager -> node-agent RPC (OpenSSL libcrypto via ctypes).

Why signatures and not a bearer token: a bearer token is a reusable credential. Sent to whatever
endpoint a Node names, it can be harvested by a rogue listener and replayed against every other
agent. Here the manager alone holds the private key; agents hold only public keys (non-secret,
a ConfigMap). Each request carries a signature bound to

    method, path + query, the target node's name, a timestamp, a nonce and the body's SHA-256

so what a wrong host receives is good for nothing but that one request to that one node within
the clock-skew window — and the agent keeps the nonces it has seen for that window. This is the
least-privilege identity the reference asks of its operator (an SP scoped to what it manages,
README.md:43-57; Workload Identity instead of shared secrets, README.md:59-60, 312).

Header (no ``Authorization`` header is sent at all)::

    X-Gpupool-Signature: v1 keyId=<16 hex> node=<node> ts=<unix ms> nonce=<32 hex>
                         body=<sha256 hex> sig=<base64url, no padding>

The C++ signer (native/src/runtime/agentauth.cc) produces the same bytes.

v2, the per-node MAC (what the manager sends once it knows the agent's key exchange key):
verifying an Ed25519 signature costs the agent ~0.17 ms of CPU per request, more than the rest of
its RPC overhead. Each agent keeps an X25519 key (``agent-kx.key`` in its state dir) and
publishes the public half on its Node (annotation ``gpupool.amd.com/agent-kx``, writable only by
that node's agent identity). The manager's X25519 key is its Ed25519 key seen on the Montgomery
curve (private: the Ed25519 secret scalar, SHA-512 of the seed; public: the Ed25519 public key
under the birational map), so agents derive it from the public keys they already trust and
nothing new is distributed. Both sides compute

    K = HMAC-SHA256(X25519(own private, peer public), "gpupool-agent-rpc-v2" | node | Xm | Xa)

once, and every request then carries ``HMAC-SHA256(K, canonical)`` (~2 us to check) over the
same canonical string as v1 (with the v2 prefix)::

    X-Gpupool-Signature: v2 keyId=<manager key id> kx=<16 hex of sha256(Xa)> node=<node>
                         ts=<unix ms> nonce=<32 hex> body=<sha256 hex> mac=<base64url>

Only the manager and that node's agent can compute K: a MAC for node B is worthless at node A,
replays are refused as in v1, and an agent restarted with another key answers ``StaleAgentKey``
(the key is kept in the state dir, so a restart does not change it).
"""
from __future__ import annotations

import base64
import ctypes
import ctypes.util
import hashlib
import hmac
import os
import threading
import time

HEADER = "x-gpupool-signature"
PREFIX = b"gpupool-agent-rpc-v1"
PREFIX2 = b"gpupool-agent-rpc-v2"
_NID_ED25519 = 1087
_NID_X25519 = 1034
_P = 2 ** 255 - 19
# DER prefixes of an Ed25519 PKCS#8 private key (RFC 8410) and SubjectPublicKeyInfo
_PRIV_DER = bytes.fromhex("302e020100300506032b657004220420")
_PUB_DER = bytes.fromhex("302a300506032b6570032100")

_lib = None
_lib_mu = threading.Lock()


def _crypto():
    global _lib
    with _lib_mu:
        if _lib is None:
            name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
            lib = ctypes.CDLL(name)
            vp, cp, sz = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t
            lib.EVP_PKEY_new_raw_public_key.restype = vp
            lib.EVP_PKEY_new_raw_public_key.argtypes = [ctypes.c_int, vp, cp, sz]
            lib.EVP_PKEY_new_raw_private_key.restype = vp
            lib.EVP_PKEY_new_raw_private_key.argtypes = [ctypes.c_int, vp, cp, sz]
            lib.EVP_PKEY_free.argtypes = [vp]
            lib.EVP_MD_CTX_new.restype = vp
            lib.EVP_MD_CTX_free.argtypes = [vp]
            lib.EVP_DigestVerifyInit.argtypes = [vp, vp, vp, vp, vp]
            lib.EVP_DigestVerify.argtypes = [vp, cp, sz, cp, sz]
            lib.EVP_DigestSignInit.argtypes = [vp, vp, vp, vp, vp]
            lib.EVP_DigestSign.argtypes = [vp, cp, ctypes.POINTER(sz), cp, sz]
            lib.EVP_PKEY_get_raw_public_key.argtypes = [vp, cp, ctypes.POINTER(sz)]
            lib.EVP_PKEY_CTX_new.restype = vp
            lib.EVP_PKEY_CTX_new.argtypes = [vp, vp]
            lib.EVP_PKEY_CTX_free.argtypes = [vp]
            lib.EVP_PKEY_derive_init.argtypes = [vp]
            lib.EVP_PKEY_derive_set_peer.argtypes = [vp, vp]
            lib.EVP_PKEY_derive.argtypes = [vp, cp, ctypes.POINTER(sz)]
            _lib = lib
        return _lib


def _pem_body(pem: str, label: str) -> bytes:
    begin, end = f"-----BEGIN {label}-----", f"-----END {label}-----"
    i, j = pem.find(begin), pem.find(end)
    if i < 0 or j < 0:
        raise ValueError(f"no {label} PEM block")
    return base64.b64decode("".join(pem[i + len(begin):j].split()))


def load_private_key(pem: str) -> bytes:
    """The 32-byte seed of an Ed25519 ``PRIVATE KEY`` PEM (``openssl genpkey -algorithm ed25519``)."""
    der = _pem_body(pem, "PRIVATE KEY")
    if not der.startswith(_PRIV_DER) or len(der) != len(_PRIV_DER) + 32:
        raise ValueError("not an Ed25519 PKCS#8 private key")
    return der[len(_PRIV_DER):]


def load_public_keys(pem: str) -> list[bytes]:
    """Every Ed25519 ``PUBLIC KEY`` block of a PEM bundle, as raw 32-byte keys."""
    out, rest = [], pem
    while "-----BEGIN PUBLIC KEY-----" in rest:
        der = _pem_body(rest, "PUBLIC KEY")
        if not der.startswith(_PUB_DER) or len(der) != len(_PUB_DER) + 32:
            raise ValueError("not an Ed25519 public key")
        out.append(der[len(_PUB_DER):])
        rest = rest[rest.index("-----END PUBLIC KEY-----") + 24:]
    return out


def private_pem(seed: bytes) -> str:
    """A 32-byte seed as an Ed25519 PKCS#8 ``PRIVATE KEY`` PEM (what ``openssl genpkey`` writes);
    a fresh key is ``private_pem(os.urandom(32))`` — any 32 bytes are an Ed25519 seed."""
    if len(seed) != 32:
        raise ValueError("an Ed25519 seed is 32 bytes")
    b = base64.b64encode(_PRIV_DER + seed).decode()
    return "-----BEGIN PRIVATE KEY-----\n" + b + "\n-----END PRIVATE KEY-----\n"


def public_pem(raw: bytes) -> str:
    b = base64.b64encode(_PUB_DER + raw).decode()
    return "-----BEGIN PUBLIC KEY-----\n" + b + "\n-----END PUBLIC KEY-----\n"


def key_id(pub: bytes) -> str:
    return hashlib.sha256(pub).hexdigest()[:16]


def public_from_private(seed: bytes, nid: int = _NID_ED25519) -> bytes:
    lib = _crypto()
    k = lib.EVP_PKEY_new_raw_private_key(nid, None, seed, len(seed))
    if not k:
        raise ValueError("bad private key")
    try:
        buf = ctypes.create_string_buffer(32)
        n = ctypes.c_size_t(32)
        if lib.EVP_PKEY_get_raw_public_key(k, buf, ctypes.byref(n)) != 1:
            raise ValueError("EVP_PKEY_get_raw_public_key failed")
        return buf.raw[:n.value]
    finally:
        lib.EVP_PKEY_free(k)


# ---------------------------------------------------------------- v2: X25519 + HMAC
def x25519_from_ed25519_public(pub: bytes) -> bytes:
    """The Montgomery u-coordinate of an Ed25519 public key: u = (1 + y) / (1 - y) mod p."""
    if len(pub) != 32:
        raise ValueError("an Ed25519 public key is 32 bytes")
    y = int.from_bytes(pub, "little") & ((1 << 255) - 1)
    u = (1 + y) * pow((1 - y) % _P, _P - 2, _P) % _P
    return u.to_bytes(32, "little")


def x25519_private_from_ed25519_seed(seed: bytes) -> bytes:
    """The Ed25519 secret scalar (SHA-512 of the seed, first half; X25519 clamps it the same
    way Ed25519 does), so the two public keys are one point on two curves."""
    return hashlib.sha512(seed).digest()[:32]


def x25519_public(priv: bytes) -> bytes:
    return public_from_private(priv, _NID_X25519)


def x25519(priv: bytes, peer: bytes) -> bytes:
    """The X25519 shared secret (OpenSSL refuses an all-zero result: a low-order peer key)."""
    lib = _crypto()
    k = lib.EVP_PKEY_new_raw_private_key(_NID_X25519, None, priv, len(priv))
    pk = lib.EVP_PKEY_new_raw_public_key(_NID_X25519, None, peer, len(peer))
    ctx = lib.EVP_PKEY_CTX_new(k, None) if k else None
    try:
        if not (k and pk and ctx) or lib.EVP_PKEY_derive_init(ctx) != 1 or \
                lib.EVP_PKEY_derive_set_peer(ctx, pk) != 1:
            raise ValueError("X25519 key agreement failed")
        buf = ctypes.create_string_buffer(32)
        n = ctypes.c_size_t(32)
        if lib.EVP_PKEY_derive(ctx, buf, ctypes.byref(n)) != 1:
            raise ValueError("X25519 key agreement failed")
        return buf.raw[:n.value]
    finally:
        if ctx:
            lib.EVP_PKEY_CTX_free(ctx)
        for x in (k, pk):
            if x:
                lib.EVP_PKEY_free(x)


def kx_id(agent_x: bytes) -> str:
    return hashlib.sha256(agent_x).hexdigest()[:16]


def mac_key(shared: bytes, node: str, manager_x: bytes, agent_x: bytes) -> bytes:
    return hmac.new(shared, PREFIX2 + b"\n" + node.encode() + b"\n" + manager_x + agent_x,
                    hashlib.sha256).digest()


def mac_header(key: bytes, kid: str, agent_x: bytes, method: str, target: str, node: str,
               body: bytes = b"", ts_ms: int | None = None, nonce: str | None = None) -> str:
    """The v2 header for one request to ``node`` under the per-node key ``key``."""
    ts_ms = int(time.time() * 1000) if ts_ms is None else ts_ms
    nonce = nonce or os.urandom(16).hex()
    sha = hashlib.sha256(body).hexdigest()
    mac = hmac.new(key, canonical(method, target, node, ts_ms, nonce, sha, PREFIX2),
                   hashlib.sha256).digest()
    return (f"v2 keyId={kid} kx={kx_id(agent_x)} node={node} ts={ts_ms} nonce={nonce} body={sha} "
            f"mac={_b64u(mac)}")


class AgentKx:
    """The agent's X25519 key, kept (0600) in its state dir so a restart keeps it."""

    def __init__(self, path: str):
        self.path = path
        try:
            with open(path, "rb") as f:
                priv = f.read()
        except FileNotFoundError:
            priv = b""
        if len(priv) != 32:
            priv = os.urandom(32)
            tmp = path + ".tmp"
            fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
            with os.fdopen(fd, "wb") as f:
                f.write(priv)
                f.flush()
                os.fsync(f.fileno())
            os.replace(tmp, path)
        self.private = priv
        self.public = x25519_public(priv)
        self.id = kx_id(self.public)

    def annotation(self) -> str:
        return _b64u(self.public)


def sign_raw(seed: bytes, msg: bytes) -> bytes:
    lib = _crypto()
    k = lib.EVP_PKEY_new_raw_private_key(_NID_ED25519, None, seed, len(seed))
    ctx = lib.EVP_MD_CTX_new()
    try:
        if not k or lib.EVP_DigestSignInit(ctx, None, None, None, k) != 1:
            raise ValueError("EVP_DigestSignInit failed")
        sig = ctypes.create_string_buffer(64)
        n = ctypes.c_size_t(64)
        if lib.EVP_DigestSign(ctx, sig, ctypes.byref(n), msg, len(msg)) != 1:
            raise ValueError("EVP_DigestSign failed")
        return sig.raw[:n.value]
    finally:
        lib.EVP_MD_CTX_free(ctx)
        if k:
            lib.EVP_PKEY_free(k)


class PublicKey:
    """A parsed Ed25519 public key (the EVP_PKEY is built once, not per verification)."""

    def __init__(self, raw: bytes):
        self.raw = raw
        self._lib = _crypto()
        self._k = self._lib.EVP_PKEY_new_raw_public_key(_NID_ED25519, None, raw, len(raw))
        if not self._k:
            raise ValueError("bad Ed25519 public key")

    def verify(self, msg: bytes, sig: bytes) -> bool:
        lib = self._lib
        ctx = lib.EVP_MD_CTX_new()
        try:
            if lib.EVP_DigestVerifyInit(ctx, None, None, None, self._k) != 1:
                return False
            return lib.EVP_DigestVerify(ctx, sig, len(sig), msg, len(msg)) == 1
        finally:
            lib.EVP_MD_CTX_free(ctx)

    def __del__(self):
        if getattr(self, "_k", None):
            self._lib.EVP_PKEY_free(self._k)
            self._k = None


def verify_raw(pub: bytes, msg: bytes, sig: bytes) -> bool:
    try:
        return PublicKey(pub).verify(msg, sig)
    except ValueError:
        return False


def canonical(method: str, target: str, node: str, ts_ms: int, nonce: str, body_sha: str,
              prefix: bytes = PREFIX) -> bytes:
    return b"\n".join([prefix, method.upper().encode(), target.encode(), node.encode(),
                       str(ts_ms).encode(), nonce.encode(), body_sha.encode()])


def _b64u(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).decode().rstrip("=")


def _unb64u(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def sign_header(seed: bytes, method: str, target: str, node: str, body: bytes = b"",
                ts_ms: int | None = None, nonce: str | None = None,
                pub: bytes | None = None) -> str:
    """The ``X-Gpupool-Signature`` value for one request to ``node``."""
    ts_ms = int(time.time() * 1000) if ts_ms is None else ts_ms
    nonce = nonce or os.urandom(16).hex()
    sha = hashlib.sha256(body).hexdigest()
    sig = sign_raw(seed, canonical(method, target, node, ts_ms, nonce, sha))
    kid = key_id(pub or public_from_private(seed))
    return f"v1 keyId={kid} node={node} ts={ts_ms} nonce={nonce} body={sha} sig={_b64u(sig)}"


def parse_header(value: str) -> dict[str, str] | None:
    parts = value.split()
    if not parts or parts[0] not in ("v1", "v2"):
        return None
    out = {"v": parts[0]}
    for p in parts[1:]:
        k, sep, v = p.partition("=")
        if not sep:
            return None
        out[k] = v
    need = {"keyId", "node", "ts", "nonce", "body"} | ({"sig"} if parts[0] == "v1" else
                                                       {"mac", "kx"})
    return out if need <= set(out) else None


class Signer:
    """A private key file, re-read when it changes (key rotation on the manager side)."""

    def __init__(self, path: str, reload_s: float = 5.0):
        self.path = path
        self.reload_s = reload_s
        self._mu = threading.Lock()
        self._checked = -1e9
        self._mtime = None
        self.seed = b""
        self.pub = b""
        self._load(force=True)

    def _load(self, force: bool = False) -> None:
        now = time.monotonic()
        if not force and now - self._checked < self.reload_s:
            return
        self._checked = now
        try:
            st = os.stat(self.path)
        except OSError:
            return
        if not force and st.st_mtime_ns == self._mtime:
            return
        with open(self.path) as f:
            seed = load_private_key(f.read())
        self.seed, self.pub, self._mtime = seed, public_from_private(seed), st.st_mtime_ns

    def header(self, method: str, target: str, node: str, body: bytes = b"") -> str:
        with self._mu:
            self._load()
            seed, pub = self.seed, self.pub
        return sign_header(seed, method, target, node, body, pub=pub)


class Verifier:
    """The agent side: trusted public keys (a PEM bundle file, or a directory of them — the
    mounted ConfigMap — re-read when it changes: during a rotation it lists the old and the new
    key), this node's name, the clock-skew window and the nonces seen inside it."""

    def __init__(self, path: str, node: str, skew_s: float = 60.0, reload_s: float = 1.0,
                 kx: AgentKx | None = None):
        self.path = path
        self.node = node
        self.skew_ms = int(skew_s * 1000)
        self.reload_s = reload_s
        self.keys: dict[str, PublicKey] = {}
        self._sig = None
        self._checked = -1e9
        self._mu = threading.Lock()
        self._nonces: dict[str, int] = {}
        self._nonce_prune_at = 4096
        self.rejected: dict[str, int] = {}
        self.accepted: dict[str, int] = {}  # key id -> requests it signed (rotation progress)
        self.kx = kx  # v2: this agent's X25519 key; per manager key id the MAC key, derived once
        self._mac_keys: dict[str, bytes] = {}
        self.by_version: dict[str, int] = {}
        self._load(force=True)

    def _files(self) -> list[str]:
        if os.path.isdir(self.path):
            return sorted(os.path.join(self.path, f) for f in os.listdir(self.path)
                          if not f.startswith("."))
        return [self.path]

    def _load(self, force: bool = False) -> None:
        now = time.monotonic()
        if not force and now - self._checked < self.reload_s:
            return
        self._checked = now
        try:
            files = [f for f in self._files() if os.path.isfile(f)]
            sig = tuple((f, os.stat(f).st_mtime_ns) for f in files)
        except OSError:
            return
        if sig == self._sig and not force:
            return
        keys = {}
        for f in files:
            try:
                with open(f) as fh:
                    for k in load_public_keys(fh.read()):
                        keys[key_id(k)] = PublicKey(k)
            except (OSError, ValueError):
                continue
        if keys or force:
            self.keys, self._sig = keys, sig

    def trusted(self) -> list[str]:
        """Ids of the public keys currently trusted (re-read from the bundle first)."""
        with self._mu:
            self._load()
            return sorted(self.keys)

    def _reject(self, why: str) -> str:
        self.rejected[why] = self.rejected.get(why, 0) + 1
        return why

    def check_head(self, method: str, target: str, headers: dict) -> str | None:
        """Before the body: None when the signature is valid for this node (the body digest it
        names is checked by ``check_body``), else why not."""
        raw = headers.get(HEADER)
        if not raw:
            return self._reject("NoSignature")
        h = parse_header(raw)
        if h is None:
            return self._reject("BadSignatureHeader")
        if h["node"] != self.node:
            return self._reject("WrongNode")
        try:
            ts = int(h["ts"])
        except ValueError:
            return self._reject("BadSignatureHeader")
        now = int(time.time() * 1000)
        if abs(now - ts) > self.skew_ms:
            return self._reject("StaleSignature")
        with self._mu:
            self._load()
            pub = self.keys.get(h["keyId"])
        if pub is None:
            return self._reject("UnknownKey")
        try:
            sig = _unb64u(h["sig"] if h["v"] == "v1" else h["mac"])
        except ValueError:
            return self._reject("BadSignatureHeader")
        if h["v"] == "v1":
            if not pub.verify(canonical(method, target, self.node, ts, h["nonce"], h["body"]), sig):
                return self._reject("BadSignature")
        else:
            if self.kx is None:
                return self._reject("NoAgentKey")
            if h["kx"] != self.kx.id:
                return self._reject("StaleAgentKey")
            key = self._mac_key(h["keyId"], pub)
            want = hmac.new(key, canonical(method, target, self.node, ts, h["nonce"], h["body"],
                                           PREFIX2), hashlib.sha256).digest()
            if not hmac.compare_digest(want, sig):
                return self._reject("BadSignature")
        with self._mu:
            self.by_version[h["v"]] = self.by_version.get(h["v"], 0) + 1
            if h["nonce"] in self._nonces:
                return self._reject("Replay")
            self._nonces[h["nonce"]] = ts + self.skew_ms
            self.accepted[h["keyId"]] = self.accepted.get(h["keyId"], 0) + 1
            if len(self._nonces) > self._nonce_prune_at:
                # keep a nonce while its timestamp still passes the skew check (now <= ts+skew);
                # a burst that keeps more than that alive moves the next prune out (amortised
                # O(1) per request instead of a full sweep on every one)
                self._nonces = {n: e for n, e in self._nonces.items() if e >= now}
                self._nonce_prune_at = max(4096, 2 * len(self._nonces))
        return None

    def _mac_key(self, kid: str, pub: PublicKey) -> bytes:
        key = self._mac_keys.get(kid)
        if key is None:
            xm = x25519_from_ed25519_public(pub.raw)
            key = mac_key(x25519(self.kx.private, xm), self.node, xm, self.kx.public)
            with self._mu:
                self._mac_keys[kid] = key
        return key

    def check_body(self, headers: dict, body: bytes) -> str | None:
        h = parse_header(headers.get(HEADER, "")) or {}
        if h.get("body") != hashlib.sha256(body).hexdigest():
            return self._reject("BodyMismatch")
        return None
