"""Who may call the agent's RPC (the manager, an admin's gpuctl), checked by rpc.RpcServer before
a request's body is read.

Two credentials, either or both configured:

* **Request signatures** (``--manager-pubkeys``, the default deployment): the manager signs every
  request for one node with its Ed25519 key (gpupool/utils/edsig.py). No reusable secret ever
  travels, so an endpoint that is not the node's agent learns nothing it could replay elsewhere.
* **A shared bearer token** (``--auth-token-file``, for clusters not yet migrated): the file is
  re-read when it changes; during a rotation the previous token stays valid for ``grace_s``, so a
  manager that has not picked up the new one yet keeps working (client-go's projected-token
  behaviour on the other side).
"""
from __future__ import annotations

import hmac
import os
import threading
import time

from ..utils import edsig


class TokenAuth:
    def __init__(self, token: str = "", path: str = "", grace_s: float = 300.0,
                 reload_s: float = 1.0):
        self.path = path
        self.grace_s = grace_s
        self.reload_s = reload_s
        self._mu = threading.Lock()
        self._checked = -1e9
        self._mtime = None
        self.current = token.encode()
        self.previous: list[tuple[bytes, float]] = []  # (token, valid until monotonic)
        self.rotations = 0
        if path:
            self._load(force=True)

    def _load(self, force: bool = False) -> None:
        now = time.monotonic()
        if not self.path or (not force and now - self._checked < self.reload_s):
            return
        self._checked = now
        try:
            st = os.stat(self.path)
            if not force and st.st_mtime_ns == self._mtime:
                return
            with open(self.path) as f:
                tok = f.read().strip().encode()
        except OSError:
            return  # mid-swap: keep what we have
        self._mtime = st.st_mtime_ns
        if tok and tok != self.current:
            if self.current:
                self.previous = [(t, u) for t, u in self.previous if u > now] + \
                    [(self.current, now + self.grace_s)]
                self.rotations += 1
            self.current = tok

    def check_head(self, method: str, target: str, headers: dict) -> str | None:
        with self._mu:
            self._load()
            want = [self.current] + [t for t, u in self.previous if u > time.monotonic()]
        got = headers.get("authorization", "").encode()
        if any(t and hmac.compare_digest(got, b"Bearer " + t) for t in want):
            return None
        return "BadToken" if got else "NoToken"

    def check_body(self, headers: dict, body: bytes) -> str | None:
        return None


class AgentAuth:
    """Any configured credential admits a request; with none configured every request passes
    (a unix socket only root can reach, tests)."""

    def __init__(self, verifier: edsig.Verifier | None = None, token: TokenAuth | None = None):
        self.verifier = verifier
        self.token = token
        self.stats: dict[str, int] = {}

    @property
    def required(self) -> bool:
        return self.verifier is not None or self.token is not None

    @staticmethod
    def presented(headers: dict) -> bool:
        """Does the request carry any credential at all?"""
        return edsig.HEADER in headers or "authorization" in headers

    def check_head(self, method: str, target: str, headers: dict) -> str | None:
        if not self.required:
            return None
        why = []
        if self.verifier is not None and edsig.HEADER in headers:
            r = self.verifier.check_head(method, target, headers)
            if r is None:
                headers["_auth"] = "signature"
                self._count("signature")
                return None
            why.append(r)
        if self.token is not None and "authorization" in headers:
            r = self.token.check_head(method, target, headers)
            if r is None:
                headers["_auth"] = "token"
                self._count("token")
                return None
            why.append(r)
        reason = why[0] if why else "NoCredentials"
        self._count("rejected_" + reason)
        return reason

    def check_body(self, headers: dict, body: bytes) -> str | None:
        if headers.get("_auth") == "signature":
            r = self.verifier.check_body(headers, body)
            if r:
                self._count("rejected_" + r)
            return r
        return None

    def _count(self, k: str) -> None:
        self.stats[k] = self.stats.get(k, 0) + 1

    def metrics_lines(self) -> list[str]:
        out = [f'gpupool_agent_rpc_auth_total{{result="{k}"}} {v}'
               for k, v in sorted(self.stats.items())]
        if self.verifier is not None:  # key rotation: what this agent trusts and sees in use
            out += [f'gpupool_agent_trusted_key{{keyId="{k}"}} 1' for k in self.verifier.trusted()]
            out += [f'gpupool_agent_rpc_signatures_total{{keyId="{k}"}} {v}'
                    for k, v in sorted(self.verifier.accepted.items())]
            # v1: Ed25519 signature; v2: the per-node MAC (edsig.py)
            out += [f'gpupool_agent_rpc_signature_versions_total{{version="{k}"}} {v}'
                    for k, v in sorted(self.verifier.by_version.items())]
        return out
