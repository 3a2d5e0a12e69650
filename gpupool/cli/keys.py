"""``gpuctl keys``: the manager's agent-RPC signing key, created and rotated without a failed RPC.

The manager signs every agent RPC with the Ed25519 key in Secret ``gpupool-manager-signing-key``
(``key``); agents trust the public keys in ConfigMap ``gpupool-manager-pubkeys`` (one
``<key id>.pem`` per key). Both are mounted files the kubelet keeps in sync and both sides re-read
(gpupool/utils/edsig.py, native/src/runtime/agentauth.cc). A rotation is three steps, each safe
to run only once the cluster caught up with the one before — which is what this module checks,
from what every agent reports on its (unauthenticated) ``/metrics``:

1. ``rotate``: a new key; its private half parked in Secret ``gpupool-manager-signing-key-next``,
   its public half added to the ConfigMap. Nothing signs with it yet.
2. ``rotate`` again, once every agent lists the new key as trusted
   (``gpupool_agent_trusted_key``): the new private key moves into the manager's Secret.
3. ``prune``, once the agents see the new key in use (``gpupool_agent_rpc_signatures_total``):
   every other public key leaves the ConfigMap.

``status`` shows where a cluster is. (Least-privilege identity, reference README.md:43-60.)
"""
from __future__ import annotations

import os
import re
import sys
from typing import Any

from ..api import schema
from ..kube import CONFIGMAPS, NODES, SECRETS, Client, KubeError
from ..utils import edsig

SECRET = "gpupool-manager-signing-key"
NEXT_SECRET = "gpupool-manager-signing-key-next"
CONFIGMAP = "gpupool-manager-pubkeys"
_TRUSTED = re.compile(r'^gpupool_agent_trusted_key\{keyId="([0-9a-f]+)"\} 1', re.M)
_USED = re.compile(r'^gpupool_agent_rpc_signatures_total\{keyId="([0-9a-f]+)"\} (\d+)', re.M)


class KeyError_(Exception):
    """A step that must wait for the cluster (or was asked out of order)."""


def _b64(s: str) -> str:
    import base64
    return base64.b64encode(s.encode()).decode()


def _unb64(s: str) -> str:
    import base64
    return base64.b64decode(s).decode()


def _get(c: Client, res, name: str, ns: str) -> dict | None:
    try:
        return c.get(res, name, ns)
    except KubeError as e:
        if e.code == 404:
            return None
        raise


def _kid_of(pem: str) -> str:
    return edsig.key_id(edsig.public_from_private(edsig.load_private_key(pem)))


def _new_key() -> tuple[str, str, str]:
    """(key id, private PEM, public PEM) of a fresh Ed25519 key."""
    seed = os.urandom(32)
    pub = edsig.public_from_private(seed)
    return edsig.key_id(pub), edsig.private_pem(seed), edsig.public_pem(pub)


def _add_pubkey(c: Client, ns: str, kid: str, pem: str) -> None:
    cm = _get(c, CONFIGMAPS, CONFIGMAP, ns)
    if cm is None:
        c.create(CONFIGMAPS, {"apiVersion": "v1", "kind": "ConfigMap",
                              "metadata": {"name": CONFIGMAP}, "data": {f"{kid}.pem": pem}}, ns)
    else:
        c.patch(CONFIGMAPS, CONFIGMAP, {"data": {f"{kid}.pem": pem}}, ns)


def init(c: Client, ns: str) -> str:
    """The first key: Secret + ConfigMap. Refuses if the Secret exists (use rotate)."""
    if _get(c, SECRETS, SECRET, ns) is not None:
        raise KeyError_(f"secret {ns}/{SECRET} exists: rotate it instead")
    kid, priv, pub = _new_key()
    _add_pubkey(c, ns, kid, pub)  # trusted before anything signs with it
    c.create(SECRETS, {"apiVersion": "v1", "kind": "Secret", "type": "Opaque",
                       "metadata": {"name": SECRET}, "data": {"key": _b64(priv)}}, ns)
    return kid


def agents(c: Client) -> dict[str, dict[str, Any]]:
    """node -> {"trusted": [key ids], "used": {key id: signed requests}} (or {"error"})."""
    from .gpuctl import _agent_endpoint
    out: dict[str, dict[str, Any]] = {}
    for node in c.list(NODES)["items"]:
        name = node["metadata"]["name"]
        ep = _agent_endpoint(c, node)
        if not ep:
            continue
        try:
            text = Client(ep, timeout=5.0).request("GET", "/metrics")
        except Exception as e:  # noqa: BLE001 — reported per node
            out[name] = {"error": f"{type(e).__name__}: {e}"}
            continue
        text = text if isinstance(text, str) else ""
        out[name] = {"trusted": sorted(set(_TRUSTED.findall(text))),
                     "used": {k: int(v) for k, v in _USED.findall(text)}}
    return out


def status(c: Client, ns: str) -> dict[str, Any]:
    sec, nxt = _get(c, SECRETS, SECRET, ns), _get(c, SECRETS, NEXT_SECRET, ns)
    cm = _get(c, CONFIGMAPS, CONFIGMAP, ns)
    return {"signing": _kid_of(_unb64(sec["data"]["key"])) if sec else None,
            "next": _kid_of(_unb64(nxt["data"]["key"])) if nxt else None,
            "published": sorted(k[:-4] for k in ((cm or {}).get("data") or {}) if k.endswith(".pem")),
            "agents": agents(c)}


def rotate(c: Client, ns: str, force: bool = False) -> tuple[str, str]:
    """Step 1 (no pending key): ("trusting", new key id). Step 2 (a pending key every agent
    trusts): ("signing", new key id)."""
    nxt = _get(c, SECRETS, NEXT_SECRET, ns)
    if nxt is None:
        if _get(c, SECRETS, SECRET, ns) is None:
            raise KeyError_(f"no secret {ns}/{SECRET}: run `gpuctl keys init` first")
        kid, priv, pub = _new_key()
        _add_pubkey(c, ns, kid, pub)
        c.create(SECRETS, {"apiVersion": "v1", "kind": "Secret", "type": "Opaque",
                           "metadata": {"name": NEXT_SECRET}, "data": {"key": _b64(priv)}}, ns)
        return "trusting", kid
    priv = _unb64(nxt["data"]["key"])
    kid = _kid_of(priv)
    if not force:
        behind = {n: a.get("error") or f"trusts {a['trusted']}"
                  for n, a in agents(c).items() if kid not in a.get("trusted", [])}
        if behind:
            raise KeyError_(f"key {kid} is not trusted yet by: " +
                            "; ".join(f"{n} ({why})" for n, why in sorted(behind.items())) +
                            " — the kubelet syncs the ConfigMap within about a minute")
    c.patch(SECRETS, SECRET, {"data": {"key": nxt["data"]["key"]}}, ns)
    c.delete(SECRETS, NEXT_SECRET, ns)
    return "signing", kid


def prune(c: Client, ns: str, force: bool = False) -> list[str]:
    """Step 3: drop every published key but the signing one, once the agents that saw any signed
    request have seen one made with it. Returns the key ids removed."""
    if _get(c, SECRETS, NEXT_SECRET, ns) is not None and not force:
        raise KeyError_("a rotation is half done (a pending key): run `gpuctl keys rotate` first")
    sec = _get(c, SECRETS, SECRET, ns)
    if sec is None:
        raise KeyError_(f"no secret {ns}/{SECRET}")
    kid = _kid_of(_unb64(sec["data"]["key"]))
    if not force:
        stale = [n for n, a in agents(c).items()
                 if a.get("used") and not a["used"].get(kid)]
        if stale:
            raise KeyError_(f"the manager has not signed with {kid} to {', '.join(sorted(stale))} "
                            "yet (it re-reads its key within seconds of the kubelet's Secret sync)")
    cm = _get(c, CONFIGMAPS, CONFIGMAP, ns) or {}
    gone = [k[:-4] for k in (cm.get("data") or {}) if k.endswith(".pem") and k[:-4] != kid]
    if gone:
        c.patch(CONFIGMAPS, CONFIGMAP, {"data": {f"{k}.pem": None for k in gone}}, ns)
    return gone


def main(c: Client, args) -> int:
    ns = args.key_namespace or schema.AGENT_NAMESPACE
    try:
        if args.keys_cmd == "init":
            print(f"signing key {init(c, ns)} created (secret {ns}/{SECRET}, configmap {CONFIGMAP})")
        elif args.keys_cmd == "rotate":
            step, kid = rotate(c, ns, args.force)
            if step == "trusting":
                print(f"key {kid} published to the agents; run `gpuctl keys rotate` again once "
                      "every agent trusts it (`gpuctl keys status`)")
            else:
                print(f"the manager signs with {kid} once its Secret is synced; run `gpuctl keys "
                      "prune` once the agents see it in use")
        elif args.keys_cmd == "prune":
            gone = prune(c, ns, args.force)
            print(f"removed {', '.join(gone)}" if gone else "nothing to remove")
        else:
            st = status(c, ns)
            print(f"signing:   {st['signing']}\nnext:      {st['next'] or '-'}\n"
                  f"published: {', '.join(st['published']) or '-'}")
            for n, a in sorted(st["agents"].items()):
                if "error" in a:
                    print(f"  {n}: unreachable ({a['error']})")
                else:
                    used = ", ".join(f"{k}={v}" for k, v in sorted(a["used"].items())) or "-"
                    print(f"  {n}: trusts {', '.join(a['trusted']) or '-'}; signed requests {used}")
    except KeyError_ as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    return 0
