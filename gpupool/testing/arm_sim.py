"""Azure Resource Manager simulator: the token endpoint and the slice of ARM that AzureVmPool uses.

There is no Azure access here, so the ``--cloud azure-arm`` provider
(native/src/provider/azure_arm.cc) is tested against this HTTPS server. It models what the
provider depends on, with ARM's wire shapes:

* ``POST /{tenant}/oauth2/v2.0/token`` — client_credentials with a client secret or a federated
  client assertion; issues opaque bearer tokens with ``expires_in`` (short lifetimes and
  revocation are settable, to exercise the provider's refresh-on-401).
* ``/subscriptions/{sub}/resourceGroups/{rg}/providers/Microsoft.Compute/virtualMachines[/{vm}]``
  — PUT (201 Creating -> Succeeded after ``vm_delay``; idempotent re-PUT), GET, list with
  ``nextLink`` paging, DELETE (202 Deleting -> gone after ``delete_delay``; NIC and OS disk removed
  with the VM only when their ``deleteOption`` is Delete, else left detached = orphans).
* ``.../Microsoft.Network/networkInterfaces[/{nic}]`` — PUT (subnet reference checked), GET,
  list, DELETE (``NicInUse`` while attached).
* ``.../Microsoft.Compute/disks[/{disk}]`` — list, DELETE (refused while ``managedBy`` is set).
* Principals are scoped to subscriptions (403 AuthorizationFailed), resource groups must exist
  (404 ResourceGroupNotFound), VMs per resource group are capped (409 OperationNotAllowed).
* ``POST /_sim/faults`` queues failures (``throttle``: n 429s, ``failVmPut``: n 500s,
  ``lostVmPut``: n VM PUTs accepted but answered 504 and hidden from lists for 2 s,
  ``revokeTokens``), ``GET /_sim/state`` dumps everything (tests assert on it).

Run in-process (``ArmSim(...).start()``, a daemon thread with its own event loop) or as
``python -m gpupool.testing.arm_sim --port-file F --cert C --key K``.
"""
from __future__ import annotations

import argparse
import asyncio
import datetime as _dt
import json
import os
import secrets
import ssl
import threading
import time
import urllib.parse

from aiohttp import web

COMPUTE = "Microsoft.Compute"
NETWORK = "Microsoft.Network"


def _now() -> str:
    return _dt.datetime.now(_dt.timezone.utc).isoformat().replace("+00:00", "Z")


def _err(status: int, code: str, message: str) -> web.Response:
    return web.json_response({"error": {"code": code, "message": message}}, status=status)


class ArmSim:
    def __init__(self, principals: dict | None = None, resource_groups: dict | None = None,
                 vm_delay: float = 0.3, delete_delay: float = 0.3, nic_delay: float = 0.0,
                 page_size: int = 50, quota_per_rg: int = 100, token_ttl: int = 3600,
                 certfile: str | None = None, keyfile: str | None = None):
        # client id -> {"tenant", "secret" | None (federated), "subscriptions": [...]}
        self.principals = principals if principals is not None else {}
        # "sub/rg" -> {"location", "vnets": {vnet: [subnets]}}
        self.rgs = resource_groups if resource_groups is not None else {}
        self.vm_delay, self.delete_delay, self.nic_delay = vm_delay, delete_delay, nic_delay
        self.page_size, self.quota_per_rg, self.token_ttl = page_size, quota_per_rg, token_ttl
        self.certfile, self.keyfile = certfile, keyfile
        self.tokens: dict[str, dict] = {}
        self.vms: dict[str, dict] = {}    # lower-cased id -> resource
        self.nics: dict[str, dict] = {}
        self.disks: dict[str, dict] = {}
        self.faults = {"throttle": 0, "failVmPut": 0, "lostVmPut": 0}
        self.calls: list[tuple[str, str, int]] = []
        self.token_requests = 0
        self.mu = threading.Lock()
        self.port = 0
        self._loop: asyncio.AbstractEventLoop | None = None
        self._runner: web.AppRunner | None = None
        self._thread: threading.Thread | None = None

    # ------------------------------------------------------------------ lifecycle
    @property
    def url(self) -> str:
        return f"{'https' if self.certfile else 'http'}://127.0.0.1:{self.port}"

    def app(self) -> web.Application:
        a = web.Application()
        a.router.add_post("/_sim/faults", self._h_faults)
        a.router.add_get("/_sim/state", self._h_state)
        a.router.add_post("/{tenant}/oauth2/v2.0/token", self._h_token)
        a.router.add_route("*", "/subscriptions/{tail:.*}", self._h_arm)
        return a

    def start(self, port: int = 0) -> "ArmSim":
        ready = threading.Event()

        def run():
            self._loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self._loop)
            self._runner = web.AppRunner(self.app(), access_log=None)
            self._loop.run_until_complete(self._runner.setup())
            ctx = None
            if self.certfile:
                ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
                ctx.load_cert_chain(self.certfile, self.keyfile)
            site = web.TCPSite(self._runner, "127.0.0.1", port, ssl_context=ctx)
            self._loop.run_until_complete(site.start())
            self.port = site._server.sockets[0].getsockname()[1]
            ready.set()
            self._loop.run_forever()

        self._thread = threading.Thread(target=run, daemon=True, name="arm-sim")
        self._thread.start()
        if not ready.wait(10):
            raise RuntimeError("ARM simulator did not start")
        return self

    def stop(self) -> None:
        if self._loop is None:
            return
        fut = asyncio.run_coroutine_threadsafe(self._runner.cleanup(), self._loop)
        try:
            fut.result(5)
        finally:
            self._loop.call_soon_threadsafe(self._loop.stop)
            self._thread.join(5)

    # ------------------------------------------------------------------ state
    def _advance(self) -> None:
        """Move long-running operations forward (lazily, on every request)."""
        now = time.monotonic()
        for vid, vm in list(self.vms.items()):
            p = vm["properties"]
            if p["provisioningState"] == "Creating" and now >= vm["_ready_at"]:
                p["provisioningState"] = "Succeeded"
            elif p["provisioningState"] == "Deleting" and now >= vm["_gone_at"]:
                del self.vms[vid]
                for ref in p["networkProfile"]["networkInterfaces"]:
                    nic = self.nics.get(ref["id"].lower())
                    if not nic:
                        continue
                    if (ref.get("properties") or {}).get("deleteOption") == "Delete":
                        del self.nics[ref["id"].lower()]
                    else:
                        nic["properties"].pop("virtualMachine", None)
                osd = p["storageProfile"]["osDisk"]
                did = f"{vm['_rg']}/providers/{COMPUTE}/disks/{osd['name']}".lower()
                if did in self.disks:
                    if osd.get("deleteOption") == "Delete":
                        del self.disks[did]
                    else:
                        self.disks[did]["managedBy"] = None
        for nic in self.nics.values():
            if nic["properties"]["provisioningState"] == "Updating" and now >= nic["_ready_at"]:
                nic["properties"]["provisioningState"] = "Succeeded"

    def state(self) -> dict:
        with self.mu:
            self._advance()
            strip = lambda d: {k: v for k, v in d.items() if not k.startswith("_")}  # noqa: E731
            return {"vms": [strip(v) for v in self.vms.values()],
                    "nics": [strip(v) for v in self.nics.values()],
                    "disks": [strip(v) for v in self.disks.values()],
                    "tokenRequests": self.token_requests,
                    "calls": len(self.calls)}

    # ------------------------------------------------------------------ handlers
    async def _h_faults(self, req: web.Request) -> web.Response:
        body = await req.json()
        with self.mu:
            for k in ("throttle", "failVmPut"):
                self.faults[k] += int(body.get(k, 0))
            if body.get("revokeTokens"):
                self.tokens.clear()
            if "tokenTtl" in body:
                self.token_ttl = int(body["tokenTtl"])
        return web.json_response(self.faults)

    async def _h_state(self, req: web.Request) -> web.Response:
        return web.json_response(self.state())

    async def _h_token(self, req: web.Request) -> web.Response:
        tenant = req.match_info["tenant"]
        form = await req.post()
        with self.mu:
            self.token_requests += 1
            p = self.principals.get(form.get("client_id", ""))
            if form.get("grant_type") != "client_credentials":
                return web.json_response({"error": "unsupported_grant_type"}, status=400)
            if not p or p["tenant"] != tenant:
                return web.json_response({"error": "unauthorized_client", "error_description":
                                          "AADSTS700016: application not found in the directory"},
                                         status=400)
            if p.get("secret") is None:  # federated credential: a client assertion is required
                ok = form.get("client_assertion_type", "").endswith("jwt-bearer") and \
                    bool(form.get("client_assertion"))
            else:
                ok = form.get("client_secret") == p["secret"]
            if not ok:
                return web.json_response({"error": "invalid_client", "error_description":
                                          "AADSTS7000215: invalid client secret provided"},
                                         status=401)
            tok = secrets.token_urlsafe(24)
            self.tokens[tok] = {"client": form["client_id"],
                                "exp": time.monotonic() + self.token_ttl}
            return web.json_response({"token_type": "Bearer", "expires_in": self.token_ttl,
                                      "access_token": tok})

    def _auth(self, req: web.Request, sub: str) -> web.Response | None:
        h = req.headers.get("Authorization", "")
        t = self.tokens.get(h[7:]) if h.startswith("Bearer ") else None
        if not t or time.monotonic() > t["exp"]:
            return _err(401, "ExpiredAuthenticationToken" if t else "InvalidAuthenticationToken",
                        "the access token is missing, invalid or expired")
        if sub not in self.principals[t["client"]].get("subscriptions", []):
            return _err(403, "AuthorizationFailed",
                        f"client {t['client']} has no access to subscription {sub}")
        return None

    async def _h_arm(self, req: web.Request) -> web.Response:
        body = await req.read()
        with self.mu:
            r = self._arm(req, body)
            self.calls.append((req.method, req.path, r.status))
            return r

    def _arm(self, req: web.Request, body: bytes) -> web.Response:
        parts = [urllib.parse.unquote(p) for p in req.path.strip("/").split("/")]
        # subscriptions/{sub}/resourceGroups/{rg}/providers/{ns}/{type}[/{name}[/...]]
        if len(parts) < 7 or parts[2].lower() != "resourcegroups" or parts[4] != "providers":
            return _err(404, "NotFound", req.path)
        sub, rg, ns, typ = parts[1], parts[3], parts[5], parts[6]
        name = parts[7] if len(parts) > 7 else None
        denied = self._auth(req, sub)
        if denied:
            return denied
        if self.faults["throttle"] > 0:
            self.faults["throttle"] -= 1
            return _err(429, "TooManyRequests", "throttled; retry after 1 s")
        if "api-version" not in req.query:
            return _err(400, "MissingApiVersionParameter", "api-version is required")
        rgkey = f"{sub}/{rg}"
        if rgkey not in self.rgs:
            return _err(404, "ResourceGroupNotFound", f"resource group '{rg}' could not be found")
        self._advance()
        base = f"/subscriptions/{sub}/resourceGroups/{rg}"
        kind = (ns, typ)
        if kind == (COMPUTE, "virtualMachines"):
            table = self.vms
        elif kind == (NETWORK, "networkInterfaces"):
            table = self.nics
        elif kind == (COMPUTE, "disks"):
            table = self.disks
        else:
            return _err(404, "NoRegisteredProviderFound", f"{ns}/{typ}")
        coll = f"{base}/providers/{ns}/{typ}"
        if name is None:
            if req.method != "GET":
                return _err(405, "MethodNotAllowed", req.method)
            return self._list(req, table, coll)
        rid = f"{coll}/{name}"
        key = rid.lower()
        if req.method == "GET":
            res = table.get(key)
            return web.json_response(self._public(res)) if res else \
                _err(404, "ResourceNotFound", f"{typ}/{name} not found")
        if req.method == "DELETE":
            return self._delete(kind, key, name)
        if req.method == "PUT":
            try:
                doc = json.loads(body or b"{}")
            except ValueError:
                return _err(400, "InvalidRequestContent", "body is not JSON")
            if kind == (NETWORK, "networkInterfaces"):
                return self._put_nic(rgkey, base, rid, name, doc)
            if kind == (COMPUTE, "virtualMachines"):
                return self._put_vm(rgkey, base, rid, name, doc)
            return _err(405, "MethodNotAllowed", "disks are created with their VM")
        return _err(405, "MethodNotAllowed", req.method)

    @staticmethod
    def _public(res: dict) -> dict:
        return {k: v for k, v in res.items() if not k.startswith("_")}

    def _list(self, req: web.Request, table: dict, coll: str) -> web.Response:
        now = time.monotonic()
        items = sorted((v for k, v in table.items() if k.startswith(coll.lower() + "/")
                        and v.get("_listed_at", 0) <= now),  # ARM's eventually consistent lists
                       key=lambda v: v["name"])
        skip = int(req.query.get("$skiptoken", "0") or 0)
        page = items[skip:skip + self.page_size]
        out = {"value": [self._public(v) for v in page]}
        if skip + self.page_size < len(items):
            q = dict(req.query)
            q["$skiptoken"] = str(skip + self.page_size)
            out["nextLink"] = f"{self.url}{coll}?{urllib.parse.urlencode(q)}"
        return web.json_response(out)

    def _put_nic(self, rgkey: str, base: str, rid: str, name: str, doc: dict) -> web.Response:
        key = rid.lower()
        if key in self.nics:  # idempotent PUT
            nic = self.nics[key]
            nic["tags"] = doc.get("tags") or nic.get("tags") or {}
            return web.json_response(self._public(nic), status=200)
        cfgs = (doc.get("properties") or {}).get("ipConfigurations") or []
        if not cfgs:
            return _err(400, "InvalidRequestFormat", "ipConfigurations is required")
        subnet_id = ((cfgs[0].get("properties") or {}).get("subnet") or {}).get("id", "")
        seg = subnet_id.split("/")
        vnets = self.rgs[rgkey].get("vnets", {})
        if len(seg) < 11 or seg[-4] != "virtualNetworks" or seg[-3] not in vnets or \
                seg[-2] != "subnets" or seg[-1] not in vnets[seg[-3]]:
            return _err(400, "InvalidResourceReference",
                        f"subnet {subnet_id} referenced by {name} was not found")
        state = "Updating" if self.nic_delay > 0 else "Succeeded"
        nic = {"id": rid, "name": name, "type": f"{NETWORK}/networkInterfaces",
               "location": doc.get("location", ""), "tags": doc.get("tags") or {},
               "properties": {"provisioningState": state, "ipConfigurations": cfgs},
               "_ready_at": time.monotonic() + self.nic_delay}
        self.nics[key] = nic
        return web.json_response(self._public(nic), status=201)

    def _put_vm(self, rgkey: str, base: str, rid: str, name: str, doc: dict) -> web.Response:
        key = rid.lower()
        if key in self.vms:  # idempotent PUT (tags may change)
            vm = self.vms[key]
            vm["tags"] = doc.get("tags") or vm["tags"]
            return web.json_response(self._public(vm), status=200)
        if self.faults["failVmPut"] > 0:
            self.faults["failVmPut"] -= 1
            return _err(500, "InternalServerError", "injected VM create failure")
        n_in_rg = sum(1 for k in self.vms if k.startswith(base.lower() + "/"))
        if n_in_rg >= self.quota_per_rg:
            return _err(409, "OperationNotAllowed",
                        f"operation results in exceeding quota limits ({self.quota_per_rg} VMs)")
        p = doc.get("properties") or {}
        if not (p.get("hardwareProfile") or {}).get("vmSize"):
            return _err(400, "InvalidParameter", "hardwareProfile.vmSize is required")
        img = (p.get("storageProfile") or {}).get("imageReference") or {}
        if not all(img.get(k) for k in ("publisher", "offer", "sku")):
            return _err(400, "InvalidParameter", "imageReference needs publisher, offer and sku")
        osp = p.get("osProfile") or {}
        lin = osp.get("linuxConfiguration") or {}
        keys = (lin.get("ssh") or {}).get("publicKeys") or []
        if not osp.get("adminUsername") or not (lin.get("disablePasswordAuthentication") and keys
                                                 and keys[0].get("keyData")):
            return _err(400, "InvalidParameter",
                        "a Linux VM without a password needs an SSH public key")
        refs = (p.get("networkProfile") or {}).get("networkInterfaces") or []
        if not refs:
            return _err(400, "InvalidParameter", "networkProfile.networkInterfaces is required")
        for ref in refs:
            nic = self.nics.get(ref.get("id", "").lower())
            if not nic:
                return _err(400, "InvalidResourceReference", f"NIC {ref.get('id')} not found")
            owner = nic["properties"].get("virtualMachine")
            if owner and owner["id"].lower() != key:
                return _err(400, "NicInUse", f"NIC {nic['name']} is attached to {owner['id']}")
        osd = dict((p.get("storageProfile") or {}).get("osDisk") or {})
        osd.setdefault("name", f"{name}_OsDisk_1_{secrets.token_hex(4)}")
        for ref in refs:
            self.nics[ref["id"].lower()]["properties"]["virtualMachine"] = {"id": rid}
        did = f"{base}/providers/{COMPUTE}/disks/{osd['name']}"
        self.disks[did.lower()] = {"id": did, "name": osd["name"], "type": f"{COMPUTE}/disks",
                                   "location": doc.get("location", ""), "managedBy": rid,
                                   "properties": {"provisioningState": "Succeeded",
                                                  "diskState": "Attached"}}
        vm = {"id": rid, "name": name, "type": f"{COMPUTE}/virtualMachines",
              "location": doc.get("location", ""), "tags": doc.get("tags") or {},
              "properties": {**p, "provisioningState": "Creating", "timeCreated": _now(),
                             "vmId": secrets.token_hex(16),
                             "storageProfile": {**(p.get("storageProfile") or {}), "osDisk": osd}},
              "_ready_at": time.monotonic() + self.vm_delay, "_rg": base}
        self.vms[key] = vm
        if self.faults["lostVmPut"] > 0:
            # accepted, but the reply is lost (gateway timeout) and lists will not show the VM
            # for a while: a retry that picks a new name would create a second VM
            self.faults["lostVmPut"] -= 1
            vm["_listed_at"] = time.monotonic() + 2.0
            return _err(504, "GatewayTimeout", "the request was accepted but the response timed out")
        return web.json_response(self._public(vm), status=201)

    def _delete(self, kind: tuple, key: str, name: str) -> web.Response:
        if kind == (COMPUTE, "virtualMachines"):
            vm = self.vms.get(key)
            if not vm:
                return web.Response(status=204)
            if vm["properties"]["provisioningState"] != "Deleting":
                vm["properties"]["provisioningState"] = "Deleting"
                vm["_gone_at"] = time.monotonic() + self.delete_delay
            return web.Response(status=202)
        if kind == (NETWORK, "networkInterfaces"):
            nic = self.nics.get(key)
            if not nic:
                return web.Response(status=204)
            if nic["properties"].get("virtualMachine"):
                return _err(400, "NicInUse", f"NIC {name} is attached to a VM")
            del self.nics[key]
            return web.Response(status=200)
        disk = self.disks.get(key)
        if not disk:
            return web.Response(status=204)
        if disk.get("managedBy"):
            return _err(409, "OperationNotAllowed", f"disk {name} is attached to a VM")
        del self.disks[key]
        return web.Response(status=200)

    # ------------------------------------------------------------------ test helpers
    def add_orphans(self, sub: str, rg: str, owner: str, prefix: str) -> None:
        """A NIC (tagged for ``owner``) and an OS disk left by an interrupted create."""
        base = f"/subscriptions/{sub}/resourceGroups/{rg}"
        with self.mu:
            nid = f"{base}/providers/{NETWORK}/networkInterfaces/{prefix}-nic"
            self.nics[nid.lower()] = {
                "id": nid, "name": f"{prefix}-nic", "type": f"{NETWORK}/networkInterfaces",
                "tags": {"managed-by": "azurevmpool-operator", "owner": owner},
                "properties": {"provisioningState": "Succeeded", "ipConfigurations": []},
                "_ready_at": 0}
            did = f"{base}/providers/{COMPUTE}/disks/{prefix}-osdisk"
            self.disks[did.lower()] = {"id": did, "name": f"{prefix}-osdisk",
                                       "type": f"{COMPUTE}/disks", "managedBy": None,
                                       "properties": {"provisioningState": "Succeeded",
                                                      "diskState": "Unattached"}}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--port-file")
    ap.add_argument("--cert")
    ap.add_argument("--key")
    ap.add_argument("--config", help="JSON: {principals, resourceGroups, vmDelay, ...}")
    a = ap.parse_args()
    cfg = json.load(open(a.config)) if a.config else {}
    sim = ArmSim(principals=cfg.get("principals"), resource_groups=cfg.get("resourceGroups"),
                 vm_delay=cfg.get("vmDelay", 0.3), delete_delay=cfg.get("deleteDelay", 0.3),
                 page_size=cfg.get("pageSize", 50), certfile=a.cert, keyfile=a.key).start(a.port)
    if a.port_file:
        tmp = a.port_file + ".tmp"
        with open(tmp, "w") as f:
            f.write(str(sim.port))
        os.replace(tmp, a.port_file)
    print(f"ARM simulator on {sim.url}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        sim.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
