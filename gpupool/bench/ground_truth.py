"""Independent ground truth for ``status.readyReplicas`` (BASELINE.json: "readyReplicas exactly
matching rocm-smi ground truth").

Deliberately shares no code path with the operator's readiness computation:
  * device presence/health comes from the ``amd-smi`` CLI parsed here in Python (real hardware:
    xGMI link state, hotspot vs the device's own limit, **uncorrectable ECC since the bench
    baseline** and retired HBM pages), or from the fake fixture + fault overlay file read directly
    (fake backend);
  * per-pool ownership + advertisement come from the **kubelet**: PodResources
    ``GetAllocatableResources`` lists the device IDs the kubelet holds per extended resource, and
    every bench pool uses its own resource name, so "devices of pool P" = the kubelet's IDs for
    P's resource (the reference's tag-scoped ownership, README.md:238, re-expressed per resource);
  * the agent's claim ledger is read from disk only as a cross-check (``ledgerAgrees``), never to
    decide the count.
truth(pool) = #{kubelet-advertised devices of P's resource that the CLI reports present+healthy}.
"""
from __future__ import annotations

import json
import os
import subprocess

import grpc

from ..agent.deviceplugin.proto import PR, Stub, unix_target


def _amdsmi(*cmd: str) -> object:
    out = subprocess.run(["amd-smi", *cmd, "--json"], capture_output=True, text=True, timeout=60)
    if out.returncode != 0:
        raise RuntimeError(f"amd-smi {' '.join(cmd)} failed: {out.stderr[-300:]}")
    return json.loads(out.stdout)


def _by_gpu(doc: object) -> dict:
    rows = doc.get("gpu_data", doc) if isinstance(doc, dict) else doc
    return {d["gpu"]: d for d in rows or [] if isinstance(d, dict) and "gpu" in d}


def _num(v: object) -> float | None:
    """amd-smi values come as numbers, {"value": n, "unit": u} or "N/A"."""
    if isinstance(v, dict):
        v = v.get("value")
    if isinstance(v, bool):
        return None
    if isinstance(v, (int, float)):
        return v
    try:
        return float(str(v))
    except (TypeError, ValueError):
        return None


def _int(v: object) -> int:
    n = _num(v)
    return int(n) if n is not None else 0


# CLI temperature sensors -> (our name, metric key, slowdown limit key, shutdown limit key)
_CLI_SENSORS = (("edge", "edge", "slowdown_edge_temperature", "shutdown_edge_temperature"),
                ("hotspot", "hotspot", "slowdown_hotspot_temperature", "shutdown_hotspot_temperature"),
                ("vram", "mem", "slowdown_vram_temperature", "shutdown_vram_temperature"))


def cli_state() -> dict[str, dict]:
    """uuid -> device in the fault overlay's field layout (``index, present, ecc{correctable,
    uncorrectable}, xgmi.links, temps{sensor: {current, critical=slowdown limit, emergency=
    shutdown limit}}, ras{retiredPages, pendingPages}, partition``), parsed here in Python from
    one pass of the amd-smi CLI (list, metric, static, xgmi, partition, bad-pages). Shares no
    code with the operator's amdsmi/C++ path."""
    lst = _amdsmi("list")
    metric = _by_gpu(_amdsmi("metric"))
    static = _by_gpu(_amdsmi("static"))
    xgmi = _amdsmi("xgmi")
    links = {d["gpu"]: d.get("link_status", []) for d in
             (xgmi.get("link_port_status", []) if isinstance(xgmi, dict) else [])}
    try:
        part = _amdsmi("partition")
        parts = {d.get("gpu"): d for d in (part.get("current_partition", [])
                                          if isinstance(part, dict) else [])}
    except Exception:
        parts = {}
    try:
        bad = _by_gpu(_amdsmi("bad-pages"))
    except Exception:  # not supported / not permitted: retired pages stay unknown
        bad = {}
    out: dict[str, dict] = {}
    for d in lst:
        g = d["gpu"]
        m, s = metric.get(g, {}), static.get(g, {})
        ecc = m.get("ecc") or {}
        temps = {}
        for ours, cli, slow, shut in _CLI_SENSORS:
            cur = _num((m.get("temperature") or {}).get(cli))
            if cur is None:
                continue
            t = {"current": cur}
            lim = s.get("limit") or {}
            if _num(lim.get(slow)) is not None:
                t["critical"] = _num(lim.get(slow))
            if _num(lim.get(shut)) is not None:
                t["emergency"] = _num(lim.get(shut))
            temps[ours] = t
        b = bad.get(g)
        ras = {"badPagesSupported": False}
        if isinstance(b, dict):
            ras = {"badPagesSupported": True,
                   "retiredPages": len(b["retired"]) if isinstance(b.get("retired"), list) else 0,
                   "pendingPages": len(b["pending"]) if isinstance(b.get("pending"), list) else 0,
                   "unreservablePages": len(b["un_res"]) if isinstance(b.get("un_res"), list) else 0}
        p = parts.get(g) or {}
        out[d["uuid"]] = {
            "index": g, "uuid": d["uuid"], "present": True,
            "xgmi": {"links": list(links.get(g, []))} if g in links else {},
            "temps": temps,
            "ecc": {"uncorrectable": _int(ecc.get("total_uncorrectable_count")),
                    "correctable": _int(ecc.get("total_correctable_count"))},
            "ras": ras,
            "partition": {k: v for k, v in (("compute", p.get("accelerator_type")),
                                            ("memory", p.get("memory"))) if isinstance(v, str)},
        }
    return out


def _merge(dst: dict, src: dict) -> dict:
    out = dict(dst)
    for k, v in src.items():
        out[k] = _merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


def apply_overlay(devs: dict[str, dict], overlay: dict | None) -> dict[str, dict]:
    """The fault overlay (``{"devices": {uuid|hipUUID|index: partial device}}``) deep-merged
    onto a device map, keyed the way the overlay names devices. An injected fault is part of
    the ground truth by construction; the CLI cannot see it."""
    faults = (overlay or {}).get("devices") or {}
    if not faults:
        return devs
    out = {}
    for u, d in devs.items():
        for key in (u, str(d.get("hipUUID", "")), str(d.get("index", ""))):
            if key in faults and isinstance(faults[key], dict):
                d = _merge(d, faults[key])
        out[u] = d
    return out


HEALTH_DEFAULTS = {"maxUncorrectableECC": 0, "maxCorrectableECC": 100000,
                   "requireAllXGMILinks": True, "minXGMILinksUp": 7, "thermal": "belowCritical",
                   "thermalMarginC": 0, "maxRetiredPages": 64, "maxPendingPages": 0}


def device_healthy(dev: dict, base: dict | None, policy: dict | None = None) -> tuple[bool, list[str]]:
    """The pool's health rule, restated from the CRD's documented semantics (spec.health,
    spec.partition) — not the operator's evaluator: present; xGMI links (all up / at least
    minXGMILinksUp); uncorrectable and correctable ECC *since* ``base`` within the limits;
    retired / pending / unreservable HBM pages; every temperature sensor below its critical
    (slowdown) or emergency (shutdown) limit minus the margin; required partition mode."""
    pol = policy or {}
    h = {**HEALTH_DEFAULTS, **(pol.get("health") or {})}
    why: list[str] = []
    if dev.get("present") is False:
        return False, ["missing"]
    links = (dev.get("xgmi") or {}).get("links")
    if not isinstance(links, list):
        if h["requireAllXGMILinks"] or h["minXGMILinksUp"] > 0:
            why.append("xgmi status unavailable")
    else:
        up = sum(1 for x in links if str(x).upper() in ("U", "UP"))
        down = sum(1 for x in links if str(x).upper() in ("D", "DOWN"))
        if h["requireAllXGMILinks"] and down:
            why.append(f"xgmi {down} down")
        if up < h["minXGMILinksUp"]:
            why.append(f"xgmi {up} up")
    b = base or dev
    ecc, becc = dev.get("ecc") or {}, (b.get("ecc") or {})
    if ecc.get("uncorrectable", 0) - becc.get("uncorrectable", ecc.get("uncorrectable", 0)) > \
            h["maxUncorrectableECC"]:
        why.append("uncorrectable ecc")
    umc, bumc = dev.get("eccUmc"), b.get("eccUmc") or {}
    if isinstance(umc, dict) and umc.get("uncorrectable", 0) - \
            bumc.get("uncorrectable", umc.get("uncorrectable", 0)) > h["maxUncorrectableECC"]:
        why.append("uncorrectable ecc (umc)")
    if ecc.get("correctable", 0) - becc.get("correctable", ecc.get("correctable", 0)) > \
            h["maxCorrectableECC"]:
        why.append("correctable ecc")
    if "maxLifetimeUncorrectableECC" in h and \
            ecc.get("uncorrectable", 0) > h["maxLifetimeUncorrectableECC"]:
        why.append("lifetime ecc")
    ras = dev.get("ras") or {}
    if ras.get("badPagesSupported", True):
        if ras.get("retiredPages", 0) > h["maxRetiredPages"]:
            why.append("retired pages")
        if ras.get("pendingPages", 0) > h["maxPendingPages"]:
            why.append("pending pages")
        if ras.get("unreservablePages", 0) > 0:
            why.append("unreservable pages")
    if h["thermal"] != "ignore":
        lim_key = "emergency" if h["thermal"] == "belowEmergency" else "critical"
        for name, t in (dev.get("temps") or {}).items():
            if not isinstance(t, dict):
                continue
            cur, lim = t.get("current"), t.get(lim_key)
            if isinstance(cur, (int, float)) and isinstance(lim, (int, float)) and \
                    cur + h["thermalMarginC"] >= lim:
                why.append(f"{name} {cur} >= {lim_key} {lim}")
    want = pol.get("partition") or {}
    for k in ("compute", "memory"):
        w, have = want.get(k, "Any"), (dev.get("partition") or {}).get(k, "")
        if w != "Any" and have and have != w:
            why.append(f"partition {k}")
    return not why, why


def healthy_from_cli(state: dict[str, dict], baseline: dict[str, dict] | None = None,
                     policy: dict | None = None, overlay: dict | None = None) -> set[str]:
    """Healthy GPUs of one ``cli_state()`` (plus any injected fault overlay) under ``policy``:
    ECC counts as a delta since ``baseline`` (a ``cli_state()`` from when the bench started or
    the GPU was claimed: historic counts are not new faults, the rule the pool CRD documents)."""
    state = apply_overlay(state, overlay)
    return {u for u, d in state.items()
            if device_healthy(d, (baseline or {}).get(u), policy)[0]}


def healthy_uuids_cli() -> set[str]:
    return healthy_from_cli(cli_state())


def _fnv1a(s: str) -> int:
    h = 2166136261
    for c in s.encode():
        h ^= c
        h = (h * 16777619) & 0xFFFFFFFF
    return h


def fixture_uuids(fixture: str, node: str) -> list[str]:
    """UUIDs of the fake fixture, salted by node name exactly like the fake backend."""
    with open(fixture) as f:
        snap = json.load(f)
    h = _fnv1a(node)
    return [d["uuid"][:-8] + f"{(h ^ d['index']) & 0xFFFFFFFF:08x}" for d in snap["devices"]]


def fixture_state(fixture: str, node: str) -> dict[str, dict]:
    """uuid -> fixture device (no faults), uuids salted like the fake backend."""
    with open(fixture) as f:
        snap = json.load(f)
    return {u: {**d, "uuid": u} for d, u in zip(snap["devices"], fixture_uuids(fixture, node))}


def read_overlay(faults: str | None) -> dict:
    if faults and os.path.exists(faults):
        try:
            with open(faults) as f:
                return json.load(f) or {}
        except ValueError:
            return {}
    return {}


def healthy_uuids_fixture(fixture: str, faults: str | None, node: str,
                          policy: dict | None = None,
                          baseline: dict[str, dict] | None = None) -> set[str]:
    """Fake backend truth: fixture + fault overlay, read straight from the files, judged by
    ``device_healthy`` (ECC deltas against ``baseline``, default: the unfaulted fixture)."""
    base = fixture_state(fixture, node)
    cur = apply_overlay(base, read_overlay(faults))
    return {u for u, d in cur.items()
            if device_healthy(d, (baseline or base).get(u), policy)[0]}


def kubelet_allocatable(pod_resources_socket: str, timeout: float = 2.0) -> dict[str, set[str]]:
    """resource name -> device IDs the kubelet holds (PodResources v1 GetAllocatableResources)."""
    with grpc.insecure_channel(unix_target(pod_resources_socket)) as ch:
        resp = Stub(ch, "v1.PodResourcesLister").GetAllocatableResources(
            PR.AllocatableResourcesRequest(), timeout=timeout)
    out: dict[str, set[str]] = {}
    for dev in resp.devices:
        out.setdefault(dev.resource_name, set()).update(dev.device_ids)
    return out


def ledger_claims(state_dir: str, pool_uid: str) -> tuple[set[str], set[str]]:
    """Claims of ``pool_uid`` read straight from the agent's ledger file on disk: (probed and
    passed — state Claimed, durable probe verdict; claimed with the verdict still on its way to the
    disk — state Probing). A claim is made durable as 'Probing' before its probe runs and the
    agent replies as soon as the probe passed; the Probing -> Claimed write follows through the
    ledger's background writer (a crash in between re-probes the GPU), so right at Ready a loaded
    host may still show 'Probing' on disk for a claim whose probe passed."""
    with open(os.path.join(state_dir, "ledger.json")) as f:
        claims = (json.load(f) or {}).get("claims") or {}
    mine = {u: rec for u, rec in claims.items() if rec.get("poolUID") == pool_uid}
    passed = {u for u, rec in mine.items()
              if rec.get("state") == "Claimed" and (rec.get("probe") or {}).get("passed")}
    probing = {u for u, rec in mine.items() if rec.get("state") == "Probing"}
    return passed, probing


def pool_truth(pod_resources_socket: str, resource: str, healthy: set[str],
               state_dir: str | None = None, pool_uid: str | None = None,
               allocatable: dict[str, set[str]] | None = None) -> dict:
    """Ground truth for one pool that owns ``resource`` exclusively on this node."""
    alloc = allocatable if allocatable is not None else kubelet_allocatable(pod_resources_socket)
    adv = alloc.get(resource, set())
    good = adv & healthy
    out = {"advertised": len(adv), "healthyAdvertised": len(good), "ready": len(good)}
    if state_dir and pool_uid:
        passed, probing = ledger_claims(state_dir, pool_uid)
        out["ledgerClaimed"] = len(passed)
        out["ledgerProbing"] = len(probing)  # durable claims whose verdict write is pending
        out["ledgerAgrees"] = ((passed | probing) & healthy) == good
    return out
