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


def _int(v: object) -> int:
    if isinstance(v, dict):
        v = v.get("value")
    try:
        return int(v)  # "N/A" and friends -> 0
    except (TypeError, ValueError):
        return 0


def cli_state() -> dict[str, dict]:
    """uuid -> {present, xgmiDown, hotspot, hotspotLimit, eccUncorrectable, eccCorrectable,
    retiredPages} from one pass of the amd-smi CLI (list, metric, static, xgmi, bad-pages)."""
    lst = _amdsmi("list")
    metric = _by_gpu(_amdsmi("metric"))
    static = _by_gpu(_amdsmi("static"))
    xgmi = _amdsmi("xgmi")
    links = {d["gpu"]: d.get("link_status", []) for d in
             (xgmi.get("link_port_status", []) if isinstance(xgmi, dict) else [])}
    try:
        bad = _by_gpu(_amdsmi("bad-pages"))
    except Exception:  # not supported / not permitted: retired pages stay unknown (0)
        bad = {}
    out: dict[str, dict] = {}
    for d in lst:
        g = d["gpu"]
        m, s = metric.get(g, {}), static.get(g, {})
        ecc = m.get("ecc") or {}
        retired = (bad.get(g) or {}).get("retired")
        out[d["uuid"]] = {
            "present": True,
            "xgmiDown": sum(1 for x in links.get(g, []) if x == "D"),
            "hotspot": _int((m.get("temperature") or {}).get("hotspot")),
            "hotspotLimit": _int((s.get("limit") or {}).get("slowdown_hotspot_temperature")) or None,
            "eccUncorrectable": _int(ecc.get("total_uncorrectable_count")),
            "eccCorrectable": _int(ecc.get("total_correctable_count")),
            "retiredPages": len(retired) if isinstance(retired, list) else 0,
        }
    return out


def healthy_from_cli(state: dict[str, dict], baseline: dict[str, dict] | None = None,
                     max_retired_pages: int | None = None) -> set[str]:
    """Present GPUs with no xGMI link down, hotspot below the device's slowdown limit, no new
    uncorrectable ECC since ``baseline`` (a ``cli_state()`` taken when the bench started: historic
    counts are not new faults, the same rule the pool CRD documents) and, when
    ``max_retired_pages`` is set, at most that many retired HBM pages."""
    ok = set()
    for u, s in state.items():
        if not s["present"] or s["xgmiDown"]:
            continue
        if s["hotspotLimit"] and s["hotspot"] >= s["hotspotLimit"]:
            continue
        base = (baseline or {}).get(u, s)
        if s["eccUncorrectable"] > base["eccUncorrectable"]:
            continue
        if max_retired_pages is not None and s["retiredPages"] > max_retired_pages:
            continue
        ok.add(u)
    return ok


def healthy_uuids_cli() -> set[str]:
    return healthy_from_cli(cli_state())


def fixture_uuids(fixture: str, node: str) -> list[str]:
    """UUIDs of the fake fixture, salted by node name exactly like the fake backend."""
    with open(fixture) as f:
        snap = json.load(f)

    def fnv1a(s: str) -> int:
        h = 2166136261
        for c in s.encode():
            h ^= c
            h = (h * 16777619) & 0xFFFFFFFF
        return h
    h = fnv1a(node)
    return [d["uuid"][:-8] + f"{(h ^ d['index']) & 0xFFFFFFFF:08x}" for d in snap["devices"]]


def healthy_uuids_fixture(fixture: str, faults: str | None, node: str) -> set[str]:
    """Fake backend truth: fixture + fault overlay, read straight from the files."""
    with open(fixture) as f:
        snap = json.load(f)
    ov = {}
    if faults and os.path.exists(faults):
        with open(faults) as f:
            ov = (json.load(f) or {}).get("devices", {})
    ok = set()
    for d, u in zip(snap["devices"], fixture_uuids(fixture, node)):
        f = ov.get(u) or ov.get(str(d["index"])) or {}
        if f.get("present") is False:
            continue
        if "D" in ((f.get("xgmi") or {}).get("links") or []):
            continue
        if ((f.get("ecc") or {}).get("uncorrectable", 0) or 0) > 0:
            continue
        hot = ((f.get("temps") or {}).get("hotspot") or {}).get("current")
        if hot is not None and hot >= d["temps"]["hotspot"]["critical"]:
            continue
        ok.add(u)
    return ok


def kubelet_allocatable(pod_resources_socket: str, timeout: float = 2.0) -> dict[str, set[str]]:
    """resource name -> device IDs the kubelet holds (PodResources v1 GetAllocatableResources)."""
    with grpc.insecure_channel(unix_target(pod_resources_socket)) as ch:
        resp = Stub(ch, "v1.PodResourcesLister").GetAllocatableResources(
            PR.AllocatableResourcesRequest(), timeout=timeout)
    out: dict[str, set[str]] = {}
    for dev in resp.devices:
        out.setdefault(dev.resource_name, set()).update(dev.device_ids)
    return out


def ledger_claims(state_dir: str, pool_uid: str) -> set[str]:
    """Claims of ``pool_uid`` read straight from the agent's ledger file on disk."""
    with open(os.path.join(state_dir, "ledger.json")) as f:
        claims = (json.load(f) or {}).get("claims") or {}
    return {u for u, rec in claims.items()
            if rec.get("poolUID") == pool_uid and rec.get("state") == "Claimed"
            and (rec.get("probe") or {}).get("passed")}


def pool_truth(pod_resources_socket: str, resource: str, healthy: set[str],
               state_dir: str | None = None, pool_uid: str | None = None,
               allocatable: dict[str, set[str]] | None = None) -> dict:
    """Ground truth for one pool that owns ``resource`` exclusively on this node."""
    alloc = allocatable if allocatable is not None else kubelet_allocatable(pod_resources_socket)
    adv = alloc.get(resource, set())
    good = adv & healthy
    out = {"advertised": len(adv), "healthyAdvertised": len(good), "ready": len(good)}
    if state_dir and pool_uid:
        claimed = ledger_claims(state_dir, pool_uid)
        out["ledgerClaimed"] = len(claimed)
        out["ledgerAgrees"] = (claimed & healthy) == good
    return out
