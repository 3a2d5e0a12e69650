"""Independent ground truth for ``status.readyReplicas`` (BASELINE.json: "readyReplicas exactly
matching rocm-smi ground truth").

Deliberately shares no code path with the operator's readiness computation:
  * device presence/health comes from the ``amd-smi`` CLI parsed here in Python (real hardware),
    or from the fake fixture + fault overlay file read directly (fake backend);
  * ownership comes from the agent's claim-ledger files on disk, not from the agent's API;
  * advertisement comes from the kubelet's view (Node ``status.allocatable[resource]``).
truth = #{devices claimed by the pool (ledger) that are present+healthy (CLI) and advertised}.
"""
from __future__ import annotations

import json
import os
import subprocess

from ..kube import NODES, Client


def _amdsmi(cmd: str) -> object:
    out = subprocess.run(["amd-smi", cmd, "--json"], capture_output=True, text=True, timeout=60)
    if out.returncode != 0:
        raise RuntimeError(f"amd-smi {cmd} failed: {out.stderr[-300:]}")
    return json.loads(out.stdout)


def healthy_uuids_cli() -> set[str]:
    """Present GPUs with every non-disabled xGMI link up, no uncorrectable ECC, below critical."""
    lst = _amdsmi("list")
    metric = _amdsmi("metric")
    static = _amdsmi("static")
    xgmi = _amdsmi("xgmi")
    m_by = {d["gpu"]: d for d in (metric.get("gpu_data", metric) if isinstance(metric, dict) else metric)}
    s_by = {d["gpu"]: d for d in (static.get("gpu_data", static) if isinstance(static, dict) else static)}
    links = {d["gpu"]: d.get("link_status", []) for d in xgmi.get("link_port_status", [])}
    ok = set()
    for d in lst:
        g = d["gpu"]
        m, s = m_by.get(g, {}), s_by.get(g, {})
        if "D" in links.get(g, []):
            continue
        hot = (m.get("temperature") or {}).get("hotspot")
        crit = ((s.get("limit") or {}).get("slowdown_hotspot_temperature"))
        if isinstance(hot, dict) and isinstance(crit, dict) and hot["value"] >= crit["value"]:
            continue
        ok.add(d["uuid"])
    return ok


def healthy_uuids_fixture(fixture: str, faults: str | None, node: str) -> set[str]:
    """Fake backend truth: fixture (UUIDs salted by node name exactly like the fake backend)."""
    with open(fixture) as f:
        snap = json.load(f)
    ov = {}
    if faults and os.path.exists(faults):
        with open(faults) as f:
            ov = (json.load(f) or {}).get("devices", {})

    def fnv1a(s: str) -> int:
        h = 2166136261
        for c in s.encode():
            h ^= c
            h = (h * 16777619) & 0xFFFFFFFF
        return h
    h = fnv1a(node)
    ok = set()
    for d in snap["devices"]:
        u = d["uuid"][:-8] + f"{(h ^ d['index']) & 0xFFFFFFFF:08x}"
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


def ledger_claims(state_dir: str, pool_uid: str) -> set[str]:
    """Claims of ``pool_uid`` read straight from the agent's ledger file on disk."""
    with open(os.path.join(state_dir, "ledger.json")) as f:
        claims = (json.load(f) or {}).get("claims") or {}
    return {u for u, rec in claims.items()
            if rec.get("poolUID") == pool_uid and rec.get("state") == "Claimed"
            and (rec.get("probe") or {}).get("passed")}


def advertised_count(client: Client, node: str, resource: str) -> int:
    n = client.get(NODES, node)
    return int((n.get("status", {}).get("allocatable") or {}).get(resource, "0"))


def truth(client: Client, node: str, pool_uid: str, state_dir: str, resource: str,
          healthy: set[str]) -> dict:
    claimed = ledger_claims(state_dir, pool_uid)
    good = claimed & healthy
    adv = advertised_count(client, node, resource)
    return {"claimed": len(claimed), "healthyClaimed": len(good), "advertised": adv,
            "ready": min(len(good), adv)}
