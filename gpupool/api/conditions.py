"""metav1.Condition semantics (Python mirror of native/src/api/conditions.cc).

``set_condition`` merges by ``type`` (README.md:127 ``patchMergeKey:"type"``) and only moves
``lastTransitionTime`` when ``status`` actually flips — the apimachinery ``meta.SetStatusCondition``
contract.
"""
from __future__ import annotations

import datetime as _dt


def now_rfc3339() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def find(conds: list[dict] | None, ctype: str) -> dict | None:
    for c in conds or []:
        if c.get("type") == ctype:
            return c
    return None


def is_true(conds: list[dict] | None, ctype: str) -> bool:
    c = find(conds, ctype)
    return bool(c) and c.get("status") == "True"


def set_condition(conds: list[dict], ctype: str, status: str, reason: str, message: str,
                  generation: int, now: str | None = None) -> bool:
    """Upsert a condition; returns True when anything changed."""
    now = now or now_rfc3339()
    cur = find(conds, ctype)
    if cur is None:
        conds.append({"type": ctype, "status": status, "observedGeneration": generation,
                      "lastTransitionTime": now, "reason": reason, "message": message})
        return True
    changed = False
    if cur.get("status") != status:
        cur["status"] = status
        cur["lastTransitionTime"] = now
        changed = True
    for k, v in (("reason", reason), ("message", message), ("observedGeneration", generation)):
        if cur.get(k) != v:
            cur[k] = v
            changed = True
    return changed
