"""Node registration and the agent's Node heartbeat.

The kubelet owns a Node: it creates the object, and it writes ``status.capacity``,
``status.allocatable`` (from the device plugins — the only advertising path the reference's GPU
node side uses, GPU调度平台搭建.md:128-132) and the ``Ready`` condition with its heartbeat. The
agent adds facts of its own and nothing else:

* metadata: GPU labels and the agent-endpoint annotation, as a JSON merge patch of
  ``metadata.labels`` / ``metadata.annotations`` only. A Node that does not exist yet is not
  created (agent RBAC has no ``nodes: create``): registration waits for the kubelet;
* status: exactly two conditions, ``GPUPoolAgentReady`` and ``ROCmReady`` (the node preflight,
  SURVEY B2), sent as a strategic merge patch of ``status.conditions`` (merge key ``type``). No
  GET-modify-PATCH of ``status``: the apiserver merges the two entries into whatever the kubelet
  wrote last, so a kubelet write that lands between two agent calls survives.

``lastTransitionTime`` follows the ``metav1.Condition`` contract: it moves only when
the condition's status flips. The agent seeds what it last published from one read of the Node at
start (its own two conditions), so a restart does not reset them either.
"""
from __future__ import annotations

import datetime as _dt
import logging
from typing import Callable

log = logging.getLogger("gpupool.agent.node")

OWN_CONDITIONS = ("GPUPoolAgentReady", "ROCmReady")


def now_rfc3339() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


class NodeRegistrar:
    """``client``: a ``gpupool.kube.Client``; ``conditions()`` returns the agent's current
    ``{type: (status, reason, message)}`` for the types in ``OWN_CONDITIONS``."""

    def __init__(self, client, node: str, labels: dict[str, str], annotations: dict[str, str],
                 conditions: Callable[[], dict[str, tuple[str, str, str]]],
                 clock: Callable[[], str] = now_rfc3339):
        self.client = client
        self.node = node
        self.labels = dict(labels)
        self.annotations = dict(annotations)
        self.conditions = conditions
        self.clock = clock
        self.registered = False
        self.seeded = False
        # type -> (status, lastTransitionTime) as last published (or found at start)
        self.published: dict[str, tuple[str, str]] = {}
        self.stats = {"heartbeats": 0, "heartbeat_failures": 0, "register_waits": 0}

    # ------------------------------------------------------------ metadata
    def register(self) -> bool:
        """Labels + annotations onto the kubelet's Node. False while the Node does not exist."""
        from ..kube import NODES, KubeError
        try:
            node = self.client.patch(NODES, self.node, {"metadata": {
                "labels": self.labels, "annotations": self.annotations}})
        except KubeError as e:
            if e.code == 404:
                self.stats["register_waits"] += 1
                return False
            raise
        self.registered = True
        self._seed(node)
        return True

    def _seed(self, node: dict) -> None:
        """Remember the agent's own conditions as a previous process left them (read only)."""
        if self.seeded:
            return
        for c in (node.get("status") or {}).get("conditions") or []:
            if c.get("type") in OWN_CONDITIONS and c.get("lastTransitionTime"):
                self.published.setdefault(c["type"], (c.get("status", ""),
                                                       c["lastTransitionTime"]))
        self.seeded = True

    # ------------------------------------------------------------ status
    def patch_body(self) -> dict:
        """The strategic merge patch of one heartbeat: the agent's own conditions only."""
        now = self.clock()
        conds = []
        for ctype, (status, reason, message) in sorted(self.conditions().items()):
            if ctype not in OWN_CONDITIONS:
                raise ValueError(f"{ctype} is not an agent-owned Node condition")
            prev = self.published.get(ctype)
            ltt = prev[1] if prev and prev[0] == status else now
            conds.append({"type": ctype, "status": status, "reason": reason, "message": message,
                          "lastHeartbeatTime": now, "lastTransitionTime": ltt})
        return {"status": {"conditions": conds}}

    def heartbeat(self) -> bool:
        from ..kube import NODES, KubeError
        try:
            if not self.registered and not self.register():
                return False
        except (KubeError, OSError) as e:
            self.stats["heartbeat_failures"] += 1
            log.warning("node registration failed: %s", e)
            return False
        body = self.patch_body()
        try:
            self.client.patch(NODES, self.node, body, sub="status", ptype="strategic")
        except (KubeError, OSError) as e:
            self.stats["heartbeat_failures"] += 1
            if isinstance(e, KubeError) and e.code == 404:  # the Node was deleted: register again
                self.registered = False
            log.warning("node heartbeat failed: %s", e)
            return False
        for c in body["status"]["conditions"]:
            self.published[c["type"]] = (c["status"], c["lastTransitionTime"])
        self.stats["heartbeats"] += 1
        return True
