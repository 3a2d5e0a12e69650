"""Device-plugin glue (a mixin of ``agent.Agent``): what each extended resource advertises, the
advertised-set bookkeeping a claim waits on, GetPreferredAllocation and Allocate's container spec
(devices, ROCR_VISIBLE_DEVICES, torchrun env, slot isolation mounts).
"""
from __future__ import annotations

import time

from ..api import schema
from ..ops import devlib
from .common import SLOT_SEP, gpu_of


class AdvertiseMixin:

    def plugin_devices(self, resource: str) -> list[dict]:
        """The device-plugin view of ``resource``: one entry per advertised device ID. A GPU of a
        pool with ``sharing.replicasPerGPU`` = K is K IDs ``<uuid>::<slot>``, all with the GPU's
        health (HAMi / time-slicing style: the kubelet places up to K pods on it)."""
        with self.lock:
            out = []
            for u, rec in sorted(self.records.items(),
                                 key=lambda kv: self.by_uuid.get(kv[0], {}).get("index", 99)):
                if rec.get("resourceName", schema.DEFAULT_RESOURCE) != resource:
                    continue
                k = self._slots_of(rec)
                ok = self._advertisable(u)
                numa = self.by_uuid.get(u, {}).get("numa")
                for i in range(k):
                    out.append({"id": u if k == 1 else f"{u}{SLOT_SEP}{i}", "uuid": u,
                                "advertisable": ok, "numa": numa})
            return out

    def mark_advertised(self, resource: str, healthy: set[str] | None) -> None:
        with self.lock:
            plugin = self.plugins.get(resource)
            before = set(self.advertised.get(resource, set()))
            if healthy is None:
                if plugin is None or plugin.streams <= 0:
                    self.advertised[resource] = set()
            else:
                self.advertised[resource] = set(healthy)
            flipped = before ^ self.advertised.get(resource, set())
            pools = {self.records[u]["poolUID"] for u in flipped if u in self.records}
        with self._adv_cv:
            self._adv_gen += 1
            self._adv_cv.notify_all()
        if pools:  # readiness depends on the advertised bit: tell the manager
            self._bump(pools)

    def _advertise_done(self, resource: str, uuids: list[str]) -> bool:
        """Every advertisable GPU of ``uuids`` reached the kubelet — or there is no registered
        plugin to wait for (no kubelet: readiness follows via events, never block the claim)."""
        with self.lock:
            want = [u for u in uuids if self._advertisable(u)]
            if all(u in self.advertised.get(resource, set()) for u in want):
                return True
            plugin = self.plugins.get(resource)
            return plugin is None or not plugin.registered

    def _wait_advertised(self, resource: str, uuids: list[str]) -> None:
        if not self.cfg.plugin_dir:
            return
        deadline = time.monotonic() + self.cfg.advertise_wait_s
        while time.monotonic() < deadline:
            with self._adv_cv:
                gen = self._adv_gen
            if self._advertise_done(resource, uuids):
                return
            with self._adv_cv:
                self._adv_cv.wait_for(lambda: self._adv_gen != gen, timeout=0.05)


    def _ensure_plugin(self, resource: str) -> None:
        if not self.cfg.plugin_dir:
            return
        with self.lock:
            if resource in self.plugins:
                return
            from .deviceplugin.server import DevicePluginServer
            p = DevicePluginServer(self, resource, self.cfg.plugin_dir)
            self.plugins[resource] = p
        p.start()

    def _notify_plugins(self, sync: bool = False) -> None:
        for p in list(self.plugins.values()):
            p.notify(sync)

    def preferred(self, resource: str, available: list[str], must: list[str], size: int) -> list[str]:
        if any(SLOT_SEP in i for i in available + must):
            # shared GPUs: a pod's slots go to as few GPUs as possible, lowest index first
            with self.lock:
                idx = {u: self.by_uuid.get(u, {}).get("index", 99) for u in
                       {gpu_of(i) for i in available + must}}
            def key(i: str) -> tuple[int, int]:
                u, _, slot = i.partition(SLOT_SEP)
                return idx.get(u, 99), int(slot or 0)
            rest = sorted((i for i in available if i not in must), key=key)
            return list(must) + rest[:max(0, size - len(must))]
        with self.lock:
            idx = {u: self.by_uuid[u]["index"] for u in available + must if u in self.by_uuid}
            inv = {v: k for k, v in idx.items()}
            topo = self.snap.get("topology") or {}
            n = len(self.snap["devices"])
            weights = topo.get("weights") or [[0 if i == j else 15 for j in range(n)]
                                              for i in range(n)]
            numa = [d.get("numa", 0) for d in sorted(self.snap["devices"], key=lambda x: x["index"])]
        need = size - len(must)
        cand = [idx[u] for u in available if u not in must and u in idx]
        sel = devlib.select(need, cand, [idx[u] for u in must if u in idx], "xgmi-packed",
                            weights, numa) if need > 0 else []
        return list(must) + [inv[i] for i in sel]

    def allocate_spec(self, resource: str, ids: list[str]) -> dict:
        slots = list(ids)
        ids = list(dict.fromkeys(gpu_of(i) for i in ids))  # slots of shared GPUs -> the GPUs
        for u in ids:  # a pod never starts while the HBM scrubber still frees its buffer
            if not self.scrubber.wait_released(u):
                raise ValueError(f"device {u}: HBM scrub buffer still being released")
        self._watch_pods()
        with self.lock:
            hip, render = [], []
            for u in ids:
                rec = self.records.get(u)
                if not rec or rec.get("resourceName", schema.DEFAULT_RESOURCE) != resource:
                    raise ValueError(f"device {u} is not in any pool advertised as {resource}")
                if not self._advertisable(u):
                    raise ValueError(f"device {u} is not healthy/allocatable (state "
                                     f"{rec.get('state')})")
                d = self.by_uuid[u]
                hip.append(d.get("hipUUID") or str(d["index"]))
                if d.get("renderNode"):
                    render.append(d["renderNode"])
            # ROCR_VISIBLE_DEVICES pins the container to exactly its GPUs (HIP ordinals then
            # start at 0); GPUPOOL_NUM_GPUS is the per-pod world-size hint and PET_NPROC_PER_NODE
            # the torchrun default for --nproc-per-node (torch.distributed.run reads PET_* env),
            # so a plain `torchrun train.py` in the pod starts one rank per allotted GPU over
            # RCCL (the reference's Kubeflow operator sets PET_*, GPU调度平台搭建.md:623).
            envs = {"ROCR_VISIBLE_DEVICES": ",".join(hip),
                    "GPUPOOL_DEVICE_UUIDS": ",".join(ids),
                    "GPUPOOL_NUM_GPUS": str(len(ids)),
                    "PET_NPROC_PER_NODE": str(len(ids)),
                    "GPUPOOL_NODE": self.cfg.node}
            mounts: list[dict] = []
            if slots != ids:  # time-sliced: the pod shares these GPUs with other pods
                envs["GPUPOOL_GPU_SLOTS"] = ",".join(slots)
                envs.update(self._isolation_env(slots, mounts))
        if "GPUPOOL_HBM_LIMIT_BYTES" in envs:  # the pod-wide HBM account (file I/O: off the lock)
            acct = self._share_account(slots, int(envs["GPUPOOL_HBM_LIMIT_BYTES"]), ids)
            if acct:
                mounts.append({"container_path": self.SHARE_ACCOUNT_PATH, "host_path": acct,
                               "read_only": False})
                envs["GPUPOOL_SHARE_ACCOUNT"] = self.SHARE_ACCOUNT_PATH
                # the limit itself, read-only: the account's counters must be writable by the
                # pod's processes, so its header limit is the pod's to edit — this one is not
                # (the library takes the smallest limit it is given)
                mounts.append({"container_path": self.SHARE_LIMIT_PATH,
                               "host_path": acct[:-len(".acct")] + ".limit", "read_only": True})
                envs["GPUPOOL_SHARE_LIMIT"] = self.SHARE_LIMIT_PATH
        return {"envs": envs, "devices": ["/dev/kfd"] + render, "mounts": mounts,
                "annotations": {schema.ANN_POD_DEVICES: ",".join(ids)}}
