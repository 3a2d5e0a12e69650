"""GPU sharing with isolated slots (a mixin of ``agent.Agent``; HAMi's role in the reference,
GPU调度平台搭建.md:289-298): per-slot CU masks and HBM budgets, libgpupool_share.so installed on the
host for Allocate to mount, per-allocation HBM account files and their garbage collection.
"""
from __future__ import annotations

import json
import os
import time
from uuid import uuid4

from . import slots as slotlib
from .common import SLOT_SEP, log, _ranges


class SharingMixin:
    @staticmethod
    def _slots_of(rec: dict) -> int:
        """spec.sharing.replicasPerGPU of the record's pool (time-sliced slots per GPU)."""
        try:
            return max(1, int(((rec.get("policy") or {}).get("sharing") or {})
                              .get("replicasPerGPU") or 1))
        except (TypeError, ValueError):
            return 1

    SHARE_LIB_DIR = "/opt/gpupool/lib"  # where the pod sees libgpupool_share.so
    SHARE_ACCOUNT_PATH = "/var/run/gpupool/share.acct"  # where it sees its pod's HBM account
    SHARE_LIMIT_PATH = "/var/run/gpupool/share.limit"  # ...and, read-only, its limit
    SHARE_LIB = "libgpupool_share.so"

    def _install_share_lib(self) -> str | None:
        """Copy libgpupool_share.so from the agent's own tree (in the image) into
        ``<state_dir>/lib``. The state dir is the DaemonSet's hostPath (/var/lib/gpupool), so the
        copy exists on the HOST, where the container runtime resolves an Allocate mount's host
        path — the image path it came from does not. Atomic (temp file + rename); a copy whose
        bytes already match is kept, so pods that mapped it keep a stable inode. Returns the
        host directory, or None (isolated slots then fail their Allocate, loudly)."""
        from ..ops import native_dir
        src = os.path.join(native_dir(), self.SHARE_LIB)
        dst_dir = os.path.join(self.cfg.state_dir, "lib")
        dst = os.path.join(dst_dir, self.SHARE_LIB)
        try:
            with open(src, "rb") as f:
                data = f.read()
        except OSError as e:
            log.warning("isolated GPU sharing unavailable: %s not readable (%s)", src, e)
            return None
        try:
            os.makedirs(dst_dir, exist_ok=True)
            try:
                with open(dst, "rb") as f:
                    if f.read() == data:
                        return dst_dir
            except OSError:
                pass
            tmp = f"{dst}.{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(data)
                f.flush()
                os.fsync(f.fileno())
            os.chmod(tmp, 0o755)
            os.replace(tmp, dst)
            return dst_dir
        except OSError as e:
            log.warning("isolated GPU sharing unavailable: cannot install %s (%s)", dst, e)
            return None

    def share_mounts(self) -> list[str]:
        """Every host path an Allocate may mount (the deploy manifest must declare hostPath
        volumes covering them; tests/unit/test_deploy_manifests.py checks it)."""
        return [os.path.join(self.cfg.state_dir, "lib"), os.path.join(self.cfg.state_dir, "share")]

    def _share_account(self, slots: list[str], limit: int, gpus: list[str]) -> str | None:
        """One HBM account per allocation, shared by every process of the container: 16 KiB,
        magic + per-GPU limit + the GPUs' HIP UUIDs (what the library matches each HSA agent
        against, so ranks with different ROCR_VISIBLE_DEVICES charge the same counter for the same
        GPU), zeroed counters, the slot ids as text. A slot belongs to one container at a time, so
        an earlier account naming any of these slots belongs to a container that is gone: it is
        deleted here (and by the sampler once the kubelet lists none of its slots). Returns the
        host path (None if the state directory is not writable: the budget is then per process)."""
        d = os.path.join(self.cfg.state_dir, "share")
        mine = set(slots)
        try:
            os.makedirs(d, exist_ok=True)
            for name in os.listdir(d):
                if not name.endswith(".acct"):
                    continue
                path = os.path.join(d, name)
                if mine & set(slotlib.account_slots(path) or ()):
                    for p in (path, path[:-len(".acct")] + ".limit"):
                        try:
                            os.unlink(p)
                        except FileNotFoundError:  # the sampler's GC got there first
                            pass
            with self.lock:
                uuids = [(self.by_uuid.get(u) or {}).get("hipUUID") or "" for u in gpus]
            if not all(uuids):
                # a GPU without a hipUUID (amd-smi CLI backend, empty serial) cannot be matched by
                # identity: a version-2 account would match no GPU and silently fall back to a
                # per-process budget. A version-1 account maps by enumeration order instead.
                log.warning("HBM account for %s: GPU(s) without hipUUID %s; ordinal mapping",
                            slots, [u for u, h in zip(gpus, uuids) if not h])
                uuids = []
            stem = os.path.join(d, uuid4().hex)
            path = stem + ".acct"
            fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o666)
            try:
                os.write(fd, slotlib.account_bytes(limit, slots, uuids))
                os.fchmod(fd, 0o666)  # pods may run as any user
            finally:
                os.close(fd)
            fd = os.open(stem + ".limit", os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o644)
            try:
                os.write(fd, slotlib.limit_bytes(limit))
            finally:
                os.close(fd)
            return path
        except OSError as e:
            log.warning("HBM account for %s not created (%s): budget is per process", slots, e)
            return None

    def gc_share_accounts(self, now: float | None = None) -> list[str]:
        """Delete the HBM accounts of pods that are gone: no device ID the kubelet's last
        PodResources listing shows is one of the account's slots. Runs every sample period."""
        pod_ids = self._pod_ids
        if pod_ids is None:
            return []
        listed_at, live = pod_ids
        # an account made after that listing began may belong to a pod it could not show yet
        cutoff = min(listed_at, (now or time.time()) - self.cfg.share_acct_grace_s)
        gone = slotlib.gc_accounts(os.path.join(self.cfg.state_dir, "share"), live, cutoff)
        if gone:
            log.info("removed %d HBM account(s) of exited pods", len(gone))
        return gone

    def _slot_layout(self, uuid: str, rec: dict) -> dict:
        """The isolation a GPU's slots get under its pool's spec.sharing: per-slot CU-mask bits and
        layout, the enforced per-slot HBM budget. Memoised per (GPU, sharing policy, CU count,
        partition, HBM size): node views ask for it on every observe. Called under self.lock."""
        share = (rec.get("policy") or {}).get("sharing") or {}
        d = self.by_uuid.get(uuid) or {}
        key = (uuid, json.dumps(share, sort_keys=True), (d.get("asic") or {}).get("computeUnits"),
               json.dumps(d.get("partition") or {}, sort_keys=True), d.get("memTotalBytes"))
        hit = self._layouts.get(key)
        if hit is None:
            if len(self._layouts) > 4096:
                self._layouts.clear()
            hit = self._layouts[key] = self._compute_slot_layout(rec, share, d)
        return {k: (list(v) if isinstance(v, list) else v) for k, v in hit.items()}

    def _compute_slot_layout(self, rec: dict, share: dict, d: dict) -> dict:
        k = self._slots_of(rec)
        out: dict = {"replicasPerGPU": k}
        per_slot = int(share.get("hbmBytesPerSlot") or 0)
        if per_slot > 0:
            # never more than a fair share of what the agent leaves free, whatever the spec says
            # (claims of an overcommitted pool are refused; this covers a later spec edit)
            mem = int(d.get("memTotalBytes") or 0)
            if mem > 0:
                per_slot = min(per_slot, max(0, mem - self.cfg.hbm_reserve_bytes) // k)
            out["hbmBytesPerSlot"] = per_slot
        cu = int(share.get("cuPerSlot") or 0)
        if cu > 0:
            cus = int((d.get("asic") or {}).get("computeUnits") or 256)
            xcds = slotlib.xcd_count(d)
            masks, layout = [], "striped"
            for i in range(k):
                bits, layout = slotlib.slot_cus(i, k, cu, cus, xcds)
                masks.append(bits)
            out.update({"cuLayout": layout, "cuPerSlot": len(masks[0]), "xcds": xcds,
                        "masks": masks,
                        # per slot: its CU-mask bits and the XCDs they land on (node views)
                        "slotCUMasks": [_ranges(m) for m in masks],
                        "slotXcds": [_ranges(slotlib.slot_xcds(m, xcds)) for m in masks]})
        return out

    def _isolation_env(self, slots: list[str], mounts: list[dict]) -> dict[str, str]:
        """spec.sharing.hbmBytesPerSlot / cuPerSlot of the pool owning these slots: the ROCm
        runtime loads libgpupool_share.so (HSA_TOOLS_LIB) into the pod, which caps its HBM per
        GPU at (its slots on that GPU) x hbmBytesPerSlot and confines its queues to its slots'
        CUs — contiguous mask bits, disjoint from the other slots, the same number of CUs on every
        XCD (slots.py: why not whole XCDs). The library is mounted from its host copy under the
        state dir. Called under self.lock."""
        per_gpu: dict[str, list[int]] = {}
        for sid in slots:
            u, _, i = sid.partition(SLOT_SEP)
            per_gpu.setdefault(u, []).append(int(i or 0))
        hbm, cu_mask = 0, set()
        per_gpu_mask: dict[str, set[int]] = {}  # hipUUID -> the CUs of this pod's slots there
        for u, idx in per_gpu.items():
            lay = self._slot_layout(u, self.records.get(u) or {})
            if lay.get("hbmBytesPerSlot"):
                hbm = max(hbm, lay["hbmBytesPerSlot"] * len(idx))
            if "masks" in lay:
                hip = (self.by_uuid.get(u) or {}).get("hipUUID") or ""
                for i in idx:
                    bits = lay["masks"][i % len(lay["masks"])]
                    cu_mask.update(bits)
                    if hip:
                        per_gpu_mask.setdefault(hip, set()).update(bits)
        if not hbm and not cu_mask:
            return {}
        if not self.share_lib_dir:
            raise ValueError("isolated GPU sharing requested but libgpupool_share.so is not "
                             f"installed under {self.cfg.state_dir}/lib (see the agent log)")
        mounts.append({"container_path": self.SHARE_LIB_DIR, "host_path": self.share_lib_dir,
                       "read_only": True})
        env = {"HSA_TOOLS_LIB": f"{self.SHARE_LIB_DIR}/{self.SHARE_LIB}"}
        xcds = {lay.get("xcds") for lay in (self._slot_layout(u, self.records.get(u) or {})
                                             for u in per_gpu) if lay.get("xcds")}
        if cu_mask and xcds:  # a narrowed app mask must keep a CU on each XCD (share.cc)
            env["GPUPOOL_CU_XCDS"] = str(max(xcds))
        if hbm:  # allocate_spec adds the pod-wide account file (GPUPOOL_SHARE_ACCOUNT)
            env["GPUPOOL_HBM_LIMIT_BYTES"] = str(hbm)
        if cu_mask:
            # each GPU's own slot CUs, keyed by the UUID the library reads from the queue's agent: a
            # pod holding slot 0 of GPU A and slot 1 of GPU B must not get the union on both (it
            # overlaps the sibling tenants); the union stays as the fallback for a GPU not named
            env["GPUPOOL_CU_MASK"] = _ranges(sorted(cu_mask))
            env["GPUPOOL_CU_LAYOUT"] = "striped"
            if per_gpu_mask:
                env["GPUPOOL_CU_MASKS"] = ";".join(f"{h}={_ranges(sorted(b))}"
                                                   for h, b in sorted(per_gpu_mask.items()))
        return env
