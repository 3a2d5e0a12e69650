"""Isolated GPU sharing on a real MI355X (spec.sharing.hbmBytesPerSlot / cuPerSlot; the HAMi layer
of the reference platform, GPU调度平台搭建.md:289-298): libgpupool_share.so, loaded by the ROCm
runtime through HSA_TOOLS_LIB exactly as the device plugin's Allocate sets it up, caps a slot's HBM
and confines its waves to the slot's CUs. Each case runs in child processes (the library is loaded
at HSA init), with a time limit."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB = os.path.join(ROOT, "build", "native", "libgpupool_share.so")
pytestmark = pytest.mark.gpu
GiB = 1 << 30

ALLOC = r"""
import json, sys, time, torch
hold = int(sys.argv[1]); extra = int(sys.argv[2]); wait = float(sys.argv[3])
free, total = torch.cuda.mem_get_info(0)
out = {"total": total, "free": free}
a = torch.empty(hold, dtype=torch.uint8, device="cuda")
a.fill_(1); torch.cuda.synchronize()
out["held"] = hold
try:
    b = torch.empty(extra, dtype=torch.uint8, device="cuda"); b.fill_(2); torch.cuda.synchronize()
    out["extra"] = "ok"
except torch.OutOfMemoryError as e:
    out["extra"] = "oom"
print(json.dumps(out), flush=True)
time.sleep(wait)
"""

CENSUS = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from gpupool.ops import probe
probe.init()
r = probe.run(0, hbm_bytes=64 << 20, mfma=True, gemm_n=1024, cuKeys=1)
print(json.dumps({"keys": r["cus"]["cuKeys"], "verified": r["cus"]["mfmaVerified"],
                  "perXcd": r["cus"]["perXcd"], "mfmaOk": r["mfma"]["elementMismatches"] == 0}))
"""


SECOND = r"""
import json, sys, torch
size = int(sys.argv[1])
torch.zeros(1, device="cuda"); torch.cuda.synchronize()
free, total = torch.cuda.mem_get_info(0)

def attempt():
    try:
        b = torch.empty(size, dtype=torch.uint8, device="cuda"); b.fill_(3); torch.cuda.synchronize()
        del b
        torch.cuda.empty_cache()
        return "ok"
    except torch.OutOfMemoryError:
        torch.cuda.empty_cache()
        return "oom"

print(json.dumps({"free": free, "total": total, "first": attempt()}), flush=True)
sys.stdin.readline()
print(json.dumps({"second": attempt()}), flush=True)
"""


def _account(path: str, limit: int) -> str:
    """The agent's account file (gpupool/agent/agent.py _share_account)."""
    buf = bytearray(16384)
    buf[0:24] = b"GPSHARE1" + limit.to_bytes(8, "little") + (1).to_bytes(4, "little") + \
        (1).to_bytes(4, "little")
    with open(path, "wb") as f:
        f.write(bytes(buf))
    return path


def _env(**kw) -> dict:
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("HSA_TOOLS_LIB", "GPUPOOL_HBM_LIMIT_BYTES", "GPUPOOL_CU_MASK", "GPUPOOL_SHARE_ACCOUNT"):
        env.pop(k, None)
    env.update({k: str(v) for k, v in kw.items()})
    return env


def _json(p: subprocess.Popen, timeout: float = 90) -> dict:
    deadline = time.monotonic() + timeout
    line = ""
    while time.monotonic() < deadline:
        line = p.stdout.readline()
        if line.startswith("{"):
            return json.loads(line)
        if not line and p.poll() is not None:
            break
    p.kill()
    raise AssertionError(f"no result (rc={p.poll()}): {line} {p.stderr.read()[-2000:]}")


def test_hbm_budget_per_slot_and_sibling_unaffected():
    """Slot A (8 GiB budget) holds 6 GiB, then asks for 10 GiB more -> hipErrorOutOfMemory
    (torch.OutOfMemoryError); torch.cuda.mem_get_info reports the 8 GiB budget. Its sibling slot,
    running at the same time with its own 8 GiB, allocates its 6 GiB fine; an unshared process
    allocates 16 GiB."""
    assert os.path.exists(LIB), "build the native targets first"
    slot = _env(HSA_TOOLS_LIB=LIB, GPUPOOL_HBM_LIMIT_BYTES=8 * GiB)
    a = subprocess.Popen([sys.executable, "-c", ALLOC, str(6 * GiB), str(10 * GiB), "20"], env=slot,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        ra = _json(a)
        b = subprocess.Popen([sys.executable, "-c", ALLOC, str(6 * GiB), str(1 * GiB), "0"],
                             env=slot, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        rb = _json(b)
        b.wait(timeout=60)
    finally:
        a.kill()
        a.wait(timeout=30)
    assert ra["total"] == 8 * GiB, ra
    assert ra["held"] == 6 * GiB and ra["extra"] == "oom", ra
    assert rb["held"] == 6 * GiB and rb["extra"] == "ok", rb
    free = subprocess.run([sys.executable, "-c", ALLOC, str(16 * GiB), str(1 * GiB), "0"],
                          env=_env(), capture_output=True, text=True, timeout=120)
    rf = json.loads([x for x in free.stdout.splitlines() if x.startswith("{")][-1])
    assert rf["total"] > 200 * GiB and rf["extra"] == "ok", rf


def test_cu_share_confines_waves_to_the_slot():
    """Four slots of 64 CUs: each slot's census (every CU that runs an MFMA wave marks its
    XCC/SE/SH/CU hardware id) sees at most its own 64 CUs, the four slots' CU sets are disjoint,
    and together they cover the GPU's 256; an unmasked process reaches all 256."""
    assert os.path.exists(LIB), "build the native targets first"
    full = subprocess.run([sys.executable, "-c", CENSUS, ROOT], env=_env(), capture_output=True,
                          text=True, timeout=120)
    assert full.returncode == 0, full.stderr[-2000:]
    all_keys = set(json.loads(full.stdout.splitlines()[-1])["keys"])
    assert len(all_keys) == 256, len(all_keys)
    seen = []
    for i in range(4):
        r = subprocess.run([sys.executable, "-c", CENSUS, ROOT],
                           env=_env(HSA_TOOLS_LIB=LIB, GPUPOOL_CU_MASK=f"{64 * i}-{64 * i + 63}"),
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        out = json.loads(r.stdout.splitlines()[-1])
        assert out["mfmaOk"], out
        keys = set(out["keys"])
        print(f"slot {i}: {len(keys)} CUs, per XCD {out['perXcd']}")
        assert 0 < len(keys) <= 64, (i, len(keys), out["perXcd"])
        seen.append(keys)
    for i in range(4):
        for j in range(i + 1, 4):
            assert not (seen[i] & seen[j]), (i, j, sorted(seen[i] & seen[j])[:8])
    assert set().union(*seen) <= all_keys


def test_hbm_budget_is_the_pods_across_its_processes(tmp_path):
    """GPUPOOL_SHARE_ACCOUNT: two processes of one pod share its 8 GiB. Process A holds 6 GiB;
    process B then sees at most 2 GiB free (mem_get_info) and a 4 GiB allocation fails. A is killed
    with SIGKILL (no free runs); B's next 4 GiB allocation finds the budget exhausted, returns the
    dead process's bytes to the account and succeeds."""
    assert os.path.exists(LIB), "build the native targets first"
    acct = _account(str(tmp_path / "pod.acct"), 8 * GiB)
    env = _env(HSA_TOOLS_LIB=LIB, GPUPOOL_HBM_LIMIT_BYTES=8 * GiB, GPUPOOL_SHARE_ACCOUNT=acct)
    a = subprocess.Popen([sys.executable, "-c", ALLOC, str(6 * GiB), str(1 << 20), "60"], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    b = None
    try:
        ra = _json(a)
        assert ra["held"] == 6 * GiB and ra["extra"] == "ok", ra
        used = int.from_bytes(open(acct, "rb").read()[64:72], "little")
        assert 6 * GiB <= used < 7 * GiB, used
        b = subprocess.Popen([sys.executable, "-c", SECOND, str(4 * GiB)], env=env, text=True,
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        rb = _json(b)
        print("pod account after A + B:", rb, "bytes", used)
        # hipMemGetInfo in B reports what the pod has left, not what B holds
        assert rb["total"] == 8 * GiB and rb["free"] <= 8 * GiB - used, (rb, used)
        assert rb["first"] == "oom", rb
        a.kill()
        a.wait(timeout=30)
        b.stdin.write("\n")
        b.stdin.flush()
        rb2 = _json(b)
        assert rb2["second"] == "ok", rb2
        b.wait(timeout=60)
    finally:
        for p in (a, b):
            if p is not None and p.poll() is None:
                p.kill()
                p.wait(timeout=30)


def test_smallest_slot_spans_every_xcd():
    """The smallest slot the agent builds on an SPX MI355X is 8 CUs (cuPerSlot below the XCD count
    is refused: a mask that leaves an XCD empty is not applied by the hardware at all, see
    gpupool/agent/slots.py and profiles/r4b_cu_mask_layouts.json). Four 8-CU slots: each one's
    census shows exactly one CU on every XCD, and the slots' CUs are disjoint."""
    from gpupool.agent.agent import _ranges
    from gpupool.agent.slots import cu_floor, slot_cus
    assert os.path.exists(LIB), "build the native targets first"
    spx = {"asic": {"computeUnits": 256}, "partition": {"compute": "SPX"}}
    assert cu_floor({"replicasPerGPU": 4, "cuPerSlot": 4}, spx)
    assert not cu_floor({"replicasPerGPU": 4, "cuPerSlot": 8}, spx)
    seen = []
    for i in range(4):
        bits, layout = slot_cus(i, 32, 8, 256, 8)
        r = subprocess.run([sys.executable, "-c", CENSUS, ROOT],
                           env=_env(HSA_TOOLS_LIB=LIB, GPUPOOL_CU_MASK=_ranges(bits)),
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        out = json.loads(r.stdout.splitlines()[-1])
        print(f"8-CU slot {i}: mask {_ranges(bits)} per XCD {out['perXcd']}")
        assert out["mfmaOk"], out
        assert out["perXcd"] == [1] * 8, (i, out["perXcd"])
        seen.append(set(out["keys"]))
    for i in range(4):
        for j in range(i + 1, 4):
            assert not (seen[i] & seen[j]), (i, j)


ACCT_ALLOC = r"""
import json, sys, torch
torch.zeros(1, device="cuda"); torch.cuda.synchronize()
a = torch.empty(int(sys.argv[1]), dtype=torch.uint8, device="cuda"); a.fill_(1)
torch.cuda.synchronize()
print(json.dumps({"held": int(sys.argv[1])}), flush=True)
sys.stdin.readline()  # hold the memory until the parent has read the account
"""


def test_hbm_account_is_keyed_by_the_gpus_hip_uuid(tmp_path):
    """A version-2 account names its GPUs: the real GPU's HIP UUID (HSA agent UUID) sits at
    account index 1 behind a GPU this box does not have. A process that sees only that GPU (its
    HIP ordinal 0) must charge index 1, not index 0 — so ranks with different
    ROCR_VISIBLE_DEVICES charge one counter per physical GPU."""
    from gpupool.agent.slots import account_bytes
    info = subprocess.run([sys.executable, "-c",
                           "import json,sys; sys.path.insert(0, sys.argv[1]);"
                           "from gpupool.ops import probe; probe.init();"
                           "print(json.dumps(probe.identify(0)))", ROOT],
                          env=_env(), capture_output=True, text=True, timeout=120)
    assert info.returncode == 0, info.stderr[-2000:]
    uuid = json.loads(info.stdout.splitlines()[-1])["hipUUID"]
    assert uuid.startswith("GPU-"), uuid
    acct = tmp_path / "pod.acct"
    acct.write_bytes(account_bytes(8 * GiB, ["x::0"], ["GPU-0000000000000000", uuid]))
    p = subprocess.Popen([sys.executable, "-c", ACCT_ALLOC, str(1 * GiB)], text=True,
                         env=_env(HSA_TOOLS_LIB=LIB, GPUPOOL_HBM_LIMIT_BYTES=8 * GiB,
                                  GPUPOOL_SHARE_ACCOUNT=str(acct), ROCR_VISIBLE_DEVICES=uuid),
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        assert _json(p)["held"] == 1 * GiB
        raw = acct.read_bytes()
    finally:
        p.kill()
        p.wait(timeout=30)
    used0 = int.from_bytes(raw[64:72], "little")
    used1 = int.from_bytes(raw[72:80], "little")
    print(f"account: index0 {used0} B, index1 ({uuid}) {used1} B")
    assert used0 == 0, used0
    assert 1 * GiB <= used1 < 2 * GiB, used1


def test_share_library_loads_and_reports_in_this_process():
    """The tools library as the test process itself maps it (the isolation tests above load it in
    their child processes through HSA_TOOLS_LIB): it loads with nothing but libc and its
    diagnostics entry point answers — not hooked here (ROCr never called OnLoad), so no limits."""
    import ctypes
    lib = ctypes.CDLL(LIB)
    buf = ctypes.create_string_buffer(512)
    n = lib.gpupool_share_stats(buf, len(buf))
    st = json.loads(buf.value.decode())
    assert n > 0 and st["limit"] == 0 and st["maskBits"] == 0 and st["shared"] == 0, st
    assert hasattr(lib, "OnLoad") and hasattr(lib, "OnUnload")
