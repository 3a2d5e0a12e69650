#!/usr/bin/env python3
"""Slot-interference A/B on one MI355X: CU-masked slots vs plain time-slicing.

Four 64-CU slots per GPU (spec.sharing replicasPerGPU=4, cuPerSlot=64). Slot A (slot 0) is the
victim, slot B (slot 1) the aggressor; each is its own process, loading libgpupool_share.so through
HSA_TOOLS_LIB with GPUPOOL_CU_MASK exactly as an isolated slot's Allocate sets it up.

  striped:  A = mask bits 0-63, B = 64-127 (the agent's layout: 8 CUs of every XCD each; the
            slots share the XCDs' L2s — whole-XCD masks are not applied by the hardware,
            profiles/r4b_cu_mask_layouts.json)
  unmasked: A and B both on all 256 CUs (replicasPerGPU without cuPerSlot: time-slicing only)

Per layout and round (layouts interleaved round by round), the victim measures alone and then
while the aggressor streams HBM (2 GiB copy, L2-thrashing):
  * gemm — torch bf16 4096^3 matmul TFLOP/s (hipBLASLt), median of 10 timed batches of 10;
  * l2   — libmi355x_interfere.so L2-resident re-read of a 2 MB buffer, GB/s (median of 20);
and a CU census of each mask proves what the slot really runs on.

    python scripts/slot_interference_ab.py --rounds 3 --out gpurun_out/slot_ab.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gpupool.agent.agent import _ranges  # noqa: E402
from gpupool.agent.slots import slot_cus  # noqa: E402

NATIVE = os.path.join(ROOT, "build", "native")
SHARE = os.path.join(NATIVE, "libgpupool_share.so")
INTERFERE = os.path.join(NATIVE, "libmi355x_interfere.so")

GEMM = r"""
import json, torch
n = 4096
a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    c = a @ b
torch.cuda.synchronize()
ts = []
for _ in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 10)
ts.sort()
print(json.dumps({"tflops": 2 * n ** 3 / (ts[len(ts) // 2] * 1e9), "ms": ts[len(ts) // 2]}), flush=True)
"""

L2 = r"""
import ctypes, json, sys
lib = ctypes.CDLL(sys.argv[1])
g = ctypes.c_double()
rc = lib.mi355x_interfere_l2(0, ctypes.c_ulonglong(2 << 20), 256, 20, ctypes.byref(g))
print(json.dumps({"rc": rc, "GBps": g.value}), flush=True)
"""

STREAM = r"""
import ctypes, json, sys
lib = ctypes.CDLL(sys.argv[1])
lib.mi355x_interfere_stream.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_double,
                                        ctypes.POINTER(ctypes.c_double)]
g = ctypes.c_double()
print("go", flush=True)
rc = lib.mi355x_interfere_stream(0, 2 << 30, float(sys.argv[2]), ctypes.byref(g))
print(json.dumps({"rc": rc, "GBps": g.value}), flush=True)
"""

CENSUS = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from gpupool.ops import probe
probe.init()
r = probe.run(0, hbm_bytes=64 << 20, mfma=True, gemm_n=1024, cuKeys=1)
print(json.dumps({"cus": len(r["cus"]["cuKeys"]), "perXcd": r["cus"]["perXcd"]}), flush=True)
"""


def env_for(mask: list[int] | None) -> dict:
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("HSA_TOOLS_LIB", "GPUPOOL_CU_MASK", "GPUPOOL_HBM_LIMIT_BYTES", "GPUPOOL_SHARE_ACCOUNT"):
        env.pop(k, None)
    if mask is not None:
        env.update(HSA_TOOLS_LIB=SHARE, GPUPOOL_CU_MASK=_ranges(mask))
    return env


def run_json(code: str, args: list[str], env: dict, timeout: float = 120) -> dict:
    r = subprocess.run([sys.executable, "-c", code, *args], env=env, capture_output=True, text=True,
                       timeout=timeout)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not lines:
        raise RuntimeError(f"child failed rc={r.returncode}: {r.stderr[-1500:]}")
    return json.loads(lines[-1])


def victim(mask: list[int] | None) -> dict:
    env = env_for(mask)
    out = {"gemm": run_json(GEMM, [], env)["tflops"]}
    l2 = run_json(L2, [INTERFERE], env)
    if l2["rc"] != 0:
        raise RuntimeError(f"l2 victim rc={l2['rc']}")
    out["l2"] = l2["GBps"]
    return out


def contended(mask_a: list[int] | None, mask_b: list[int] | None, seconds: float) -> dict:
    agg = subprocess.Popen([sys.executable, "-c", STREAM, INTERFERE, str(seconds)], env=env_for(mask_b),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        line = agg.stdout.readline()
        if line.strip() != "go":
            raise RuntimeError(f"aggressor did not start: {line!r} {agg.stderr.read()[-1500:]}")
        time.sleep(0.5)  # the copy is running
        t0 = time.monotonic()
        out = victim(mask_a)
        busy = time.monotonic() - t0
        rest = agg.stdout.read()
        agg.wait(timeout=seconds + 60)
        res = json.loads([x for x in rest.splitlines() if x.startswith("{")][-1])
        out["aggressorGBps"] = res["GBps"]
        out["victimSeconds"] = busy
        if busy + 0.5 > seconds:
            out["warning"] = "victim outlasted the aggressor"
        return out
    finally:
        if agg.poll() is None:
            agg.kill()
            agg.wait(timeout=30)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=20.0, help="aggressor duration per round")
    ap.add_argument("--out", default="gpurun_out/slot_ab.json")
    a = ap.parse_args()
    for p in (SHARE, INTERFERE):
        if not os.path.exists(p):
            raise SystemExit(f"{p} missing: make -C native")
    layouts = {"striped": (slot_cus(0, 4, 64, 256, 8)[0], slot_cus(1, 4, 64, 256, 8)[0]),
               "unmasked": (None, None)}
    res: dict = {"config": {"slots": 4, "cuPerSlot": 64, "victim": "slot 0", "aggressor": "slot 1",
                            "gemm": "torch bf16 4096^3", "l2": "2 MB re-read x256 per launch",
                            "aggressorBuffer": "2 GiB copy"},
                 "masks": {k: {"victim": _ranges(v[0]) if v[0] else "all",
                               "aggressor": _ranges(v[1]) if v[1] else "all"}
                           for k, v in layouts.items()},
                 "census": {}, "rounds": []}
    for name, (ma, mb) in layouts.items():
        res["census"][name] = {"victim": run_json(CENSUS, [ROOT], env_for(ma)),
                               "aggressor": run_json(CENSUS, [ROOT], env_for(mb))}
        print(name, "census", res["census"][name], flush=True)
    for r in range(a.rounds):
        order = list(layouts) if r % 2 == 0 else list(reversed(list(layouts)))
        for name in order:
            ma, mb = layouts[name]
            alone = victim(ma)
            cont = contended(ma, mb, a.seconds)
            row = {"round": r, "layout": name, "alone": alone, "contended": cont,
                   "gemmSlowdown": 1 - cont["gemm"] / alone["gemm"],
                   "l2Slowdown": 1 - cont["l2"] / alone["l2"]}
            res["rounds"].append(row)
            print(json.dumps(row), flush=True)
    summ = {}
    for name in layouts:
        rows = [x for x in res["rounds"] if x["layout"] == name]
        summ[name] = {k: statistics.median(x[k] for x in rows) for k in ("gemmSlowdown", "l2Slowdown")}
        summ[name].update({
            "gemmAloneTflops": statistics.median(x["alone"]["gemm"] for x in rows),
            "gemmContendedTflops": statistics.median(x["contended"]["gemm"] for x in rows),
            "l2AloneGBps": statistics.median(x["alone"]["l2"] for x in rows),
            "l2ContendedGBps": statistics.median(x["contended"]["l2"] for x in rows),
            "aggressorGBps": statistics.median(x["contended"]["aggressorGBps"] for x in rows)})
    res["summary"] = summ
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(summ, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
