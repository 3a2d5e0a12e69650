"""One launcher for every GPU-box measurement: ``python scripts/gpu_run.py <scenario>... --tag T``.

Replaces the per-pass ``gpu_r4*.sh`` launchers. A scenario is a list of steps; each step runs under
its own ``timeout -k 10`` and the run stops at the first failing step (no GPU step after a fault,
an abort or a time limit). Outputs go to ``gpurun_out/<tag>/<step>.*``; copy the summaries worth
keeping into ``profiles/``.

    /usr/local/graft/bin/gpurun --timeout 1200 -- python scripts/gpu_run.py tier bench --tag r5d

``--dry-run`` (CPU, no GPU touched): prints every step and checks that what it runs exists in this
tree — each script present and compiling, each argparse script answering ``--help`` — which is
how tests/unit/test_gpu_run.py keeps every scenario runnable against the current code.
"""
from __future__ import annotations

import argparse
import json
import os
import py_compile
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable


def _bench(*extra: str) -> list[str]:
    return [PY, "-u", "bench.py", *extra]


def _prof(tag_dir: str, name: str, *cmd: str, pmc: tuple[str, ...] = ()) -> list[str]:
    """rocprofv3 with the program itself after ``--`` (never a shell or env hop). Counter passes
    (``pmc``) carry kernel-trace only beside them; timing passes kernel-trace + stats."""
    base = ["rocprofv3"]
    if pmc:
        base += ["--pmc", *pmc, "--kernel-trace"]
    else:
        base += ["--kernel-trace", "--stats"]
    return base + ["--output-format", "csv", "-d", os.path.join(tag_dir, name), "-o", name, "--",
                   *cmd]


GEMM_SQ_PASSES = (("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                   "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
                   "SQ_WAIT_INST_LDS", "GRBM_GUI_ACTIVE"),)


# scenario -> steps: (name, argv or callable(tag_dir) -> argv, timeout s, env overrides)
def scenarios(tag_dir: str) -> dict[str, list[tuple]]:
    pytest = [PY, "-u", "-m", "pytest", "-x", "-v", "--timeout", "200", "--timeout-method",
              "thread", "-p", "no:cacheprovider"]
    return {
        # driver facts for preflight (host amdgpu vs the image's ROCm userspace)
        "facts": [("facts", [PY, "scripts/gpu_run.py", "--facts"], 60, {})],
        # the GPU tier and the driver's smoke
        "tier": [("pytest_gpu", pytest + ["-m", "gpu", "tests"], 900, {}),
                 ("smoke", [PY, "-c", "import __graft_entry__ as g; g.smoke()"], 300, {})],
        "sharing": [("pytest_sharing", pytest + ["tests/gpu/test_sharing_gpu.py"], 400, {}),
                    ("slot_interference", [PY, "scripts/slot_interference_ab.py"], 300, {}),
                    ("cu_mask_layouts", [PY, "scripts/cu_mask_layouts.py"], 200, {})],
        # the headline (BASELINE config 2) as the driver runs it
        "bench": [("bench", _bench("--steps", "20", "--warmup", "3"), 300, {})],
        "soak": [("bench_soak300", _bench("--steps", "300", "--warmup", "3"), 900, {})],
        "soak600": [("bench_soak600", _bench("--steps", "600", "--warmup", "3", "--budget-s",
                                             "1100"), 1150, {})],
        # the probe helper's cost: interleaved helper / in-process runs, and the call itself
        "bench-ab": [(f"bench_{m}_{i}", _bench("--steps", "40", "--warmup", "3", "--probe-mode", m),
                      240, {}) for i in (1, 2) for m in ("helper", "inproc")],
        "helper-ab": [("helper_ab", [PY, "scripts/helper_overhead_ab.py"], 300, {})],
        # kernel timing over the headline bench. The probe runs in-process here: a helper forked
        # from the agent's forkserver under rocprofv3's preloaded tool never came up (r5d: the
        # bench sat silent until the box's 180 s hang guard), and the kernels are the same ones
        # (helper vs inproc bench A/B: profiles/r5c_bench_helper_vs_inproc_ab.json)
        "prof": [("bench_prof", _prof(tag_dir, "bench_prof", PY, os.path.join(ROOT, "bench.py"),
                                      "--gpus", "1", "--steps", "10", "--warmup", "2",
                                      "--health-steps", "0", "--probe-mode", "inproc"), 400, {})],
        # counters of the probe GEMM (one pass: 4 TCC counters at most per run)
        "pmc": [(f"gemm_l2_g{g}", _prof(tag_dir, f"gemm_l2_g{g}", PY,
                                          os.path.join(ROOT, "scripts", "gemm_l2_pmc.py"), "8192",
                                          str(g), pmc=("TCC_HIT_sum", "TCC_MISS_sum")), 120, {})
                for g in (0, 4)],
        # SQ counters of the GEMM K-loops (2-phase, half-tile pipeline, staggered), 8 SQ per pass
        "gemm-sq": [(f"gemm_sq{i}_p{p}", _prof(tag_dir, f"gemm_sq{i}_p{p}", PY,
                                              os.path.join(ROOT, "scripts", "gemm_l2_pmc.py"),
                                              "4096", "4", str(p), pmc=c), 120, {})
                    for i, c in enumerate(GEMM_SQ_PASSES) for p in (0, 1, 2)],
        # HBM bytes per probe kernel as the memory system counts them (one TCC group per pass)
        "probe-pmc": [(f"probe_{c.lower()}", _prof(tag_dir, f"probe_{c.lower()}", PY,
                                                  os.path.join(ROOT, "scripts", "probe_hbm_pmc.py"),
                                                  "5", pmc=(c,)), 120, {})
                      for c in ("FETCH_SIZE", "WRITE_SIZE")],
        "gemm": [("gemm_vs_hipblaslt", [PY, "scripts/gemm_vs_hipblaslt.py"], 300, {})],
        "gemm-ab": [("gemm_kloop_ab", [PY, "scripts/gemm_kloop_ab.py"], 300, {})],
        "hbm-cache": [("hbm_cache_residency", [PY, "scripts/hbm_cache_residency.py"], 300, {})],
        "claim-gemm-ab": [("claim_probe_gemm_ab", [PY, "scripts/claim_probe_gemm_ab.py"], 300, {})],
        # the probe's two-stream shape as one hipGraph vs eager launches (r5l: not adopted)
        "graph": [("graph_events", [os.path.join(ROOT, "build", "native", "graph_events"), "1024",
                                    "15"], 120, {})],
        "probe": [("probe_report", [PY, "scripts/probe_report.py"], 200, {}),
                  ("probe_size_sweep", [PY, "scripts/probe_size_sweep.py"], 300, {})],
        "footprint": [("helper_footprint", [PY, "scripts/helper_footprint.py", "8"], 240, {}),
                      ("hip_host_memory", [PY, "scripts/hip_host_memory.py"], 240, {}),
                      ("agent_footprint", [PY, "scripts/agent_footprint.py"], 300, {}),
                      ("amdsmi_call_costs", [PY, "scripts/amdsmi_call_costs.py"], 200, {}),
                      ("helper_init_breakdown", [PY, "scripts/helper_init_breakdown.py"], 400, {})],
    }


def facts() -> dict:
    """What the preflight reads, from this box: host amdgpu driver and the image's ROCm."""
    out: dict = {}
    for k, p in (("amdgpuVersion", "/sys/module/amdgpu/version"),
                 ("amdgpuSrcversion", "/sys/module/amdgpu/srcversion"),
                 ("kernelRelease", "/proc/sys/kernel/osrelease"),
                 ("rocmVersion", "/opt/rocm/.info/version")):
        try:
            with open(p) as f:
                out[k] = f.read().strip()
        except OSError as e:
            out[k] = None
            out[k + "Error"] = e.strerror
    out["amdgpuLoaded"] = os.path.isdir("/sys/module/amdgpu")
    try:
        sys.path.insert(0, ROOT)
        from gpupool.agent import preflight
        out["preflight"] = preflight.check({"devices": [{"asic": {"gfx": "gfx950"}}]})
    except Exception as e:  # report, never fail the fact collection
        out["preflightError"] = repr(e)
    return out


def dry_check(argv: list[str]) -> str:
    """'' if the step's program is present and runnable here (without a GPU), else why not."""
    if argv and argv[0].startswith(ROOT) and not os.access(argv[0], os.X_OK):
        return f"{os.path.relpath(argv[0], ROOT)} missing (make -C native)"
    scripts = [a for a in argv if a.endswith(".py")]
    for s in scripts:
        path = s if os.path.isabs(s) else os.path.join(ROOT, s)
        if not os.path.exists(path):
            return f"{s} missing"
        try:
            py_compile.compile(path, doraise=True)
        except py_compile.PyCompileError as e:
            return f"{s} does not compile: {e}"
        if os.path.basename(path) in ("bench.py", "gpu_run.py") or "argparse" in open(path).read():
            r = subprocess.run([PY, path, "--help"], capture_output=True, text=True, timeout=120,
                               cwd=ROOT, env={**os.environ, "PYTHONPATH": ROOT})
            if r.returncode != 0:
                return f"{s} --help exited {r.returncode}: {r.stderr[-300:]}"
    if "-m" in argv and "pytest" in argv:
        tgt = argv[-1]
        if not os.path.exists(os.path.join(ROOT, tgt)):
            return f"pytest target {tgt} missing"
    return ""


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("scenario", nargs="*", help="scenario names ('all' with --dry-run)")
    ap.add_argument("--tag", default="run", help="output directory under gpurun_out/")
    ap.add_argument("--dry-run", action="store_true", help="print and check the steps; run nothing")
    ap.add_argument("--facts", action="store_true", help="print the driver facts as JSON")
    ap.add_argument("--list", action="store_true")
    a = ap.parse_args()
    if a.facts:
        print(json.dumps(facts(), indent=1))
        return 0
    tag_dir = os.path.join(ROOT, "gpurun_out", a.tag)
    table = scenarios(tag_dir)
    if a.list or not a.scenario:
        for k, steps in table.items():
            print(f"{k:10s} " + ", ".join(s[0] for s in steps))
        return 0
    names = list(table) if a.scenario == ["all"] else a.scenario
    unknown = [n for n in names if n not in table]
    if unknown:
        print(f"unknown scenario(s) {unknown}; known: {sorted(table)}", file=sys.stderr)
        return 2
    if a.dry_run:
        bad = 0
        for n in names:
            for step, argv, timeout, env in table[n]:
                why = dry_check(argv)
                bad += bool(why)
                print(f"[{n}] {step}: timeout {timeout}s {' '.join(argv)}"
                      + (f"  !! {why}" if why else "  ok"))
        return 1 if bad else 0
    os.makedirs(tag_dir, exist_ok=True)
    env0 = {**os.environ, "PYTHONPATH": ROOT, "TMPDIR": os.environ.get("TMPDIR", "/tmp")}
    for n in names:
        for step, argv, timeout, env in table[n]:
            out = os.path.join(tag_dir, step + (".json" if "bench" in step or step in ("facts",
                               "helper_ab", "helper_footprint", "hip_host_memory") else ".txt"))
            cmd = ["timeout", "-k", "10", str(timeout), *argv]
            print(f"[{n}] {step}: {' '.join(argv)} > {out}", flush=True)
            with open(out, "w") as fo, open(os.path.join(tag_dir, step + ".err"), "w") as fe:
                r = subprocess.run(cmd, cwd=ROOT, env={**env0, **env}, stdout=fo, stderr=fe)
            print(f"[{n}] {step}: exit {r.returncode}", flush=True)
            if r.returncode != 0:  # a fault, an abort or a time limit: no further GPU step
                return r.returncode
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
