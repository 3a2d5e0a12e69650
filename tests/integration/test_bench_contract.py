"""bench.py output contract on the CPU (fake 8x MI355X backend): the driver's JSON line, the
replicas sweep (per_n 1/2/4/8), config 4 scale-down, config 5 two pools and the health latencies."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pytestmark = pytest.mark.slow


def run_bench(*args: str, timeout: float = 600) -> dict:
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--backend", "fake", *args],
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_gpus8_sweep_scale_down_two_pools(native_built):
    out = run_bench("--gpus", "8", "--steps", "1", "--warmup", "0", "--scale-down-steps", "1",
                    "--pool-steps", "1", "--health-steps", "1", "--fault-steps", "20")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert out["n_gpus"] == 8 and out["higher_is_better"] is False and out["unit"] == "s"
    assert "apiserver-sim" in out["data"] and "fake" in out["data"]
    cfg = out["config"]
    assert sorted(cfg["per_n"], key=int) == ["1", "2", "4", "8"]
    for k, v in cfg["per_n"].items():
        if v["accuracy"] != 1.0:  # keep the whole record for the diagnosis
            with open(os.path.join(tempfile.gettempdir(), "bench_contract_mismatch.json"), "w") as f:
                json.dump(out, f, indent=1)
        assert v["accuracy"] == 1.0 and 0 < v["p50_s"] < 30, (k, json.dumps(v))
        # the truth is read once, at Ready, with no grace: readiness is strict by default
        assert v["truth_first_read_agrees"] == 1.0, (k, v)
    assert out["value"] == cfg["per_n"]["8"]["p50_s"]
    # the xGMI fabric helper warmed every directed pair of the 8 GPUs before any claim
    fw = cfg["per_n"]["8"]["agent"]["fabric_warm"]
    assert fw["links"] == 8 * 7 and fw["passed"], fw
    # device-level evidence per N: every claim's probe, and the xGMI ring of every multi-GPU
    # claim (N links per claim of N GPUs), with the pair coverage the rotating order reached
    for k, v in cfg["per_n"].items():
        assert v["probe_ms_p50"] > 0, (k, v)
        if int(k) >= 2:
            assert v["xgmi_links_measured"] == int(k) * v["n"], (k, v)
            assert v["xgmi_link_GBps_min"] > 0 and v["xgmi_pairs_total"] == 7, (k, v)
            assert len(v["xgmi_pairs_covered_last"]) == int(k)
        else:
            assert "xgmi_links_measured" not in v
        # what the agent costs at this N: its RSS, the HIP contexts it holds (0: simulated probe
        # on the fake backend), VRAM in use on each GPU the N-GPU claim got
        ag = v["agent"]
        assert ag["rss_mib"] > 0 and ag["hip_devices"] == 0, (k, ag)
        assert len(ag["vram_used_mib_per_gpu"]) == int(k), (k, ag)
        assert all(x is not None and x > 0 for x in ag["vram_used_mib_per_gpu"]), (k, ag)
    # the N=8 point carries the fabric evidence the first real 8-GPU run must produce: 8 links
    # measured by the claim's xGMI ring, pair coverage over the node's 7 peers per GPU
    n8 = cfg["per_n"]["8"]
    assert n8["xgmi_links_measured"] == 8 and n8["xgmi_pairs_total"] == 7
    assert len(n8["xgmi_pairs_covered_last"]) == 8 and all(1 <= p <= 7 for p in n8["xgmi_pairs_covered_last"])
    assert cfg["readyReplicas_accuracy"] == 1.0
    assert cfg["truth_first_read_agrees"] == 1.0
    assert cfg["readiness_mode"].startswith("strict")
    # the probe helpers beside the agent (helper-sim on the fake backend)
    assert cfg["per_n"]["1"]["agent"]["probe_helpers"] >= 1
    # agent + manager footprint around the timed region (Prometheus process_* metrics)
    for when in ("before_timed", "after_timed"):
        for who in ("agent", "manager"):
            fp = cfg["footprint"][when][who]
            assert fp["rss_mib"] > 0 and fp["threads"] > 0 and fp["open_fds"] > 0, (when, who, fp)
    # ground-truth time is reported apart from the operator's own time
    assert cfg["operator_ms_per_step"] + cfg["ground_truth_ms_per_step"] == \
        pytest.approx(out["ms_per_step"], abs=0.05)
    sd = cfg["scale_down"]
    assert sd["from"] == 8 and sd["to"] == 4 and sd["accuracy"] == 1.0
    assert sd["evicted_per_step"] == [4] and sd["pods_left_on_released_gpus"] == 0
    tp = cfg["two_pools"]
    assert tp["pools"] == [4, 4] and tp["accuracy"] == 1.0 and tp["cross_pool_devices"] == 0
    h = cfg["health_condition_latency"]
    for k in ("fault_to_condition_p50_s", "forced_sample_to_condition_p50_s",
              "fault_cleared_to_ready_p50_s"):
        assert h[k] is not None and h[k] < 30
    assert h["readyReplicas_accuracy"] == 1.0 and h["accuracy_samples"] == 6
    # readyReplicas against the independent truth after every random fault / clear step
    af = cfg["accuracy_under_faults"]
    assert af["samples"] == 20 and af["accuracy"] == 1.0, af["mismatches"]
    # per-N claim-pass breakdown, and the secondary scenarios' own pass traces
    assert sorted(cfg["claim_pass_span_p50_ms_per_n"], key=int) == ["1", "2", "4", "8"]
    assert cfg["claim_pass_span_p50_ms"] == cfg["claim_pass_span_p50_ms_per_n"]["8"]
    assert "agent:POST /v1/claims" in cfg["claim_pass_span_p50_ms"]
    assert cfg["scale_down"]["pass_span_p50_ms"]["passes"] >= 1
    assert "agent:POST /v1/release" in cfg["scale_down"]["pass_span_p50_ms"]
    # a replicas-only edit pushes no policy to the agent (only a changed policy is re-sent)
    assert "agent:POST /v1/policy" not in cfg["scale_down"]["pass_span_p50_ms"]
    assert out["status"] == "ok" and out["value_n"] == 8


def test_bench_isolates_a_hung_n8_and_keeps_the_curve(native_built):
    """A claim of 8 GPUs that hangs past the per-transition timeout costs only the N=8 point:
    per_n 1/2/4 are measured, N=8 carries the error and its phase, ``value`` falls back to the
    largest N that completed (and says so), the pool is recovered and the secondary scenarios
    still run (scale-down, which needs 8 GPUs, records its own error)."""
    out = run_bench("--gpus", "8", "--steps", "2", "--warmup", "0", "--timeout", "4",
                    "--inject-claim-hang", "8:12", "--scale-down-steps", "1", "--pool-steps", "1",
                    "--health-steps", "0", "--fault-steps", "0", "--azure-steps", "1",
                    timeout=400)
    cfg = out["config"]
    for k in ("1", "2", "4"):
        assert cfg["per_n"][k]["n"] == 2 and cfg["per_n"][k]["accuracy"] == 1.0, cfg["per_n"][k]
    n8 = cfg["per_n"]["8"]
    assert n8["n"] == 0 and n8["p50_s"] is None
    assert "TimeoutError" in n8["error"] and n8["phase"] == "timed:scale_up", n8
    assert out["status"] == "partial" and out["value_n"] == 4
    assert out["value"] == cfg["per_n"]["4"]["p50_s"] and "largest N" in cfg["value_note"]
    assert "phase" in cfg["scale_down"]["error"]
    assert cfg["two_pools"]["accuracy"] == 1.0 and cfg["azure_config1"]["accuracy"] == 1.0


def test_bench_wall_budget_always_prints_json(native_built):
    out = run_bench("--gpus", "2", "--steps", "50", "--warmup", "0", "--budget-s", "1",
                    "--scale-down-steps", "1", "--pool-steps", "1", "--health-steps", "1")
    cfg = out["config"]
    assert out["value"] is None and out["status"] == "failed"
    assert "wall budget" in cfg["budget"]["skipped"]["timed_steps"]
    assert all("skipped" in v for v in cfg["per_n"].values())
    assert "wall budget" in cfg["scale_down"]["skipped_steps"]


def test_bench_gpus1_contract(native_built):
    out = run_bench("--gpus", "1", "--steps", "2", "--warmup", "0", "--scale-down-steps", "1",
                    "--pool-steps", "1", "--health-steps", "0")
    cfg = out["config"]
    assert list(cfg["per_n"]) == ["1"] and out["value"] == cfg["per_n"]["1"]["p50_s"]
    assert cfg["scale_down"]["from"] == 1 and cfg["scale_down"]["to"] == 0
    assert cfg["scale_down"]["accuracy"] == 1.0
    assert "skipped" in cfg["two_pools"]
    az = cfg["azure_config1"]  # BASELINE config 1 on the same manager
    assert az["replicas"] == 0 and az["accuracy"] == 1.0 and az["p50_s"] < 30


def test_bench_under_torchrun_two_ranks_with_comm_check(native_built):
    """The driver's N>1 launch shape (torch.distributed.run, one rank per GPU, 127.0.0.1): rank 0
    drives the control plane, exactly one JSON line is printed, and the post-run collective check
    (here gloo on CPU; RCCL on real GPUs) reports every rank exact."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr=127.0.0.1", f"--master-port={port}",
                        os.path.join(ROOT, "bench.py"), "--backend", "fake", "--gpus", "2",
                        "--steps", "1", "--warmup", "0", "--scale-down-steps", "0",
                        "--pool-steps", "0", "--health-steps", "0", "--comm-check", "gloo"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["world_size"] == 2
    comm = out["config"]["rccl_allreduce"]
    assert comm["world"] == 2 and comm["ranks_ok"] == 2 and comm["exact"], comm
    assert comm["min_busbw_GBps"] > 0
