"""The bench's independent ground truth (gpupool/bench/ground_truth.py) against the operator.

* property: ``device_healthy`` (Python, restated from the CRD's spec.health semantics) agrees with
  the operator's native evaluator (libmi355x_dev ``evaluate``) on random device states, baselines
  and policies — two implementations of one documented rule;
* integration: ``accuracy_under_faults`` on the 8-GPU fake node is exact, and a truth that applies
  a different rule than the pool (belowEmergency vs the pool's belowCritical) is caught.
"""
from __future__ import annotations

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gpupool.bench import ground_truth as gt

LINK = st.sampled_from(["U", "U", "U", "D", "X"])


@st.composite
def device_case(draw):
    links = draw(st.one_of(st.none(), st.lists(LINK, min_size=8, max_size=8)))
    unc0, cor0 = draw(st.integers(0, 5)), draw(st.integers(0, 50))
    dev = {"present": draw(st.sampled_from([True, True, True, False])),
           "ecc": {"uncorrectable": unc0 + draw(st.integers(-1, 3)),
                   "correctable": cor0 + draw(st.integers(-5, 30))},
           "temps": {}, "partition": {"compute": draw(st.sampled_from(["SPX", "CPX"])),
                                      "memory": "NPS1"}}
    if links is not None:
        dev["xgmi"] = {"links": links}
    for s, crit, emer in (("hotspot", 100, 112), ("vram", 115, 125), ("edge", 90, 105)):
        if draw(st.booleans()):
            dev["temps"][s] = {"current": draw(st.integers(crit - 15, emer + 3)),
                               "critical": crit, "emergency": emer}
    if draw(st.booleans()):
        dev["ras"] = {"badPagesSupported": draw(st.booleans()),
                      "retiredPages": draw(st.integers(0, 10)),
                      "pendingPages": draw(st.integers(0, 2)),
                      "unreservablePages": draw(st.sampled_from([0, 0, 0, 1]))}
    base = {"ecc": {"uncorrectable": unc0, "correctable": cor0}}
    health = {}
    if draw(st.booleans()):
        health = {"maxUncorrectableECC": draw(st.integers(0, 2)),
                  "maxCorrectableECC": draw(st.integers(0, 20)),
                  "requireAllXGMILinks": draw(st.booleans()),
                  "minXGMILinksUp": draw(st.integers(0, 8)),
                  "thermal": draw(st.sampled_from(["belowCritical", "belowEmergency", "ignore"])),
                  "thermalMarginC": draw(st.integers(0, 10)),
                  "maxRetiredPages": draw(st.integers(0, 8)),
                  "maxPendingPages": draw(st.integers(0, 1))}
    policy = {"health": health,
              "partition": {"compute": draw(st.sampled_from(["Any", "SPX", "CPX"]))}}
    return dev, base, policy


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(device_case())
def test_truth_predicate_matches_the_operator_rule(native_built, case):
    from gpupool.ops import devlib
    dev, base, policy = case
    ours, why = gt.device_healthy(dev, base, policy)
    op = devlib.evaluate_batch([(dev, base, policy)])[0]
    assert ours == bool(op["healthy"]), (why, op.get("reasons"), dev, base, policy)


def test_cli_parsing_of_the_captured_mi355x(monkeypatch):
    """cli_state() over the amd-smi JSON captured on the real MI355X box (tests/fixtures/
    real_mi355x): limits mapped to critical = slowdown, emergency = shutdown; a healthy idle GPU."""
    import json
    import os
    d = os.path.join(os.path.dirname(os.path.dirname(__file__)), "fixtures", "real_mi355x")
    files = {"list": "amdsmi_list.json", "metric": "amdsmi_metric.json",
             "static": "amdsmi_static.json", "xgmi": "amdsmi_xgmi.json",
             "partition": "amdsmi_partition.json"}

    def fake(*cmd):
        if cmd[0] not in files:
            raise RuntimeError("unsupported")
        with open(os.path.join(d, files[cmd[0]])) as f:
            return json.load(f)
    monkeypatch.setattr(gt, "_amdsmi", fake)
    state = gt.cli_state()
    assert state
    dev = next(iter(state.values()))
    assert dev["temps"]["hotspot"]["critical"] == 100 and dev["temps"]["hotspot"]["emergency"] == 112
    assert dev["temps"]["vram"]["critical"] == 115
    assert gt.healthy_from_cli(state, state) == set(state)
    # an injected hotspot at the slowdown limit is a fault; one degree under is not
    u = next(iter(state))
    hot = {"devices": {u: {"temps": {"hotspot": {"current": 100}}}}}
    assert u not in gt.healthy_from_cli(state, state, overlay=hot)
    warm = {"devices": {u: {"temps": {"hotspot": {"current": 99}}}}}
    assert u in gt.healthy_from_cli(state, state, overlay=warm)


@pytest.mark.slow
def test_accuracy_under_faults_and_a_wrong_rule_is_caught(cluster_factory):
    from gpupool.bench.runner import BenchRun
    from gpupool.testing.cluster import NodeSpec
    node = NodeSpec("gt-node", extra_args=["--probe-sim-ms", "1"])
    c = cluster_factory(nodes=[node], sample_interval=0.5)
    run = BenchRun(c, node, real=False, timeout=60)
    good = run.accuracy_under_faults(8, 24, seed=1)
    assert good["accuracy"] == 1.0 and good["samples"] == 24, good["mismatches"]
    assert good["ownership_stable"]
    # a truth that judges thermals against the shutdown limit, while the pool uses the slowdown
    # limit, must disagree on some hotspot fault of the same sequence
    bad = run.accuracy_under_faults(8, 24, seed=1, truth_policy={
        "health": {"maxCorrectableECC": 10, "maxRetiredPages": 4, "thermal": "belowEmergency"}},
        settle_s=0.5)
    assert bad["accuracy"] < 1.0, bad
