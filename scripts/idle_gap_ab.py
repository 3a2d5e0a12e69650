"""A/B of the 0->1 reconcile-to-Ready latency after different idle gaps on the real node:
back-to-back cycles, a 1 s sleep before each cycle, and an amd-smi CLI read before each cycle
(what bench.py's per-step ground-truth read does). Prints p50 + the claim-pass spans per mode."""
import json
import statistics
import sys
import tempfile
import time

sys.path.insert(0, ".")
from gpupool.bench import ground_truth as gt  # noqa: E402
from gpupool.bench.runner import BenchRun  # noqa: E402
from gpupool.testing.cluster import Cluster, NodeSpec  # noqa: E402

real = "--fake" not in sys.argv
reps = 12
node = NodeSpec("mi355x-node-0", backend="amdsmi" if real else "fake",
                probe="inproc" if real else "simulated", count=-1 if real else 8)
cl = Cluster(tempfile.mkdtemp(prefix="gap-"), nodes=[node], sample_interval=1.0)
cl.start()
out = {}
try:
    run = BenchRun(cl, node, real)
    pool = run.make_pool("p", "amd.com/gpu", 0)
    run.scale("p", 0)
    run.refresh_health()
    modes = {"none": lambda: None, "sleep1s": lambda: time.sleep(1.0),
             "amdsmi_cli": (lambda: gt.cli_state()) if real else (lambda: time.sleep(0.9))}
    for rnd in range(2):
        for m, gap in modes.items():
            for _ in range(reps // 2):
                gap()
                out.setdefault(m, []).append(run.cycle(pool, 1)["readySeconds"] * 1e3)
    res = {m: {"p50_ms": round(statistics.median(v), 3), "min_ms": round(min(v), 3),
               "max_ms": round(max(v), 3), "n": len(v)} for m, v in out.items()}
    tr = sorted(cl.manager_traces(key="Mi355xPool/default/p", n=512), key=lambda t: t["start"])
    claims = [t for t in tr if any(s["name"] == "agent:POST /v1/claims" for s in t["spans"])]
    res["claim_spans_last"] = [[(s["name"], round(s["ms"], 3)) for s in t["spans"]] for t in claims[-6:]]
    print(json.dumps(res, indent=1))
finally:
    cl.stop()
