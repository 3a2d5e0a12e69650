#!/usr/bin/env python3
"""`make run`: bring up a local control plane (apiserver-sim + gpupool-manager + node agent(s) +
fake kubelet(s)) in the foreground — the analogue of the reference's `make run` against a local
kubeconfig (README.md:259-263) — and point gpuctl at it via a context.

  python scripts/run_local.py [--backend fake|amdsmi] [--nodes 1] [--workdir DIR]
  # then, in another shell:  bin/gpuctl apply -f config/samples/compute_v1alpha1_mi355xpool.yaml
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import tempfile
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gpupool.cli.gpuctl import load_config, save_config  # noqa: E402
from gpupool.testing.cluster import Cluster, NodeSpec  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="fake", choices=["fake", "amdsmi", "cli"])
    ap.add_argument("--nodes", type=int, default=1)
    ap.add_argument("--workdir", default="")
    ap.add_argument("--no-kubelet", action="store_true")
    a = ap.parse_args()
    wd = a.workdir or tempfile.mkdtemp(prefix="gpupool-run-")
    nodes = [NodeSpec(f"mi355x-node-{i}", backend=a.backend, kubelet=not a.no_kubelet,
                      probe="" if a.backend == "fake" else "helper") for i in range(a.nodes)]
    c = Cluster(wd, nodes=nodes)
    c.start()
    cfg = load_config()
    cfg.setdefault("contexts", {})["local"] = {"server": c.url, "namespace": "default"}
    cfg["current-context"] = "local"
    save_config(cfg)
    print(f"control plane up: apiserver {c.url}, manager metrics :{c.metrics_port}, logs {wd}")
    print("gpuctl context 'local' selected; try:")
    print("  bin/gpuctl apply -f config/samples/compute_v1alpha1_mi355xpool.yaml")
    print("  bin/gpuctl get mi355xpools && bin/gpuctl describe mi355xpool mi355x-pool")
    stop = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    stop.wait()
    c.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
