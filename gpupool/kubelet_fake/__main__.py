"""``python -m gpupool.kubelet_fake --node n0 --apiserver URL --root /tmp/kubelet``"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import threading

from .kubelet import FakeKubelet


def main() -> None:
    from ..utils import parent_watch
    parent_watch.start()  # test harness only: exit when the test runner is gone
    ap = argparse.ArgumentParser(description="fake kubelet (device plugins + pod runtime)")
    ap.add_argument("--node", required=True)
    ap.add_argument("--apiserver", required=True)
    ap.add_argument("--token", default=os.environ.get("GPUPOOL_TOKEN") or None)
    ap.add_argument("--root", required=True, help="kubelet root dir (device-plugins/, pod-resources/)")
    ap.add_argument("--workdir", default=os.getcwd(), help="cwd for pod processes")
    ap.add_argument("--no-schedule", action="store_true")
    ap.add_argument("--node-status-delay", type=float, default=0.02,
                    help="coalescing delay between a device-plugin update and the Node status PATCH (s)")
    ap.add_argument("--status-interval", type=float, default=10.0,
                    help="periodic node-status sync (Ready heartbeat, capacity/allocatable), s")
    ap.add_argument("--host-path", action="append", default=None,
                    help="strict mounts: a host path a device plugin may hand out (repeatable; "
                         "an Allocate mount or device outside all of them fails the pod)")
    ap.add_argument("--ready-file", default="")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    # same GIL hand-off setting as the agent (ListAndWatch consumer, runtime and API threads)
    sw = float(os.environ.get("GPUPOOL_GIL_SWITCH_INTERVAL", "0.0005"))
    if sw > 0:
        sys.setswitchinterval(sw)
    logging.basicConfig(level=logging.DEBUG if a.verbose else logging.INFO,
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    k = FakeKubelet(a.node, a.apiserver, os.path.join(a.root, "device-plugins"),
                    os.path.join(a.root, "pod-resources", "kubelet.sock"), workdir=a.workdir,
                    log_dir=os.path.join(a.root, "pod-logs"), token=a.token,
                    schedule=not a.no_schedule, node_status_delay=a.node_status_delay,
                    host_paths=a.host_path, status_interval=a.status_interval)
    k.start()
    if a.ready_file:
        with open(a.ready_file, "w") as f:
            f.write("ok")
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    k.stop()


if __name__ == "__main__":
    main()
