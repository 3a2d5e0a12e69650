"""``python -m gpupool.apiserver_sim --port 0 --port-file /tmp/port --crd-dir config/crd``."""
from __future__ import annotations

import argparse
import asyncio
import logging

from .server import ApiServerSim, serve


def main() -> None:
    from ..utils import parent_watch
    parent_watch.start()  # test harness only: exit when the test runner is gone
    ap = argparse.ArgumentParser(description="gpupool kube-apiserver simulator")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=6443)
    ap.add_argument("--port-file", default=None, help="write the bound port here (for --port 0)")
    ap.add_argument("--crd-dir", default=None, help="pre-install every CRD YAML in this dir")
    ap.add_argument("--token", default=None, help="require 'Authorization: Bearer <token>'")
    ap.add_argument("--users-file", default=None,
                    help="JSON {token: {username, groups, extra, expiresAt}}: more identities "
                         "beside --token (changeable at run time through POST /debug/tokens)")
    ap.add_argument("--bookmark-interval", type=float, default=5.0)
    ap.add_argument("--window", type=int, default=50000, help="watch event-log window")
    ap.add_argument("--unix", default=None, help="also listen on this unix socket")
    ap.add_argument("--tls-cert", default=None, help="serve HTTPS with this PEM certificate chain")
    ap.add_argument("--tls-key", default=None, help="PEM private key for --tls-cert")
    ap.add_argument("--client-ca", default=None, help="require client certs signed by this CA")
    ap.add_argument("--watch-delay", type=float, default=0.0,
                    help="deliver every watch event this many seconds late (stale informers)")
    ap.add_argument("--profile", default=None, help="write cProfile stats here on exit")
    ap.add_argument("--fail-list", action="append", default=[],
                    help="fault injection: LIST/WATCH of this resource plural answer 503 until "
                         "cleared through POST /debug/faults (repeatable)")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    prof = None
    if a.profile:
        import cProfile
        import signal
        prof = cProfile.Profile()
        import os

        def _dump_and_exit(*_):  # open watch streams would keep asyncio.run's shutdown waiting
            prof.disable()
            prof.dump_stats(a.profile)
            os._exit(0)
        signal.signal(signal.SIGTERM, _dump_and_exit)
        prof.enable()
    logging.basicConfig(level=logging.DEBUG if a.verbose else logging.WARNING,
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    sim = ApiServerSim(token=a.token, bookmark_interval=a.bookmark_interval, window=a.window,
                       watch_delay=a.watch_delay)
    sim.fail_list = {r: -1 for r in a.fail_list}
    if a.users_file:
        import json
        with open(a.users_file) as f:
            sim.users = {str(k): dict(v) for k, v in json.load(f).items()}
    try:
        asyncio.run(serve(a.host, a.port, sim, a.port_file, a.crd_dir, a.unix,
                          tls_cert=a.tls_cert, tls_key=a.tls_key, client_ca=a.client_ca))
    except KeyboardInterrupt:
        pass
    finally:
        if prof is not None:
            prof.disable()
            prof.dump_stats(a.profile)


if __name__ == "__main__":
    main()
