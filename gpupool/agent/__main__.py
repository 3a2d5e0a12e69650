"""``python -m gpupool.agent --node mi355x-node-0 --backend amdsmi --socket /run/gpupool/agent.sock
--apiserver http://127.0.0.1:6443 --plugin-dir /var/lib/kubelet/device-plugins``"""
from __future__ import annotations

import argparse
import logging
import os
import socket
import sys



def _count_seconds(v: str) -> tuple[int, float]:
    if not v:
        return (0, 0.0)
    c, _, sec = v.partition(":")
    return (int(c), float(sec or 0))


def main() -> None:
    from ..utils import parent_watch
    parent_watch.start()  # test harness only: exit when the test runner is gone
    # Before anything touches a GPU (amdsmi in the device library, HIP anywhere): the forkserver the
    # probe helpers are forked from, so no helper inherits GPU state (probehost.py).
    from .probehost import start_spawner
    start_spawner()
    ap = argparse.ArgumentParser(description="gpupool node agent (MI355X)")
    ap.add_argument("--node", default=os.environ.get("GPUPOOL_NODE", socket.gethostname()))
    ap.add_argument("--backend", default=os.environ.get("GPUPOOL_BACKEND", "auto"),
                    choices=["auto", "amdsmi", "cli", "fake"])
    ap.add_argument("--fixture", default="", help="fake backend node snapshot JSON")
    ap.add_argument("--faults", default=os.environ.get("GPUPOOL_FAULTS", ""),
                    help="fault overlay JSON (hot-reloaded)")
    ap.add_argument("--count", type=int, default=-1, help="fake backend: limit #devices")
    ap.add_argument("--cli-dir", default="", help="cli backend: read captured amd-smi JSON")
    ap.add_argument("--state-dir", default=os.environ.get("GPUPOOL_STATE_DIR", "/var/lib/gpupool"))
    ap.add_argument("--socket", default="", help="unix socket for the manager RPC")
    ap.add_argument("--listen", default="", help="host:port for the manager RPC (TCP)")
    ap.add_argument("--endpoint", default="", help="endpoint written to the Node annotation")
    ap.add_argument("--tls-cert", default=os.environ.get("GPUPOOL_AGENT_TLS_CERT", ""),
                    help="PEM certificate: serve --listen over HTTPS (the manager verifies it "
                         "with --agent-ca-file)")
    ap.add_argument("--tls-key", default=os.environ.get("GPUPOOL_AGENT_TLS_KEY", ""))
    ap.add_argument("--apiserver", default=os.environ.get("GPUPOOL_APISERVER", ""))
    ap.add_argument("--token", default=os.environ.get("GPUPOOL_TOKEN", ""))
    ap.add_argument("--token-file", default=os.environ.get("GPUPOOL_TOKEN_FILE", ""),
                    help="apiserver bearer token file, re-read as it rotates (projected "
                         "ServiceAccount token); in-cluster config does this by itself")
    ap.add_argument("--heartbeat-interval", type=float, default=10.0,
                    help="period of the agent's Node condition heartbeat (s)")
    ap.add_argument("--auth-token-file", default=os.environ.get("GPUPOOL_AGENT_TOKEN_FILE", ""),
                    help="shared secret accepted on the RPC (Authorization: Bearer), re-read "
                         "when the file changes; $GPUPOOL_AGENT_TOKEN also works")
    ap.add_argument("--auth-grace", type=float, default=300.0,
                    help="seconds a rotated-out --auth-token-file token stays valid")
    ap.add_argument("--manager-pubkeys", default=os.environ.get("GPUPOOL_MANAGER_PUBKEYS", ""),
                    help="PEM bundle or directory of the manager's Ed25519 public keys: requests "
                         "must carry its signature for this node (X-Gpupool-Signature)")
    ap.add_argument("--plugin-dir", default="", help="kubelet device-plugin directory")
    ap.add_argument("--pod-resources", default="", help="kubelet PodResources socket")
    ap.add_argument("--probe", default="",
                    choices=["", "helper", "helper-sim", "inproc", "subprocess", "simulated", "off"],
                    help="where the claim-time probe runs: helper (default with GPUs: per-GPU "
                         "child processes, isolated, with a deadline), helper-sim (the same with "
                         "simulated kernels), inproc (in the agent; A/B only), subprocess, "
                         "simulated (default with the fake backend), off")
    ap.add_argument("--probe-sim-ms", type=float, default=20.0)
    ap.add_argument("--probe-gemm-n", type=int, default=4096,
                    help="GEMM size of the serial probe (pools with performance floors)")
    ap.add_argument("--probe-overlap-gemm-n", type=int, default=2048,
                    help="GEMM size of the claim-time probe, which overlaps the HBM pattern test")
    ap.add_argument("--sample-interval", type=float, default=2.0,
                    help="full telemetry sample period (s): activity, power, VRAM, bad pages, pods")
    ap.add_argument("--health-interval", type=float, default=0.1,
                    help="health-only poll period (s): ECC, xGMI links, temperatures (0 = off)")
    ap.add_argument("--quarantine", type=float, default=300.0)
    ap.add_argument("--no-fsync", action="store_true")
    ap.add_argument("--probe-arena-idle", type=float, default=10.0,
                    help="seconds before the kept probe arena (~1.2 GiB/GPU) is freed")
    ap.add_argument("--probe-fabric-idle", type=float, default=0.0,
                    help="seconds before an idle xGMI fabric helper exits (0 = resident and "
                         "pre-warmed at start, so multi-GPU claims never pay its HIP init)")
    ap.add_argument("--scrub-interval", type=float, default=60.0,
                    help="HBM scrubber pass period over idle GPUs, seconds (0 = off)")
    ap.add_argument("--scrub-window", type=int, default=4 << 30, help="bytes per scrub window")
    ap.add_argument("--scrub-windows", type=int, default=8, help="windows per GPU per pass")
    ap.add_argument("--scrub-reserve", type=int, default=4 << 30,
                    help="HBM bytes the scrub buffer leaves free")
    ap.add_argument("--scrub-start-delay", type=float, default=30.0)
    ap.add_argument("--gil-switch-interval", type=float,
                    default=float(os.environ.get("GPUPOOL_GIL_SWITCH_INTERVAL", "0.00005")),
                    help="sys.setswitchinterval for the agent (s): how long a thread that wants "
                         "the GIL waits for the holder to yield (CPython default 0.005). A claim "
                         "returning from the HIP probe (GIL released) waits this long behind a "
                         "busy thread, e.g. the ledger writer encoding in the probe's shadow: "
                         "0.58 ms at 500 us, 0.08 ms at 50 us (profiles/r3o_probe_call_gil.json)")
    ap.add_argument("--hbm-reserve", type=int, default=2 << 30,
                    help="HBM bytes per GPU the agent keeps for itself (HIP context + probe "
                         "arena): a shared pool whose replicasPerGPU x hbmBytesPerSlot does not "
                         "fit beside it is refused (SharingOvercommitted)")
    ap.add_argument("--share-acct-grace", type=float, default=10.0,
                    help="an isolated slot's HBM account file younger than this (s) is kept even "
                         "if the kubelet does not list its pod yet")
    ap.add_argument("--xgmi-recheck", type=float, default=600.0,
                    help="idle xGMI coverage ring period over pod-free GPUs, seconds (0 = off)")
    ap.add_argument("--inject-claim-delay", default="",
                    help="fault injection (tests/bench): COUNT:SECONDS — a claim of >= COUNT GPUs "
                         "stalls SECONDS before selecting devices (a hung probe / driver call)")
    ap.add_argument("--ready-file", default="")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    from .agent import Agent, AgentConfig, serve
    if a.gil_switch_interval > 0:
        # The agent's threads (RPC loop, claim executor, sampler, device-plugin gRPC) hand the GIL
        # to each other on every claim; at the 5 ms default one hand-off can cost milliseconds.
        sys.setswitchinterval(a.gil_switch_interval)
    logging.basicConfig(level=logging.DEBUG if a.verbose else logging.INFO,
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    auth = "" if a.auth_token_file else os.environ.get("GPUPOOL_AGENT_TOKEN", "")
    cfg = AgentConfig(node=a.node, auth_token=auth, auth_token_file=a.auth_token_file,
                      auth_grace_s=a.auth_grace, manager_pubkeys=a.manager_pubkeys, backend=a.backend, fixture=a.fixture, faults=a.faults,
                      count=a.count, cli_dir=a.cli_dir, state_dir=a.state_dir, socket=a.socket,
                      listen=a.listen, tls_cert=a.tls_cert, tls_key=a.tls_key,
                      endpoint=a.endpoint, apiserver=a.apiserver, token=a.token,
                      token_file=a.token_file, heartbeat_interval=a.heartbeat_interval,
                      plugin_dir=a.plugin_dir, pod_resources=a.pod_resources, probe_mode=a.probe,
                      probe_sim_ms=a.probe_sim_ms, probe_gemm_n=a.probe_gemm_n,
                      probe_overlap_gemm_n=a.probe_overlap_gemm_n,
                      sample_interval=a.sample_interval, health_interval=a.health_interval,
                      quarantine_s=a.quarantine,
                      fsync=not a.no_fsync, probe_arena_idle_s=a.probe_arena_idle,
                      probe_fabric_idle_s=a.probe_fabric_idle,
                      scrub_interval_s=a.scrub_interval, scrub_window_bytes=a.scrub_window,
                      scrub_windows=a.scrub_windows, scrub_reserve_bytes=a.scrub_reserve,
                      scrub_start_delay_s=a.scrub_start_delay,
                      xgmi_recheck_s=a.xgmi_recheck, hbm_reserve_bytes=a.hbm_reserve,
                      share_acct_grace_s=a.share_acct_grace,
                      inject_claim_delay=_count_seconds(a.inject_claim_delay))
    agent = Agent(cfg)
    try:
        serve(agent, a.ready_file or None)
    except KeyboardInterrupt:
        pass
    finally:
        agent.stop()


if __name__ == "__main__":
    main()
