"""The agent's RPC surface: the routes the manager (and admins' gpuctl) call, and ``serve``,
which starts the listeners and the agent's background loops."""
from __future__ import annotations

import json
import os
import time
from typing import TYPE_CHECKING

if TYPE_CHECKING:
    from .agent import Agent


def build_routes(agent: Agent) -> dict:
    """The manager-facing RPC surface (served by ``rpc.RpcServer``, one thread per connection;
    every route but /healthz and /metrics requires the shared bearer token)."""
    from .rpc import json_reply, text_reply

    def body_json(body: bytes) -> dict:
        return json.loads(body or b"{}")

    def node(q, body):
        return json_reply(agent.node_view(q.get("pool", "")))

    def claims(q, body):
        req = body_json(body)
        if not req.get("poolUID") or int(req.get("count", 0)) <= 0:
            return json_reply({"reason": "BadRequest", "message": "poolUID and count>0 required"},
                              400)
        req["_t_in"] = time.perf_counter()
        pool = req["poolUID"]
        try:
            out = agent.claim(req, hold_events=True)
        except BaseException:
            agent.release_events(pool)
            raise
        tm = out.get("timingsMs")
        if tm is not None:  # reply serialisation (the claim ran on this connection's thread)
            tm["executorOut"] = round((time.perf_counter() - out.pop("_t_done")) * 1e3, 3)
        deferred = out.pop("_after", [])

        def after() -> None:  # the reply goes out first; then the deferred work and the events
            try:
                for fn in deferred:
                    fn()
            finally:
                agent.release_events(pool)
        return json_reply(out, after=after)

    def cordon(q, body):
        b = body_json(body)
        return json_reply(agent.cordon(b["poolUID"], b.get("uuids", [])))

    def release(q, body):
        b = body_json(body)
        out = agent.release(b["poolUID"], b.get("uuids", []))
        return json_reply(out, 200 if out.get("ok") else 409)

    def maintenance(q, body):
        b = body_json(body)
        out = agent.set_maintenance(str(b.get("gpu", "")), bool(b.get("on", True)),
                                    str(b.get("reason", "")))
        return json_reply(out, 200 if out.get("ok") else 404)

    def policy(q, body):
        b = body_json(body)
        return json_reply(agent.update_policy(b["poolUID"], b.get("policy") or {},
                                              b.get("resourceName")))

    def events(q, body):
        since = int(q.get("since", "-1"))
        timeout = min(float(q.get("timeoutSeconds", "30")), 300.0)
        gen, pools = agent.changed_since(since)
        if gen == since:
            with agent.gen_cv:
                agent.gen_cv.wait_for(lambda: agent.gen != since, timeout)
            gen, pools = agent.changed_since(since)
        return 200, "application/json", (json.dumps({"gen": gen, "pools": pools}) + "\n").encode(), None

    def sample(q, body):
        changed = agent.sample()
        return json_reply({"changed": sorted(changed), "gen": agent.gen})

    def scrub(q, body):
        """Synchronous HBM scrub of one free GPU (admin / tests): {"gpu": uuid|hipUUID|index,
        "windows": n}."""
        b = body_json(body)
        ref = str(b.get("gpu", ""))
        uuid = next((u for u, d in list(agent.by_uuid.items())
                     if ref in (u, d.get("hipUUID"), str(d.get("index")))), None)
        if uuid is None:
            return json_reply({"ok": False, "reason": "NotFound"}, 404)
        rec = agent.scrubber.scrub_device(uuid, int(b.get("windows") or 1), grace=False)
        return json_reply({"ok": True, "uuid": uuid, "coverage": agent.scrubber.coverage(uuid),
                           "record": rec})

    def xgmi_check(q, body):
        """Run the idle xGMI coverage ring now (admin / tests)."""
        return json_reply(agent.xgmi_recheck(True))

    def healthz(q, body):
        return text_reply("ok\n")

    def metrics(q, body):
        extra = agent.rpc.metrics_lines() if agent.rpc is not None else []
        return text_reply(agent.metrics_text() + "\n".join(extra) + ("\n" if extra else ""))

    return {("GET", "/v1/node"): node, ("POST", "/v1/claims"): claims,
            ("POST", "/v1/cordon"): cordon, ("POST", "/v1/release"): release,
            ("POST", "/v1/policy"): policy, ("POST", "/v1/maintenance"): maintenance,
            ("GET", "/v1/events"): events, ("POST", "/v1/sample"): sample,
            ("POST", "/v1/scrub"): scrub, ("POST", "/v1/xgmi-check"): xgmi_check,
            ("GET", "/healthz"): healthz, ("GET", "/metrics"): metrics}


def serve(agent: Agent, ready_file: str | None = None) -> None:
    """Start the RPC listeners and the agent's background loops; block until interrupted."""
    from .rpc import RpcServer
    srv = RpcServer(build_routes(agent), guard=agent.check_leader, auth=agent.rpc_auth())
    agent.rpc = srv
    # the start-up heap (modules, gRPC/protobuf descriptors, the device model) lives for the whole
    # run: out of the collector's generations, a full collection walks only what came after — one
    # over the whole heap costs ~6-8 ms, which a claim that happened to trigger it would pay
    import gc
    gc.collect()
    gc.freeze()
    if agent.cfg.socket:
        srv.listen_unix(agent.cfg.socket)
    if agent.cfg.listen:
        host, port = agent.cfg.listen.rsplit(":", 1)
        ctx = None
        if agent.cfg.tls_cert:  # across nodes the RPC (and its bearer token) travels encrypted
            import ssl
            ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
            ctx.minimum_version = ssl.TLSVersion.TLSv1_2
            ctx.load_cert_chain(agent.cfg.tls_cert, agent.cfg.tls_key or None)
        srv.listen_tcp(host, int(port), ctx)
    agent.start_background()
    if ready_file:
        with open(ready_file + ".tmp", "w") as f:
            json.dump({"node": agent.cfg.node, "endpoint": agent.endpoint(),
                       "devices": len(agent.by_uuid), "probe": agent.probe_mode}, f)
        os.replace(ready_file + ".tmp", ready_file)
    print(f"gpupool-agent {agent.cfg.node} serving on {agent.endpoint()}", flush=True)
    try:
        while True:
            time.sleep(3600)
    finally:
        srv.close()
