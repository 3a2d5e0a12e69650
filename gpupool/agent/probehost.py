"""Probe helpers: the claim-time GPU probe, the HBM scrubber's kernels and the xGMI peer ring run
in child processes of the node agent — never in the agent itself.

Why (the reference checks a GPU in a throwaway pod, ``kubectl run --rm --gpus=1 … nvidia-smi``,
GPU调度平台搭建.md:134-138, so a bad GPU takes down that pod and nothing else): a probe kernel that
takes a GPU memory fault makes the HIP runtime abort its process, and a GPU that hangs never returns
from the probe. Inside the agent — which is also the node's device plugin, health sampler and HBM
scrubber — the first took all GPUs of the node down with it, and the second wedged the claim and
left its pool waiting on a ``Probing`` GPU forever. Here:

  * one helper per GPU, started with ``ROCR_VISIBLE_DEVICES=<that GPU's UUID>``: it holds a HIP
    context on its GPU only, and a fault takes down that helper only — probes of the other GPUs go
    on in theirs;
  * a *fabric* helper that sees all of the node's GPUs runs the xGMI peer ring. Before it reports
    ready it enables peer access for every directed GPU pair and allocates the ring windows at the
    claim-time size (warm rings of every stride); on a multi-GPU node it
    starts with the GPU helpers and is resident — replaced after an exit like them — so no
    multi-GPU claim pays its HIP init; with ``fabric_idle_s`` > 0 it exits after that long idle
    instead and is started again on demand (its contexts cost VRAM on every GPU);
  * a helper whose HIP init does not finish within ``ready_timeout`` is killed and replaced as
    after a crash, and a request waits for a starting helper no longer than its own deadline;
  * every request has a deadline (``spec.probe.timeoutSeconds`` for probes and rings): past it the
    helper is SIGKILLed and the request fails (``ProbeTimeout``); a helper that dies mid-request
    fails what it had in flight (``ProbeCrashed``); a fresh child replaces it, with a backoff while
    crashes repeat — nothing is ever re-exec'd;
  * helpers are forked from a forkserver the agent starts before it makes any GPU call (amdsmi or
    HIP, ``start_spawner`` in ``__main__``): a helper never inherits GPU state, and no process that
    holds a GPU context ever execs. A helper dies with the forkserver (PR_SET_PDEATHSIG), which
    exits when the agent does, so a helper hung in a kernel never outlives its agent.

Protocol: a multiprocessing Connection carrying dicts. Requests ``{id, op, args}``, replies
``{id, ok, result | error}``, plus one ``{op: "ready"}`` when the helper's HIP is up. The helper runs
each request on its own thread (ctypes drops the GIL), so a scrubber's buffer free and a claim's
probe of the same GPU still proceed concurrently, as they did in one process.

Kinds: ``hip`` (libmi355x_probe.so, real MI355X) and ``sim`` (simprobe.py: the fake backend's
simulated kernels, so the whole machinery is exercised on CPU). Both honour two fault-overlay hooks
on the probe request: ``probeCrash`` (the helper aborts, as HIP does on a GPU memory fault) and
``probeHang`` (the request never returns, as on a hung GPU).
"""
from __future__ import annotations

import logging
import multiprocessing as mp
import os
import select
import signal
import threading
import time
from typing import Any

log = logging.getLogger("gpupool.agent.probehost")

_ctx = None
_ctx_mu = threading.Lock()


def spawner():
    """The forkserver context the helpers are forked from (created on first use)."""
    global _ctx
    with _ctx_mu:
        if _ctx is None:
            ctx = mp.get_context("forkserver")
            ctx.set_forkserver_preload(["gpupool.agent.probehost"])
            _ctx = ctx
        return _ctx


def start_spawner() -> None:
    """Start the forkserver now. The agent calls this first thing, before any amdsmi or HIP call,
    so every helper is forked from a process that never touched a GPU."""
    spawner()
    from multiprocessing import forkserver
    forkserver.ensure_running()


# ============================================================================ the child side
def _die_with_parent() -> None:
    try:
        import ctypes
        ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGKILL)  # PR_SET_PDEATHSIG
    except Exception:
        pass


class _HipKernel:
    """libmi355x_probe.so in the helper: HIP initialised on the visible GPU(s) only."""

    def __init__(self, spec: dict):
        from ..ops import probe as hp
        self.hp = hp
        self.n = hp.init()
        self.uuids = hp.hip_uuid_map()  # hipUUID (lower) -> ordinal
        self.single = bool(spec.get("single"))
        idle_ms = int(float(spec.get("arenaIdleS", 10.0)) * 1e3)
        if idle_ms > 0:
            # probe arenas stay allocated between back-to-back claims (scale-up bursts) and are
            # handed back to the GPU's workloads once idle
            def trim():
                period = max(0.05, min(1.0, idle_ms / 4e3))
                while True:
                    time.sleep(period)
                    try:
                        hp.trim(idle_ms)
                    except Exception:
                        pass
            threading.Thread(target=trim, daemon=True, name="probe-trim").start()

    def info(self) -> dict:
        return {"devices": self.n, "uuids": self.uuids}

    WARM_RING_BYTES = 16 << 20  # the claim-time ring's size (prober: xgmiBytes default)

    def warm_ring(self) -> dict:
        """Before the helper says it is ready: every directed GPU pair's peer access enabled and
        the ring windows allocated at the claim-time size, so no claim's ring does either. The
        claims' rings rotate over the least recently checked pairs (agent._ring_order), so over a
        node's first claims every pair would otherwise pay its first enable inside a claim. Rings
        of stride s = 1 .. n-1 (each cycle of i -> i+s mod n) cover all n(n-1) directed pairs."""
        if self.n < 2:
            return {}
        n, links, ok = self.n, 0, True
        for stride in range(1, n):
            seen: set[int] = set()
            for start in range(n):
                if start in seen:
                    continue
                cycle, i = [], start
                while i not in seen:
                    seen.add(i)
                    cycle.append(i)
                    i = (i + stride) % n
                if len(cycle) < 2:
                    continue
                r = self.hp.peer_ring(cycle, self.WARM_RING_BYTES)
                links += len(r.get("links") or [])
                ok = ok and bool(r.get("passed"))
        return {"passed": ok, "links": links}

    def ordinal(self, hip_uuid: str) -> int:
        o = self.uuids.get(str(hip_uuid or "").lower())
        if o is None and self.single and self.n == 1:
            return 0  # the one GPU this helper was started for (no hipUUID to match on)
        if o is None:
            raise LookupError(f"device {hip_uuid!r} not visible to HIP in this helper")
        return o

    def call(self, op: str, a: dict) -> Any:
        hp = self.hp
        if op == "probe":
            return hp.run(self.ordinal(a.get("hipUUID")), hbm_bytes=int(a["hbmBytes"]),
                          mfma=bool(a["mfma"]), gemm_n=int(a["gemmN"]), overlap=int(a["overlap"]),
                          **{k: int(v) for k, v in (a.get("testHooks") or {}).items()})
        if op == "sweep":
            return hp.hbm_sweep(self.ordinal(a.get("hipUUID")), int(a["offset"]), int(a["bytes"]),
                                int(a["reserve"]), keep=bool(a.get("keep")))
        if op == "sweep_alloc":
            return hp.sweep_alloc(self.ordinal(a.get("hipUUID")), int(a["reserve"]))
        if op == "sweep_release":
            return hp.sweep_release(self.ordinal(a.get("hipUUID")))
        if op == "warm":
            return hp.run(self.ordinal(a.get("hipUUID")), hbm_bytes=int(a.get("hbmBytes", 1 << 30)),
                          gemm_n=int(a.get("gemmN", 4096)))
        if op == "peer_ring":
            return hp.peer_ring([self.ordinal(u) for u in a["hipUUIDs"]], int(a["bytes"]))
        if op == "peer":
            return hp.peer(self.ordinal(a["src"]), self.ordinal(a["dst"]), int(a["bytes"]))
        if op == "ping":
            return {"pid": os.getpid()}
        raise ValueError(f"unknown helper op {op!r}")


class _SimKernel:
    """The fake backend's simulated kernels (simprobe.py) behind the same protocol."""

    def __init__(self, spec: dict):
        self.sim_ms = float(spec.get("simMs", 20.0))
        self.n = int(spec.get("devices") or 1)
        if spec.get("initHang"):  # test hook: a HIP init that never returns
            threading.Event().wait()
        if spec.get("initDelayS"):  # test hook: a slow HIP init (a respawned helper)
            time.sleep(float(spec["initDelayS"]))

    def info(self) -> dict:
        return {"devices": self.n, "uuids": {}}

    def warm_ring(self) -> dict:
        return {"passed": True, "links": self.n * (self.n - 1)} if self.n >= 2 else {}

    def call(self, op: str, a: dict) -> Any:
        from . import simprobe
        if op == "probe":
            return simprobe.probe(a.get("dev") or {}, a.get("opts") or {}, self.sim_ms)
        if op == "sweep":
            return simprobe.sweep_window(a.get("dev") or {}, int(a["offset"]), int(a["bytes"]),
                                         int(a["reserve"]))
        if op in ("sweep_alloc", "warm"):
            time.sleep(0.001)
            return 1
        if op == "sweep_release":
            return 0
        if op == "peer_ring":
            devs = a["devs"]
            links = [simprobe.link(devs[i], devs[(i + 1) % len(devs)]) for i in range(len(devs))]
            return {"links": links, "passed": all(x.get("passed") for x in links)}
        if op == "peer":
            return simprobe.link(a["srcDev"], a["dstDev"])
        if op == "ping":
            return {"pid": os.getpid()}
        raise ValueError(f"unknown helper op {op!r}")


def _apply_hooks(a: dict) -> None:
    hooks = a.get("hooks") or {}
    if hooks.get("crash"):
        # what the HIP runtime does on a GPU memory fault: abort the process (no core file)
        try:
            import resource
            resource.setrlimit(resource.RLIMIT_CORE, (0, 0))
        except (ImportError, ValueError, OSError):
            pass
        os.abort()
    if hooks.get("hang"):
        # a GPU that never finishes the probe: this request never returns
        threading.Event().wait()


# run on the helper's main thread: short, and what a claim waits for; everything else gets a thread
_INLINE_OPS = ("probe", "ping")
# After a "wake" the helper polls its pipe without sleeping for at most this long: a claim sends
# "wake" as soon as it has chosen its GPUs, so the probe request that follows ~0.1-0.2 ms later is
# picked up by a running thread instead of one the kernel must first wake (tens to hundreds of us
# when the core idles in a deep C-state). Only after a wake, and bounded: an idle helper costs no
# CPU, and none spins once its probe is answered.
SPIN_S = float(os.environ.get("GPUPOOL_HELPER_SPIN_MS", "1")) / 1e3


def child_main(conn, spec: dict) -> None:
    """Entry point of a helper process (forked from the forkserver)."""
    spin_s = float(spec.get("spinS", SPIN_S))
    _die_with_parent()
    signal.signal(signal.SIGINT, signal.SIG_IGN)  # the agent decides when helpers stop
    for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        os.environ.pop(k, None)
    if spec.get("visible") is not None:
        os.environ["ROCR_VISIBLE_DEVICES"] = str(spec["visible"])
    for k, v in (spec.get("env") or {}).items():  # read by the HIP runtime at its init, below
        os.environ[str(k)] = str(v)
    send_mu = threading.Lock()

    def send(msg: dict) -> None:
        with send_mu:
            conn.send(msg)
    t0 = time.perf_counter()
    try:
        kernel = _HipKernel(spec) if spec.get("kind") == "hip" else _SimKernel(spec)
        info = kernel.info()
    except BaseException as e:  # HIP init failed: say so, then exit
        try:
            send({"op": "ready", "ok": False, "error": repr(e)})
        finally:
            os._exit(3)
    info["initMs"] = round((time.perf_counter() - t0) * 1e3, 1)
    if spec.get("warmRing"):
        # the fabric helper: its first ring's peer-access enable and window allocation happen
        # here, not inside a claim's deadline. A failure is reported, not fatal: the rings that
        # follow report it per link (XGMIPeerCheckUnavailable)
        t1 = time.perf_counter()
        try:
            info["warm"] = kernel.warm_ring()
        except Exception as e:
            info["warm"] = {"passed": False, "error": f"{type(e).__name__}: {e}"}
        info["warmMs"] = round((time.perf_counter() - t1) * 1e3, 1)
    send({"op": "ready", "ok": True, "pid": os.getpid(), **info})

    def run(msg: dict) -> None:
        try:
            a = msg.get("args") or {}
            if msg.get("op") == "probe":
                _apply_hooks(a)
            out = {"id": msg["id"], "ok": True, "result": kernel.call(msg["op"], a)}
        except Exception as e:
            out = {"id": msg["id"], "ok": False, "error": f"{type(e).__name__}: {e}"}
        try:
            send(out)
        except (OSError, ValueError):
            pass
    spin_until = 0.0
    while True:
        try:
            if spin_until:
                while time.perf_counter() < spin_until and \
                        not select.select([conn], [], [], 0)[0]:
                    pass
                spin_until = 0.0
            msg = conn.recv()
        except (EOFError, OSError):
            os._exit(0)  # the agent is gone
        if msg.get("op") == "exit":
            os._exit(0)
        if msg.get("op") == "wake":  # a request is on its way: just be awake for it
            spin_until = time.perf_counter() + spin_s
            continue
        if msg.get("op") in _INLINE_OPS:
            run(msg)  # the claim path: no thread start between the pipe and the kernels
        else:  # long operations (a sweep buffer's free takes seconds) never hold up a probe
            threading.Thread(target=run, args=(msg,), daemon=True, name=f"req-{msg.get('op')}").start()


# ============================================================================ the agent side
_start_mu = threading.Lock()


def _start_without_main(proc) -> None:
    """``proc.start()`` without the parent's ``__main__`` in the child's preparation data.
    multiprocessing re-imports the parent's main module in every child it starts (as
    ``__mp_main__``), which for a bench script or a test runner would import torch & co. into each
    probe helper; a helper needs only this module (preloaded in the forkserver)."""
    from multiprocessing import spawn
    with _start_mu:
        orig = spawn.get_preparation_data

        def prep(name):
            d = orig(name)
            d.pop("init_main_from_name", None)
            d.pop("init_main_from_path", None)
            return d
        spawn.get_preparation_data = prep
        try:
            proc.start()
        finally:
            spawn.get_preparation_data = orig


class HelperError(Exception):
    """A request the helper could not answer. ``kind``: ProbeCrashed | ProbeTimeout |
    ProbeUnavailable."""
    kind = "ProbeCrashed"


class HelperDied(HelperError):
    kind = "ProbeCrashed"


class HelperTimeout(HelperError):
    kind = "ProbeTimeout"


class HelperUnavailable(HelperError):
    kind = "ProbeUnavailable"


def describe_exit(code: int | None) -> str:
    if code is None:
        return "still running"
    if code < 0:
        try:
            return f"killed by {signal.Signals(-code).name}"
        except ValueError:
            return f"killed by signal {-code}"
    return f"exited with status {code}"


class _Slot:
    __slots__ = ("ev", "done", "ok", "result", "error", "died")

    def __init__(self):
        self.ev = threading.Event()  # "look again": the reply is in, or it is your turn to read
        self.done = False
        self.ok = False
        self.result = None
        self.error = ""
        self.died = ""


class Helper:
    """One helper process and its in-flight requests.

    Replies are read by the callers themselves, leader/follower style: whichever waiting caller
    holds ``_rd`` reads the pipe and hands out what arrives; when it has its own reply it wakes a
    follower to take over. A reply therefore wakes the thread that waits for it directly — a
    dedicated reader thread put one more thread wake-up (~0.3 ms on a CPU coming out of idle) on
    every claim-time probe. A watcher thread waits on the process sentinel for deaths between
    requests."""

    # A caller waiting for a reply polls the pipe without sleeping for this long first (the
    # claim-time probe takes ~0.85 ms on MI355X): the reply is read the moment it lands instead of
    # after the kernel has woken the blocked thread. Longer requests then block as usual.
    CALLER_SPIN_S = float(os.environ.get("GPUPOOL_CALLER_SPIN_MS", "0")) / 1e3
    FOLLOWER_SLICE_S = 0.05

    def __init__(self, key: str, spec: dict, on_exit=None, ready_timeout: float = 120.0):
        self.key = key
        self.spec = spec
        self.on_exit = on_exit
        self.ready_timeout = ready_timeout  # HIP init (+ the fabric's warm ring) must finish by then
        self.proc = None
        self.conn = None
        self.pid = 0
        self.info: dict = {}
        self.ready = threading.Event()
        self.ready_ok = False
        self.ready_error = ""
        self.dead = ""            # why it is gone ("" while alive)
        self.killed_for = ""      # what kill() was told (a missed deadline)
        self.cause = ""           # timeout | stop | idle; "" = it died on its own (a crash)
        self.started = 0.0
        self.last_used = time.monotonic()
        self._mu = threading.Lock()
        self._send_mu = threading.Lock()
        self._rd = threading.Lock()  # held by the thread reading the pipe
        self._seq = 0
        self._pending: dict[int, _Slot] = {}
        self._exited = False

    def start(self) -> "Helper":
        ctx = spawner()
        parent, child = ctx.Pipe()
        self.conn = parent
        self.started = time.monotonic()
        self.proc = ctx.Process(target=child_main, args=(child, self.spec), daemon=True,
                                name=f"gpupool-probe-{self.key}")
        _start_without_main(self.proc)
        child.close()
        self.pid = self.proc.pid
        self._rd.acquire()  # the watcher reads the ready message, then hands the pipe over
        threading.Thread(target=self._watch, daemon=True, name=f"helper-{self.key}").start()
        return self

    # ------------------------------------------------------------ reading
    def _deliver(self, msg: dict) -> None:
        if msg.get("op") == "ready":
            self.info = msg
            self.ready_ok = bool(msg.get("ok"))
            self.ready_error = str(msg.get("error") or "")
            self.ready.set()
            return
        with self._mu:
            slot = self._pending.pop(msg.get("id"), None)
        if slot is not None:
            slot.ok = bool(msg.get("ok"))
            slot.result = msg.get("result")
            slot.error = str(msg.get("error") or "")
            slot.done = True
            slot.ev.set()

    def notify(self, op: str) -> None:
        """A message that needs no reply ("wake": a request follows shortly)."""
        if self.dead or not self.ready_ok:
            return
        try:
            with self._send_mu:
                self.conn.send({"op": op})
        except (OSError, ValueError):
            pass

    def _read_one(self, timeout: float) -> bool:
        """Read and deliver one message (caller holds _rd). False: the pipe is closed."""
        try:
            # select() directly: Connection.poll builds a selector per call (~50 us measured)
            if select.select([self.conn], [], [], max(0.0, timeout))[0]:
                self._deliver(self.conn.recv())
            return True
        except (EOFError, OSError, ValueError):
            return False

    def _watch(self) -> None:
        from multiprocessing.connection import wait
        try:  # the ready message (HIP init on the GPU: up to seconds)
            give_up = self.started + self.ready_timeout
            while not self.ready.is_set():
                if time.monotonic() > give_up:  # an init that hangs: replaced like a crash
                    self.kill(f"probe helper {self.key} not ready within "
                              f"{self.ready_timeout:g} s (HIP init hung)")
                    break
                if not self._read_one(1.0):
                    break
        finally:
            self._rd.release()
            # a caller that arrived while the watcher held the pipe (its ready.wait returned,
            # then _rd was taken) must not sleep out its deadline with nobody reading
            self._wake_follower()
        try:
            wait([self.proc.sentinel])
        except (OSError, ValueError):
            pass
        # the process is gone: deliver what it wrote before it went, then fail the rest
        if self._rd.acquire(timeout=5.0):
            try:
                while self._read_one(0):
                    if not self.conn.poll(0):
                        break
            finally:
                self._rd.release()
        self._died()

    def _died(self) -> None:
        with self._mu:
            if self._exited:
                return
            self._exited = True
        code = None
        try:
            self.proc.join(2.0)
            code = self.proc.exitcode
        except Exception:
            pass
        why = self.killed_for or f"probe helper pid {self.pid} {describe_exit(code)}"
        with self._mu:
            self.dead = why
            pending, self._pending = self._pending, {}
        if not self.ready.is_set():
            self.ready_error = self.ready_error or why
            self.ready.set()
        for slot in pending.values():
            slot.died = why
            slot.done = True
            slot.ev.set()
        if self.on_exit is not None:
            try:
                self.on_exit(self, why, self.cause or "crash")
            except Exception:
                log.exception("helper exit hook failed")

    def _wake_follower(self) -> None:
        with self._mu:
            for slot in self._pending.values():
                if not slot.done:
                    slot.ev.set()
                    return

    # ------------------------------------------------------------ requests
    @property
    def alive(self) -> bool:
        return not self.dead and self.proc is not None and self.ready_ok

    def wait_ready(self, timeout: float) -> bool:
        return self.ready.wait(timeout) and self.ready_ok and not self.dead

    def call(self, op: str, args: dict, timeout: float) -> Any:
        """Run ``op`` in the helper. Raises HelperTimeout past ``timeout`` (the caller decides
        whether to kill), HelperDied if the helper is or goes away, HelperUnavailable if its HIP
        has not come up within the request's own deadline (a helper being replaced) or never
        does; RuntimeError for an error the request itself raised."""
        # one deadline for the whole request: waiting for a (re)starting helper's HIP init comes
        # out of the same spec.probe.timeoutSeconds as the probe itself
        deadline = time.monotonic() + timeout
        wait = min(timeout, self.ready_timeout)
        if not self.ready.wait(wait):
            raise HelperUnavailable(f"probe helper {self.key} still starting after {wait:g} s")
        if not self.ready_ok:
            raise HelperUnavailable(f"probe helper {self.key}: {self.ready_error or self.dead}")
        slot = _Slot()
        with self._mu:
            if self.dead:
                raise HelperDied(self.dead)
            self._seq += 1
            rid = self._seq
            self._pending[rid] = slot
        self.last_used = time.monotonic()
        try:
            with self._send_mu:
                self.conn.send({"id": rid, "op": op, "args": args})
        except (OSError, ValueError) as e:
            with self._mu:
                self._pending.pop(rid, None)
            raise HelperDied(self.dead or f"probe helper {self.key} unreachable: {e}") from None
        spin_end = time.perf_counter() + self.CALLER_SPIN_S
        while True:
            slot.ev.clear()
            if slot.done:
                break
            left = deadline - time.monotonic()
            if left <= 0:
                break
            if self._rd.acquire(blocking=False):
                closed = False
                try:
                    while not slot.done and not self.dead:
                        left = deadline - time.monotonic()
                        if left <= 0:
                            break
                        spin = time.perf_counter() < spin_end
                        if not self._read_one(0.0 if spin else min(left, 0.5)):
                            closed = True
                            break
                finally:
                    self._rd.release()
                    self._wake_follower()
                if closed:
                    self._died()  # EOF: the helper is gone (the watcher agrees shortly)
            else:
                # in slices: a hand-over of the reader role can miss this caller (the reader
                # woke a follower that was timing out, or none at all); trying _rd again every
                # FOLLOWER_SLICE_S bounds what a missed wake costs to that, not the deadline
                slot.ev.wait(min(left, self.FOLLOWER_SLICE_S))
        if not slot.done:
            with self._mu:
                self._pending.pop(rid, None)
            raise HelperTimeout(f"{op} did not finish within {timeout:g} s (including the "
                                f"helper's start)")
        self.last_used = time.monotonic()
        if slot.died:
            raise HelperDied(slot.died)
        if not slot.ok:
            raise RuntimeError(slot.error)
        return slot.result

    def kill(self, why: str) -> None:
        """SIGKILL the helper (a request past its deadline); its other requests fail."""
        self.killed_for = why
        self.cause = self.cause or "timeout"
        try:
            if self.proc is not None and self.proc.is_alive():
                self.proc.kill()
        except Exception:
            pass

    def stop(self, cause: str = "stop") -> None:
        self.cause = self.cause or cause
        self.killed_for = self.killed_for or f"probe helper pid {self.pid} stopped ({self.cause})"
        try:
            with self._send_mu:
                self.conn.send({"op": "exit"})
        except (OSError, ValueError, AttributeError):
            pass
        try:
            if self.proc is not None:
                self.proc.join(2.0)
                if self.proc.is_alive():
                    self.proc.kill()
                    self.proc.join(2.0)
        except Exception:
            pass


# Hardware queues per GPU in the fabric helper (0 = the runtime's default). Every HIP hardware
# queue of an MI355X carries a context-save area for all 256 CUs' waves — 173 MiB of host memory
# each (native/tests/queue_mem.hip, profiles/r5i_hip_host_memory.json) — and a context starts with
# two. One queue per GPU saves 175 MiB of host memory per GPU in the fabric helper (1.4 GB on an
# 8-GPU node) but measured +0.09 ms on a ring (profiles/r5j_helper_footprint.json): the default
# keeps the runtime's queues, for the multi-GPU claim's latency; set 1 where host RAM is tight.
FABRIC_HW_QUEUES = int(os.environ.get("GPUPOOL_FABRIC_HW_QUEUES", "0"))


class HelperPool:
    """The agent's helpers: one per GPU (keyed by uuid), plus the on-demand fabric helper.

    A helper that crashed or was killed at a deadline is replaced by a fresh child: at once after
    the first exit, then with a backoff doubling per further exit within ``crash_window_s`` (up to
    ``max_backoff_s``), so a GPU that kills every helper does not spin the node's CPUs."""

    def __init__(self, kind: str, sim_ms: float = 20.0, arena_idle_s: float = 10.0,
                 fabric_idle_s: float = 0.0, ready_timeout: float = 120.0,
                 max_backoff_s: float = 60.0, crash_window_s: float = 300.0,
                 resident_fabric: bool = False):
        self.kind = kind
        # resident: the fabric helper is started with the GPU helpers (2+ GPUs) and replaced
        # like them after an exit; otherwise it starts on a ring's demand
        self.resident_fabric = resident_fabric
        self.sim_ms = sim_ms
        self.arena_idle_s = arena_idle_s
        self.fabric_idle_s = fabric_idle_s
        self.ready_timeout = ready_timeout
        self.max_backoff_s = max_backoff_s
        self.crash_window_s = crash_window_s
        self._mu = threading.Lock()
        self._helpers: dict[str, Helper] = {}
        self._devs: dict[str, dict] = {}
        self._exits: dict[str, list[float]] = {}   # key -> monotonic times of recent exits
        self._respawn_at: dict[str, float] = {}
        self._stopping = False
        self.stats = {"helper_starts": 0, "helper_crashes": 0, "helper_timeouts": 0}
        self.last_exit: dict[str, str] = {}
        self._fabric_devs: list[dict] = []
        # GPUs whose helper is parked: a tenant pod holds the GPU, so the agent keeps no HIP
        # context (no VRAM, no process) on it; requests for it are refused until unpark()
        self._parked: set[str] = set()
        self._fabric_timer_armed = False
        if fabric_idle_s > 0:
            threading.Thread(target=self._fabric_reaper, daemon=True, name="fabric-idle").start()

    # ------------------------------------------------------------ specs
    def _gpu_spec(self, dev: dict) -> dict:
        spec = {"kind": self.kind, "single": True, "simMs": self.sim_ms,
                "arenaIdleS": self.arena_idle_s, "devices": 1}
        if self.kind == "hip":
            spec["visible"] = dev.get("hipUUID") or str(dev.get("index", 0))
        elif os.environ.get("GPUPOOL_HELPER_SIM_INIT_S"):  # test hook: a HIP init's duration
            spec["initDelayS"] = float(os.environ["GPUPOOL_HELPER_SIM_INIT_S"])
        return spec

    def _fabric_spec(self) -> dict:
        spec = {"kind": self.kind, "single": False, "simMs": self.sim_ms, "arenaIdleS": 0,
                "devices": len(self._fabric_devs), "warmRing": True}
        if FABRIC_HW_QUEUES > 0:
            spec["env"] = {"GPU_MAX_HW_QUEUES": str(FABRIC_HW_QUEUES)}
        if self.kind == "hip":
            ids = [d.get("hipUUID") or str(d.get("index", 0)) for d in self._fabric_devs]
            spec["visible"] = ",".join(ids)
        return spec

    # ------------------------------------------------------------ lifecycle
    def start(self, devs: list[dict], wait: bool = True) -> dict[str, dict]:
        """One helper per device, started concurrently; with ``wait`` block until each is ready
        (or failed). Returns uuid -> the helper's ready message."""
        with self._mu:
            for d in devs:
                self._devs[d["uuid"]] = d
            self._fabric_devs = self._unparked_devs_locked()
            new = [self._spawn_locked(d["uuid"]) for d in devs
                   if d["uuid"] not in self._helpers and d["uuid"] not in self._parked]
            if self._fabric_wanted_locked() and "fabric" not in self._helpers:
                self._spawn_locked("fabric")  # warms itself; nothing waits for it here
        if wait:
            deadline = time.monotonic() + self.ready_timeout
            for h in new:
                h.ready.wait(max(0.0, deadline - time.monotonic()))
        return {u: dict(h.info) for u, h in self._helpers.items()}

    def _fabric_wanted_locked(self) -> bool:
        return self.resident_fabric and len(self._fabric_devs) >= 2 and not self._stopping

    def _unparked_devs_locked(self) -> list[dict]:
        return sorted((d for u, d in self._devs.items() if u not in self._parked),
                      key=lambda d: d.get("index", 0))

    # ------------------------------------------------------------ parking
    def park(self, key: str) -> bool:
        """Stop ``key``'s helper and keep it stopped (a tenant holds the GPU). The resident
        fabric helper, which has a context on every GPU, is restarted over the others. True if
        the GPU was not parked before."""
        stop: list[Helper] = []
        with self._mu:
            if key in self._parked or key == "fabric":
                return False
            self._parked.add(key)
            h = self._helpers.pop(key, None)
            if h is not None:
                stop.append(h)
            if any(d["uuid"] == key for d in self._fabric_devs):
                self._fabric_devs = self._unparked_devs_locked()
                f = self._helpers.pop("fabric", None)
                if f is not None:
                    stop.append(f)  # it has a context on this GPU: it goes now
                self._respawn_fabric_later_locked()
            self.stats["helper_parks"] = self.stats.get("helper_parks", 0) + 1
        for x in stop:  # off the caller's path (a cordon, a pod-view refresh): ~60 ms a stop
            threading.Thread(target=x.stop, args=("park",), daemon=True,
                             name=f"park-{x.key[:8]}").start()
        return True

    def unpark(self, key: str) -> Helper | None:
        """Start ``key``'s helper again (its GPU is pod-free); the fabric helper follows. Returns
        the starting helper (its ``ready`` event fires once HIP is up), None if not parked."""
        with self._mu:
            if key not in self._parked:
                return None
            self._parked.discard(key)
            if key not in self._devs or self._stopping:
                return None
            self._respawn_at.pop(key, None)
            h = self._helpers.get(key) or self._spawn_locked(key)
            fabric_devs = self._unparked_devs_locked()
            if self.resident_fabric and {d["uuid"] for d in fabric_devs} != \
                    {d["uuid"] for d in self._fabric_devs}:
                self._fabric_devs = fabric_devs
                f = self._helpers.pop("fabric", None)
                if f is not None:
                    threading.Thread(target=f.stop, args=("park",), daemon=True).start()
                self._respawn_fabric_later_locked()
            self.stats["helper_unparks"] = self.stats.get("helper_unparks", 0) + 1
        return h

    # a burst of parks / unparks (a drain of several GPUs, a gang's pods starting) restarts the
    # resident fabric helper once, over the GPUs pod-free at the end of the burst, not once per GPU
    # (each start is a HIP init on every GPU plus the all-pairs warm-up)
    FABRIC_RESPAWN_DEBOUNCE_S = 0.25

    def _respawn_fabric_later_locked(self) -> None:
        if not self.resident_fabric or self._fabric_timer_armed:
            return
        self._fabric_timer_armed = True

        def fire() -> None:
            with self._mu:
                self._fabric_timer_armed = False
                self._fabric_devs = self._unparked_devs_locked()
                if self._fabric_wanted_locked() and "fabric" not in self._helpers:
                    self._spawn_locked("fabric")
                    self.stats["fabric_respawns"] = self.stats.get("fabric_respawns", 0) + 1
        t = threading.Timer(self.FABRIC_RESPAWN_DEBOUNCE_S, fire)
        t.daemon = True
        t.start()

    def parked(self) -> set[str]:
        with self._mu:
            return set(self._parked)

    def wait_ready(self, key: str, timeout: float) -> float:
        """Block until ``key``'s helper is up (or ``timeout``); the ms waited."""
        t0 = time.perf_counter()
        with self._mu:
            h = self._helpers.get(key)
        if h is not None:
            h.ready.wait(timeout)
        return (time.perf_counter() - t0) * 1e3

    def restart(self, key: str) -> None:
        """Replace ``key``'s helper with a fresh process (a GPU reset invalidated its context)."""
        with self._mu:
            h = self._helpers.pop(key, None)
            if key in self._parked or key not in self._devs or self._stopping:
                new = None
            else:
                self._respawn_at.pop(key, None)
                new = self._spawn_locked(key)
        if h is not None:
            h.stop("stop")
        if new is not None:
            new.ready.wait(self.ready_timeout)

    def _spawn_locked(self, key: str) -> Helper:
        spec = self._fabric_spec() if key == "fabric" else self._gpu_spec(self._devs[key])
        h = Helper(key, spec, on_exit=self._on_exit, ready_timeout=self.ready_timeout).start()
        self._helpers[key] = h
        self.stats["helper_starts"] += 1
        return h

    def _on_exit(self, h: Helper, why: str, cause: str) -> None:
        with self._mu:
            if self._stopping or self._helpers.get(h.key) is not h:
                return
            del self._helpers[h.key]
            if cause in ("stop", "idle", "park"):
                return  # let go on purpose (an idle fabric helper): started again on demand
            self.last_exit[h.key] = why
            now = time.monotonic()
            recent = [t for t in self._exits.get(h.key, []) if now - t < self.crash_window_s] + [now]
            self._exits[h.key] = recent
            if cause == "timeout":
                self.stats["helper_timeouts"] += 1
            else:
                self.stats["helper_crashes"] += 1
            delay = 0.0 if len(recent) <= 1 else min(self.max_backoff_s, 2.0 ** (len(recent) - 2))
            self._respawn_at[h.key] = now + delay
        log.warning("probe helper %s gone (%s); replacing it%s", h.key, why,
                    f" in {delay:.0f} s" if delay else "")
        if h.key != "fabric" or self.resident_fabric:
            t = threading.Timer(delay, self._respawn, args=(h.key,))
            t.daemon = True
            t.start()

    def _respawn(self, key: str) -> None:
        with self._mu:
            if self._stopping or key in self._helpers or key in self._parked:
                return
            if key not in self._devs and not (key == "fabric" and self._fabric_wanted_locked()):
                return
            if time.monotonic() < self._respawn_at.get(key, 0.0):
                return
            self._spawn_locked(key)

    def get(self, key: str, dev: dict | None = None) -> Helper:
        """The live helper for ``key`` (a GPU uuid or "fabric"), starting it if needed. Raises
        HelperUnavailable while a crashing helper's backoff runs."""
        with self._mu:
            h = self._helpers.get(key)
            if h is not None and not h.dead:
                return h
            if key in self._parked:
                raise HelperUnavailable(f"probe helper for {key} is parked: a pod holds the GPU")
            if dev is not None and key != "fabric":
                self._devs[key] = dev
            wait = self._respawn_at.get(key, 0.0) - time.monotonic()
            if wait > 0:
                raise HelperUnavailable(f"probe helper for {key} is being replaced after "
                                        f"{self.last_exit.get(key, 'an exit')} (retry in "
                                        f"{wait:.0f} s)")
            if key != "fabric" and key not in self._devs:
                raise HelperUnavailable(f"no probe helper for unknown device {key}")
            return self._spawn_locked(key)

    def fabric(self, devs: list[dict]) -> Helper:
        """The helper that sees all the node's GPUs (xGMI peer copies), for ``devs``' ring.
        Restarted when the ring needs a GPU it was not started with."""
        with self._mu:
            for d in devs:
                self._devs.setdefault(d["uuid"], d)
            want = {d["uuid"] for d in devs}
            if want & self._parked:
                raise HelperUnavailable(f"a ring over GPUs with tenant pods ({sorted(want & self._parked)}): "
                                        f"their helpers are parked")
            have = {d["uuid"] for d in self._fabric_devs}
            h = self._helpers.get("fabric")
            if not want <= have:
                self._fabric_devs = self._unparked_devs_locked()
                if h is not None:
                    self._helpers.pop("fabric", None)
                    threading.Thread(target=h.stop, daemon=True).start()
        return self.get("fabric")

    def _fabric_reaper(self) -> None:
        while not self._stopping:
            time.sleep(min(5.0, max(0.5, self.fabric_idle_s / 4)))
            with self._mu:
                h = self._helpers.get("fabric")
                if h is None or h.dead or h._pending:
                    continue
                if time.monotonic() - h.last_used < self.fabric_idle_s:
                    continue
                # out of the table first: a ring arriving now starts a fresh helper instead of
                # being sent to this one while it stops
                self._helpers.pop("fabric", None)
            h.stop("idle")

    def kill(self, key: str, why: str) -> None:
        with self._mu:
            h = self._helpers.get(key)
        if h is not None:
            h.kill(why)

    def available(self, key: str) -> bool:
        """Can a request for ``key`` be served now or once its helper has started? False while
        a helper that exited is held back by its respawn backoff, and while it is parked."""
        with self._mu:
            if key in self._parked:
                return False
            h = self._helpers.get(key)
            if h is not None and not h.dead:
                return True
            return time.monotonic() >= self._respawn_at.get(key, 0.0)

    def alive(self, key: str) -> bool:
        with self._mu:
            h = self._helpers.get(key)
        return h is not None and h.alive

    def pids(self) -> set[int]:
        with self._mu:
            return {h.pid for h in self._helpers.values() if h.pid and not h.dead}

    def snapshot(self) -> dict[str, dict]:
        """key -> {pid, alive, initMs, lastExit} (metrics, node view)."""
        with self._mu:
            out = {}
            for k, h in self._helpers.items():
                out[k] = {"pid": h.pid, "alive": h.alive, "initMs": h.info.get("initMs")}
                if "warmMs" in h.info:
                    out[k]["warmMs"] = h.info["warmMs"]
                    out[k]["warm"] = h.info.get("warm")
            for k, why in self.last_exit.items():
                out.setdefault(k, {"alive": False})["lastExit"] = why
            for k in self._parked:
                out.setdefault(k, {"alive": False})["parked"] = True
            return out

    def stop(self) -> None:
        with self._mu:
            self._stopping = True
            hs = list(self._helpers.values())
            self._helpers.clear()
        for h in hs:
            h.stop()
