"""Process fixtures: run the signal server, ``tunnel serve`` and ``tunnel
proxy`` as real child processes and wait on their log lines.

Replaces the reference's fixed ``sleep`` calls (scripts/test-local.sh:101)
with readiness on the load-bearing log strings "tunnel ready" and
"proxy listening" (reference scripts/test-tunnel.sh:79-86).
"""
from __future__ import annotations

import os
import re
import signal
import socket
import subprocess
import threading
import time
from dataclasses import dataclass, field

from p2p_llm_tunnel_amd import binary


_next_port = [0]


def free_port(host: str = "127.0.0.1") -> int:
    """A currently free TCP port, taken in order from a block below the
    kernel's ephemeral range (32768-60999 by default). A port from bind(0)
    comes from that range, so an outgoing connection made between our close()
    and the child's bind() (an upstream pre-warm, a load generator) could take
    it: on the MI355X host a proxy's listen port was once held that way for a
    whole bench run (profiles/r06/b03). P2PT_PORT_BASE picks the block (bench.py
    sets a disjoint one per rank); by default it follows the pid, so
    concurrent test processes rarely meet."""
    base = int(os.environ.get("P2PT_PORT_BASE", "0")) or 10000 + (os.getpid() * 500) % 20000
    for _ in range(500):
        port = base + _next_port[0] % 500
        _next_port[0] += 1
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind((host, port))
            except OSError:
                continue
            return port
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


@dataclass
class Proc:
    name: str
    popen: subprocess.Popen
    lines: list = field(default_factory=list)
    _cv: threading.Condition = field(default_factory=threading.Condition)

    def _pump(self):
        for raw in self.popen.stdout:
            line = raw.decode("utf-8", "replace").rstrip("\n")
            with self._cv:
                self.lines.append(line)
                self._cv.notify_all()
        with self._cv:
            self._cv.notify_all()

    def wait_for(self, pattern: str, timeout: float = 30.0, start: int = 0) -> str:
        rx = re.compile(pattern)
        deadline = time.time() + timeout
        with self._cv:
            idx = start
            while True:
                while idx < len(self.lines):
                    if rx.search(self.lines[idx]):
                        return self.lines[idx]
                    idx += 1
                left = deadline - time.time()
                if left <= 0 or (self.popen.poll() is not None and idx >= len(self.lines)):
                    raise TimeoutError(f"{self.name}: no line matching {pattern!r} within {timeout}s; "
                                       f"exit={self.popen.poll()} log tail:\n" + "\n".join(self.lines[-30:]))
                self._cv.wait(min(left, 0.2))

    def count(self, pattern: str) -> int:
        rx = re.compile(pattern)
        with self._cv:
            return sum(1 for l in self.lines if rx.search(l))

    def text(self) -> str:
        with self._cv:
            return "\n".join(self.lines)

    def stop(self, timeout: float = 5.0):
        if self.popen.poll() is None:
            self.popen.send_signal(signal.SIGTERM)
            try:
                self.popen.wait(timeout)
            except subprocess.TimeoutExpired:
                self.popen.kill()
                self.popen.wait()

    def cpu_s(self) -> float:
        """User + system CPU seconds the process has used so far (all threads)."""
        try:
            with open(f"/proc/{self.popen.pid}/stat") as f:
                fields = f.read().rsplit(")", 1)[1].split()
            return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")
        except (OSError, IndexError, ValueError):
            return 0.0

    def kill(self):
        if self.popen.poll() is None:
            self.popen.kill()
            self.popen.wait()


def fault_env(**kw) -> dict:
    """The datagram-path fault injector's environment (native/rtc/ice.cc):
    fault_env(drop=0.02, dup=0.05, delay_ms=8, rtt_ms=20, rate_mbps=100,
    queue_kb=256, blackhole="3000:4000") -> {"TUNNEL_FAULT": "drop=0.02,..."}."""
    return {"TUNNEL_FAULT": ",".join(f"{k}={v}" for k, v in kw.items())}


def spawn(name: str, argv: list[str], env: dict | None = None) -> Proc:
    e = dict(os.environ)
    e.setdefault("RUST_LOG", "info")
    if env:
        e.update(env)
    p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=e)
    proc = Proc(name, p)
    threading.Thread(target=proc._pump, daemon=True).start()
    return proc


def start_signal(port: int | None = None) -> tuple[Proc, int]:
    port = port or free_port()
    p = spawn("signal", [binary("tunnel-signal"), "--listen", f"127.0.0.1:{port}"])
    p.wait_for(r"\[signal\] listening on", 10)
    return p, port


def start_serve(room: str, upstream: str, signal_port: int | None = None, extra: list[str] | None = None,
                env: dict | None = None, transport: str | None = None) -> Proc:
    argv = [binary("tunnel"), "serve", "--room", room, "--upstream", upstream, "--stun", "none"]
    if signal_port:
        argv += ["--signal", f"ws://127.0.0.1:{signal_port}"]
    if transport:
        argv += ["--transport", transport]
    return spawn("serve", argv + (extra or []), env)


def start_proxy(room: str, listen: str, signal_port: int | None = None, extra: list[str] | None = None,
                env: dict | None = None, transport: str | None = None) -> Proc:
    argv = [binary("tunnel"), "proxy", "--room", room, "--listen", listen, "--stun", "none"]
    if signal_port:
        argv += ["--signal", f"ws://127.0.0.1:{signal_port}"]
    if transport:
        argv += ["--transport", transport]
    return spawn("proxy", argv + (extra or []), env)


class Tunnel:
    """signal server + serve + proxy for one upstream; use as a context manager."""

    def __init__(self, upstream: str, transport: str = "webrtc", serve_extra=None, proxy_extra=None,
                 env: dict | None = None, advertise: str | None = None, room: str | None = None):
        self.upstream = upstream
        self.transport = transport
        self.serve_extra = list(serve_extra or [])
        self.proxy_extra = list(proxy_extra or [])
        if advertise:
            self.serve_extra += ["--advertise", advertise]
        self.env = env
        self.room = room or f"room-{os.getpid()}-{time.time_ns()}"
        self.procs: list[Proc] = []
        self.signal = self.serve = self.proxy = None
        self.proxy_port = free_port()

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.proxy_port}"

    def start(self, timeout: float = 30.0) -> "Tunnel":
        if self.transport == "webrtc":
            self.signal, sp = start_signal()
            self.procs.append(self.signal)
            st = pt = None
        else:
            sp = None
            port = free_port()
            st, pt = f"tcp-listen:127.0.0.1:{port}", f"tcp-connect:127.0.0.1:{port}"
        self.serve = start_serve(self.room, self.upstream, sp, self.serve_extra, self.env, st)
        self.procs.append(self.serve)
        if st:
            self.serve.wait_for("tcp transport: listening", timeout)
        self.proxy = start_proxy(self.room, f"127.0.0.1:{self.proxy_port}", sp, self.proxy_extra, self.env, pt)
        self.procs.append(self.proxy)
        self.serve.wait_for("tunnel ready", timeout)
        self.proxy.wait_for("proxy listening", timeout)
        return self

    def stop(self):
        for p in reversed(self.procs):
            p.stop()

    def __enter__(self):
        # A start that fails (a side never ready) stops what it started: a
        # `with` body that never ran gets no __exit__.
        try:
            return self.start()
        except BaseException:
            self.stop()
            raise

    def __exit__(self, *exc):
        self.stop()
