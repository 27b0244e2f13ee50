"""Minimal TURN server (RFC 8656, UDP relays, long-term credentials) for tests.

Independent of the native code: the STUN codec here is written in Python so
the native TURN client (native/rtc/turn.cc) is checked against a separate
implementation. Supports Allocate (401 challenge -> authenticated), Refresh
(incl. LIFETIME 0), CreatePermission, ChannelBind, Send/Data indications and
ChannelData in both directions.

Clients reach it over UDP (default), TCP (transport="tcp": turn:...?transport=tcp)
or TLS (transport="tls" with an ssl.SSLContext: turns:...); over a stream,
STUN messages and ChannelData (padded to 4 bytes) are framed back to back
(RFC 8656 §12.5) and each connection is its own allocation. Relays to peers
are UDP in every case.

Shared bottleneck (``link=Link(...)``): everything the server relays towards
peers leaves through ONE emulated link — a rate, a drop-tail queue, a one-way
delay and Bernoulli loss — and everything relayed back to clients through a
second one (same delay; rate and queue only if given). Every tunnel relayed
through one server therefore competes for the same queue, which the
per-agent WAN emulator in native/rtc/ice.cc (one emulator per ICE agent)
cannot model: that is what the congestion response's fairness is measured on
(bench/bench_fairness.py).
"""
from __future__ import annotations

import hashlib
import heapq
import hmac
import os
import random
import select
import socket
import struct
import threading
import time
import zlib

MAGIC = 0x2112A442


def _pad(n):
    return (4 - n % 4) % 4


def parse(data: bytes):
    if len(data) < 20 or data[0] >= 4:
        return None
    t, ln, magic = struct.unpack(">HHI", data[:8])
    if magic != MAGIC or 20 + ln > len(data):
        return None
    tid = data[8:20]
    attrs, off, mi_off = [], 20, None
    while off + 4 <= 20 + ln:
        at, al = struct.unpack(">HH", data[off:off + 4])
        if at == 0x0008:
            mi_off = off
        attrs.append((at, data[off + 4:off + 4 + al]))
        off += 4 + al + _pad(al)
    return t, tid, attrs, mi_off


def build(t, tid, attrs, key=None, fingerprint=True):
    body = b"".join(struct.pack(">HH", a, len(v)) + v + b"\0" * _pad(len(v)) for a, v in attrs)
    if key is not None:
        hdr = struct.pack(">HHI", t, len(body) + 24, MAGIC) + tid
        mac = hmac.new(key, hdr + body, hashlib.sha1).digest()
        body += struct.pack(">HH", 0x0008, 20) + mac
    if fingerprint:
        hdr = struct.pack(">HHI", t, len(body) + 8, MAGIC) + tid
        crc = (zlib.crc32(hdr + body) ^ 0x5354554E) & 0xFFFFFFFF
        body += struct.pack(">HHI", 0x8028, 4, crc)
    return struct.pack(">HHI", t, len(body), MAGIC) + tid + body


def xor_addr(host: str, port: int) -> bytes:
    ip = struct.unpack(">I", socket.inet_aton(host))[0] ^ MAGIC
    return struct.pack(">BBHI", 0, 1, port ^ (MAGIC >> 16), ip)


def unxor_addr(v: bytes):
    _, fam, xp, xi = struct.unpack(">BBHI", v[:8])
    return socket.inet_ntoa(struct.pack(">I", xi ^ MAGIC)), xp ^ (MAGIC >> 16)


def frames(buf: bytearray):
    """Complete STUN / ChannelData messages at the front of a stream buffer
    (consumed from it)."""
    out = []
    while len(buf) >= 4:
        if 0x40 <= buf[0] <= 0x7F:
            n = (4 + struct.unpack(">H", buf[2:4])[0] + 3) & ~3
        elif buf[0] < 4:
            n = 20 + struct.unpack(">H", buf[2:4])[0]
        else:
            raise ValueError("stream out of sync")
        if len(buf) < n:
            break
        out.append(bytes(buf[:n]))
        del buf[:n]
    return out


class Link:
    """One direction of an emulated bottleneck: serialisation at ``rate_mbps``
    (0 = unlimited) into a drop-tail queue of ``queue_kb``, then ``delay_ms``
    of propagation; each packet is lost with probability ``loss``. Packets
    wait in a heap until their delivery time (the server's loop sends them)."""

    def __init__(self, rate_mbps=0.0, delay_ms=0.0, queue_kb=0, loss=0.0, seed=1):
        self.rate = rate_mbps * 1e6 / 8  # bytes/s
        self.delay = delay_ms / 1e3
        self.queue = queue_kb * 1024 if queue_kb else (int(self.rate * 0.05) if self.rate else 0)  # default 50 ms
        self.loss = loss
        self.rng = random.Random(seed)
        self.free_at = 0.0  # when the link finishes serialising what it holds
        self.heap = []
        self.seq = 0
        self.stats = {"packets": 0, "bytes": 0, "queue_drops": 0, "loss_drops": 0, "max_queue_bytes": 0}

    def reverse(self):
        return Link(0.0, self.delay * 1e3, 0, 0.0)

    def submit(self, data, send, now=None):
        now = time.monotonic() if now is None else now
        n = len(data)
        if self.loss and self.rng.random() < self.loss:
            self.stats["loss_drops"] += 1
            return
        if self.rate:
            backlog = max(0.0, self.free_at - now) * self.rate
            if backlog + n > self.queue:
                self.stats["queue_drops"] += 1
                return
            self.stats["max_queue_bytes"] = max(self.stats["max_queue_bytes"], int(backlog + n))
            self.free_at = max(now, self.free_at) + n / self.rate
            at = self.free_at + self.delay
        else:
            at = now + self.delay
        self.stats["packets"] += 1
        self.stats["bytes"] += n
        if at <= now:
            send(data)
            return
        self.seq += 1
        heapq.heappush(self.heap, (at, self.seq, data, send))

    def due(self, now):
        """Sends what is due; returns the time of the next packet (or None)."""
        h = self.heap
        while h and h[0][0] <= now:
            _, _, data, send = heapq.heappop(h)
            send(data)
        return h[0][0] if h else None


class TurnServer:
    def __init__(self, user="user", password="pass", realm="p2pt.test", host="127.0.0.1", transport="udp",
                 ssl_ctx=None, link: Link | None = None, back: Link | None = None):
        self.user, self.password, self.realm = user, password, realm
        self.key = hashlib.md5(f"{user}:{realm}:{password}".encode()).digest()
        self.nonce = os.urandom(8).hex().encode()
        self.transport, self.ssl_ctx = transport, ssl_ctx
        self.host = host
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)  # UDP clients (transport "udp")
        self.lsock = None
        if transport == "udp":
            self.sock.bind((host, 0))
            self.port = self.sock.getsockname()[1]
        else:
            self.lsock = socket.create_server((host, 0))
            self.port = self.lsock.getsockname()[1]
        self.conns = {}      # stream connection -> (key, rx buffer)
        self.conn_of = {}    # key -> stream connection
        self.peer_of = {}    # key -> the client's (ip, port) as seen by the server
        self.allocs = {}     # client key -> dict(relay=sock, perms=set(ip), chans={num: peer}, peers={peer: num})
        self.by_relay = {}   # relay sock -> client key
        self.stats = {"bindings": 0, "allocations": 0, "relayed_to_peer": 0, "relayed_to_client": 0, "channel_binds": 0,
                      "stream_connections": 0}
        self._stop = False
        self.link = link  # towards peers (the shared bottleneck)
        self.back = back if back is not None else (link.reverse() if link is not None else None)
        self.thread = threading.Thread(target=self._run, daemon=True)

    def _to_peer(self, relay, data, peer):
        if self.link is None:
            relay.sendto(data, peer)
        else:
            self.link.submit(data, lambda d, r=relay, p=peer: self._sendto(r, d, p))

    @staticmethod
    def _sendto(sock, data, addr):
        try:
            sock.sendto(data, addr)
        except OSError:
            pass

    @property
    def url(self):
        if self.transport == "tcp":
            return f"turn:{self.host}:{self.port}?transport=tcp"
        if self.transport == "tls":
            return f"turns:{self.host}:{self.port}"
        return f"turn:{self.host}:{self.port}"

    def _send(self, data, addr):
        c = self.conn_of.get(addr)
        if c is not None:
            try:
                c.sendall(data)
            except OSError:
                pass
        else:
            self.sock.sendto(data, addr)

    def _accept(self):
        try:
            c, peer = self.lsock.accept()
        except OSError:
            return
        try:
            if self.ssl_ctx is not None:
                c.settimeout(5)
                c = self.ssl_ctx.wrap_socket(c, server_side=True)
            c.settimeout(5)
        except OSError:
            c.close()
            return
        key = ("stream", self.stats["stream_connections"])
        self.stats["stream_connections"] += 1
        self.conns[c] = (key, bytearray())
        self.conn_of[key] = c
        self.peer_of[key] = peer

    def _drop_conn(self, c):
        key, _ = self.conns.pop(c)
        self.conn_of.pop(key, None)
        a = self.allocs.pop(key, None)
        if a:
            self.by_relay.pop(a["relay"], None)
            a["relay"].close()
        c.close()

    def _read_conn(self, c):
        key, buf = self.conns[c]
        try:
            d = c.recv(65536)
            while d and getattr(c, "pending", lambda: 0)():
                d += c.recv(65536)
        except (OSError, ValueError):
            d = b""
        if not d:
            self._drop_conn(c)
            return
        buf += d
        try:
            msgs = frames(buf)
        except ValueError:
            self._drop_conn(c)
            return
        for m in msgs:
            self._handle_client(m, key)

    def start(self):
        self.thread.start()
        return self

    def stop(self):
        self._stop = True
        self.thread.join(timeout=2)
        for a in self.allocs.values():
            a["relay"].close()
        for c in list(self.conns):
            c.close()
        if self.lsock is not None:
            self.lsock.close()
        self.sock.close()

    # ------------------------------------------------------------------
    def _auth_ok(self, data, attrs, mi_off):
        d = dict(attrs)
        if mi_off is None or d.get(0x0006) != self.user.encode() or d.get(0x0014) != self.realm.encode():
            return False
        hdr = bytearray(data[:mi_off])
        struct.pack_into(">H", hdr, 2, mi_off - 20 + 24)
        mac = hmac.new(self.key, bytes(hdr), hashlib.sha1).digest()
        return mac == data[mi_off + 4:mi_off + 24]

    def _err(self, t, tid, code, reason, addr):
        v = struct.pack(">HBB", 0, code // 100, code % 100) + reason.encode()
        attrs = [(0x0009, v), (0x0014, self.realm.encode()), (0x0015, self.nonce)]
        self._send(build(t | 0x0110, tid, attrs), addr)

    def _handle_client(self, data, addr):
        if 0x40 <= data[0] <= 0x7F:  # ChannelData
            ch, ln = struct.unpack(">HH", data[:4])
            a = self.allocs.get(addr)
            if a and ch in a["chans"]:
                self._to_peer(a["relay"], data[4:4 + ln], a["chans"][ch])
                self.stats["relayed_to_peer"] += 1
            return
        m = parse(data)
        if not m:
            return
        t, tid, attrs, mi_off = m
        method = t & 0x3EEF
        d = dict(attrs)
        if t == 0x0016:  # Send indication
            a = self.allocs.get(addr)
            if a and 0x0012 in d and 0x0013 in d:
                peer = unxor_addr(d[0x0012])
                if peer[0] in a["perms"]:
                    self._to_peer(a["relay"], d[0x0013], peer)
                    self.stats["relayed_to_peer"] += 1
            return
        if t & 0x0110:  # not a request
            return
        if method == 0x0001:  # Binding
            self.stats["bindings"] += 1
            self._send(build(0x0101, tid, [(0x0020, xor_addr(*self.peer_of.get(addr, addr)))]), addr)
            return
        if not self._auth_ok(data, attrs, mi_off):
            self._err(method, tid, 401, "Unauthorized", addr)
            return
        if method == 0x0003:  # Allocate
            if addr in self.allocs:
                self._err(method, tid, 437, "Allocation Mismatch", addr)
                return
            r = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
            r.bind((self.host, 0))
            self.allocs[addr] = {"relay": r, "perms": set(), "chans": {}, "peers": {}}
            self.by_relay[r] = addr
            self.stats["allocations"] += 1
            rh, rp = r.getsockname()
            self._send(build(0x0103, tid, [(0x0016, xor_addr(rh, rp)), (0x0020, xor_addr(*self.peer_of.get(addr, addr))),
                                            (0x000D, struct.pack(">I", 600))], self.key), addr)
        elif method == 0x0004:  # Refresh
            lt = struct.unpack(">I", d.get(0x000D, b"\0\0\x02\x58"))[0]
            if lt == 0 and addr in self.allocs:
                a = self.allocs.pop(addr)
                self.by_relay.pop(a["relay"], None)
                a["relay"].close()
            self._send(build(0x0104, tid, [(0x000D, struct.pack(">I", lt))], self.key), addr)
        elif method == 0x0008:  # CreatePermission
            a = self.allocs.get(addr)
            if a and 0x0012 in d:
                a["perms"].add(unxor_addr(d[0x0012])[0])
            self._send(build(0x0108, tid, [], self.key), addr)
        elif method == 0x0009:  # ChannelBind
            a = self.allocs.get(addr)
            ch = struct.unpack(">H", d[0x000C][:2])[0]
            peer = unxor_addr(d[0x0012])
            a["chans"][ch] = peer
            a["peers"][peer] = ch
            a["perms"].add(peer[0])
            self.stats["channel_binds"] += 1
            self._send(build(0x0109, tid, [], self.key), addr)

    def _handle_relay(self, r):
        for _ in range(64):  # drain what is queued on the relay socket
            try:
                data, peer = r.recvfrom(65536, socket.MSG_DONTWAIT)
            except OSError:
                return
            self._relay_one(r, data, peer)

    def _relay_one(self, r, data, peer):
        client = self.by_relay.get(r)
        a = self.allocs.get(client)
        if not a or peer[0] not in a["perms"]:
            return
        ch = a["peers"].get(peer)
        if ch:
            msg = struct.pack(">HH", ch, len(data)) + data + b"\0" * _pad(len(data))
        else:
            msg = build(0x0017, os.urandom(12), [(0x0012, xor_addr(*peer)), (0x0013, data)], fingerprint=False)
        if self.back is None:
            self._send(msg, client)
        else:
            self.back.submit(msg, lambda m, c=client: self._send(m, c))
        self.stats["relayed_to_client"] += 1

    def _run(self):
        while not self._stop:
            socks = [self.sock] + list(self.by_relay) + list(self.conns) + ([self.lsock] if self.lsock else [])
            timeout = 0.1
            if self.link is not None:
                now = time.monotonic()
                nxt = [t for t in (self.link.due(now), self.back.due(now)) if t is not None]
                if nxt:
                    timeout = max(0.0, min(nxt) - now)
            try:
                ready, _, _ = select.select(socks, [], [], timeout)
            except (OSError, ValueError):
                continue
            for s in ready:
                if s is self.lsock:
                    self._accept()
                elif s in self.conns:
                    self._read_conn(s)
                elif s is self.sock:
                    for _ in range(64):  # drain what is queued
                        try:
                            data, addr = s.recvfrom(65536, socket.MSG_DONTWAIT)
                        except OSError:
                            break
                        self._handle_client(data, addr)
                else:
                    self._handle_relay(s)
