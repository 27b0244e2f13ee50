"""A scriptable tunnel peer in pure Python, speaking the frame protocol over
the TCP debug transport (``--transport tcp-listen:/tcp-connect:``; each
message is ``[u32 length][frame]``). Used to pin the wire behaviour of the
native serve/proxy roles independently of the native codec.
"""
from __future__ import annotations

import json
import socket
import struct
import time

HELLO, AGREE, PING, PONG = 1, 2, 3, 4
REQ_HEADERS, REQ_BODY, REQ_END, CANCEL, CREDIT = 10, 11, 12, 13, 14
RES_HEADERS, RES_BODY, RES_END, ERROR = 20, 21, 22, 99


def frame(t: int, sid: int, payload: bytes = b"") -> bytes:
    return struct.pack(">BI", t, sid) + payload


class FramePeer:
    def __init__(self, sock: socket.socket):
        self.s = sock
        self.s.settimeout(10)
        self.buf = b""

    @classmethod
    def connect(cls, port: int, timeout: float = 10.0) -> "FramePeer":
        deadline = time.time() + timeout
        while True:
            try:
                return cls(socket.create_connection(("127.0.0.1", port), timeout=2))
            except OSError:
                if time.time() > deadline:
                    raise
                time.sleep(0.05)

    @classmethod
    def listen(cls, port: int = 0):
        srv = socket.socket()
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind(("127.0.0.1", port))
        srv.listen(1)
        return srv

    def send_raw(self, msg: bytes):
        self.s.sendall(struct.pack(">I", len(msg)) + msg)

    def send(self, t: int, sid: int, payload: bytes = b""):
        self.send_raw(frame(t, sid, payload))

    def send_json(self, t: int, sid: int, obj):
        self.send(t, sid, json.dumps(obj).encode())

    def recv(self, timeout: float = 10.0):
        self.s.settimeout(timeout)
        while len(self.buf) < 4 or len(self.buf) < 4 + struct.unpack(">I", self.buf[:4])[0]:
            d = self.s.recv(65536)
            if not d:
                raise EOFError("peer closed")
            self.buf += d
        n = struct.unpack(">I", self.buf[:4])[0]
        msg, self.buf = self.buf[4:4 + n], self.buf[4 + n:]
        t, sid = struct.unpack(">BI", msg[:5])
        return t, sid, msg[5:]

    def recv_until(self, pred, timeout: float = 10.0, skip_pings: bool = True):
        deadline = time.time() + timeout
        while True:
            t, sid, p = self.recv(max(0.05, deadline - time.time()))
            if skip_pings and t in (PING, PONG):
                if t == PING:
                    self.send(PONG, 0)
                continue
            if pred(t, sid, p):
                return t, sid, p

    def closed(self, timeout: float = 5.0) -> bool:
        try:
            self.recv_until(lambda *a: False, timeout)
        except EOFError:
            return True
        except (socket.timeout, TimeoutError):
            return False
        return False

    def close(self):
        self.s.close()
