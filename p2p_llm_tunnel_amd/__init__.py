"""p2p_llm_tunnel_amd — a from-scratch P2P HTTP tunnel for exposing an LLM
inference endpoint on an MI355X node, with the capabilities of
michaelneale/p2p-llm-tunnel (``tunnel serve`` / ``tunnel proxy``, the
room-based WebSocket signal server, and the ``[type:u8][stream_id:u32]``
frame protocol over a WebRTC data channel).

Layout:
  native/                C++ core (reactor, HTTP, WebSocket, STUN/ICE, DTLS,
                         SCTP, DCEP, SDP, tunnel roles, signal server)
  p2p_llm_tunnel_amd/    Python harness: bindings (``_native``), process
                         fixtures, mock upstreams, benchmark driver, and the
                         on-node GPU inference upstream (``models``/``ops``)
"""
from __future__ import annotations

import importlib
import os

__version__ = "0.2.0"

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_ROOT = os.path.dirname(PKG_DIR)
# P2PT_BIN_DIR points the harness at another build (e.g. build-asan/bin to run
# the end-to-end suite against sanitizer binaries).
BIN_DIR = os.path.abspath(os.environ.get("P2PT_BIN_DIR") or os.path.join(REPO_ROOT, "build", "bin"))


def native():
    """Import the compiled core bindings, failing loudly if they are missing."""
    try:
        return importlib.import_module("p2p_llm_tunnel_amd._native")
    except ImportError as e:  # pragma: no cover - exercised when unbuilt
        raise ImportError(
            "p2p_llm_tunnel_amd._native is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `cmake -S . -B build -G Ninja && ninja -C build`"
        ) from e


def binary(name: str) -> str:
    """Path of a native executable (``tunnel`` / ``tunnel-signal``)."""
    p = os.path.join(BIN_DIR, name)
    if not os.path.exists(p):
        raise FileNotFoundError(f"{p} not built; run the native build first")
    return p
