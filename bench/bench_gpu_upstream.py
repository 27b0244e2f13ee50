#!/usr/bin/env python3
"""End-to-end: the tunnel in front of the on-node GPU inference endpoint.

BASELINE.json config #2 with a real upstream instead of a mock: `tunnel serve`
fronts `p2p_llm_tunnel_amd.models.server` (random-init Llama-style model on
the gfx950 fused decode path, continuous batching with chunked prefill, one
hipGraph per step) and the native load generator streams chat completions
through `tunnel proxy` and, for the baseline, straight to the server.

    python bench/bench_gpu_upstream.py [--config tiny | --checkpoint DIR] [--streams 1,8,16] [--max-tokens 32]

Prints one JSON document: per stream count, direct and tunneled req/s,
generated tokens/s, p50/p99 time to first token, and the added p50 TTFT.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from p2p_llm_tunnel_amd import binary  # noqa: E402
from p2p_llm_tunnel_amd.utils.build import ensure_native  # noqa: E402
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, spawn  # noqa: E402


def loadgen(port, streams, steps, body, warmup=1):
    # --warm-conns 1: the warmup runs on the timed keep-alive connections, so
    # connection setup stays out of the timed steps for both paths (a burst of
    # 32+ fresh connections to the Python endpoint costs its first step
    # 130-210 ms on the MI355X box; serve's upstream pool is connected ahead).
    out = subprocess.run([binary("tunnel-loadgen"), "--target", f"127.0.0.1:{port}", "--streams", str(streams),
                          "--steps", str(steps), "--warmup", str(warmup), "--path", "/v1/chat/completions",
                          "--body", body, "--warm-conns", "1"], capture_output=True, text=True, timeout=900)
    try:
        return json.loads(out.stdout.strip().splitlines()[-1])
    except (IndexError, ValueError):
        raise RuntimeError(f"loadgen failed (rc={out.returncode}): {out.stdout[-500:]} {out.stderr[-500:]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="tiny")
    ap.add_argument("--checkpoint", default=None, help="serve this HF Llama checkpoint (models.server --checkpoint)")
    ap.add_argument("--max-batch", type=int, default=16)
    ap.add_argument("--streams", default="1,8,16")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--max-tokens", type=int, default=32)
    ap.add_argument("--prompt-bytes", type=int, default=200)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ensure_native()
    port = free_port()
    model = ["--checkpoint", a.checkpoint] if a.checkpoint else ["--config", a.config]
    srv = spawn("gpu-server", [sys.executable, "-m", "p2p_llm_tunnel_amd.models.server", "--port", str(port),
                               *model, "--max-batch", str(a.max_batch)])
    try:
        srv.wait_for("inference endpoint on", 300)
        body = json.dumps({"model": "p2pt", "stream": True, "max_tokens": a.max_tokens,
                           "messages": [{"role": "user", "content": "x" * a.prompt_bytes}]})
        rows = []
        counts = [int(x) for x in a.streams.split(",")]
        # Direct baselines first, with no tunnel attached.
        direct = {s: loadgen(port, s, a.steps, body) for s in counts}
        with Tunnel(f"http://127.0.0.1:{port}", transport=os.environ.get("P2PT_TRANSPORT", "webrtc")) as t:
            for s in counts:
                tr = loadgen(t.proxy_port, s, a.steps, body)
                dr = direct[s]
                row = {"streams": s, "max_tokens": a.max_tokens, "prompt_bytes": a.prompt_bytes,
                       "tunneled_req_s": tr["req_s"], "direct_req_s": dr["req_s"],
                       "tunneled_tok_s": tr["req_s"] * a.max_tokens, "direct_tok_s": dr["req_s"] * a.max_tokens,
                       "tunneled_p50_ttft_ms": tr["p50_ttft_ms"], "direct_p50_ttft_ms": dr["p50_ttft_ms"],
                       "added_p50_ttft_ms": round(tr["p50_ttft_ms"] - dr["p50_ttft_ms"], 3),
                       "tunneled_p99_ttft_ms": tr["p99_ttft_ms"], "direct_p99_ttft_ms": dr["p99_ttft_ms"],
                       "tunneled_p50_total_ms": tr["p50_total_ms"], "direct_p50_total_ms": dr["p50_total_ms"],
                       "errors": tr["errors"] + dr["errors"],
                       "tunneled_step_ms": tr.get("step_ms"), "direct_step_ms": dr.get("step_ms")}
                rows.append(row)
                print(json.dumps(row), file=sys.stderr, flush=True)
        doc = {"upstream": f"p2p_llm_tunnel_amd.models.server ({a.config}, fused gfx950 decode, hipGraph)",
               "time": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), "rows": rows}
        text = json.dumps(doc, indent=1)
        if a.out:
            with open(a.out, "w") as f:
                f.write(text + "\n")
        print(text)
    finally:
        srv.stop()


if __name__ == "__main__":
    main()
