"""Diagnostic: per-step durations of the GPU endpoint at 16 streams, direct and
through the tunnel (the direct 16-stream row of bench_gpu_upstream.py runs at
about half the tunneled rate with a ~200 ms p99 TTFT outlier)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from p2p_llm_tunnel_amd import binary  # noqa: E402
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, spawn  # noqa: E402


def lg(port, streams, steps, body, warmup=1):
    out = subprocess.run([binary("tunnel-loadgen"), "--target", f"127.0.0.1:{port}", "--streams", str(streams),
                          "--steps", str(steps), "--warmup", str(warmup), "--path", "/v1/chat/completions",
                          "--body", body], capture_output=True, text=True, timeout=300)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    return {k: d[k] for k in ("req_s", "p50_ttft_ms", "p99_ttft_ms", "step_ms", "errors")}


def main():
    port = free_port()
    srv = spawn("gpu-server", [sys.executable, "-m", "p2p_llm_tunnel_amd.models.server", "--port", str(port),
                               "--config", "tiny", "--max-batch", "16"])
    try:
        srv.wait_for("inference endpoint on", 300)
        body = json.dumps({"model": "p2pt", "stream": True, "max_tokens": 32,
                           "messages": [{"role": "user", "content": "x" * 200}]})
        print("direct 16 (cold)", lg(port, 16, 6, body), flush=True)
        print("direct 16 (again)", lg(port, 16, 6, body), flush=True)
        print("direct 16 warmup 0", lg(port, 16, 6, body, warmup=0), flush=True)
        with Tunnel(f"http://127.0.0.1:{port}", transport="webrtc") as t:
            print("tunneled 16", lg(t.proxy_port, 16, 6, body), flush=True)
            print("direct 16 (tunnel up)", lg(port, 16, 6, body), flush=True)
        print("direct 8", lg(port, 8, 6, body), flush=True)
    finally:
        srv.stop()


if __name__ == "__main__":
    main()
