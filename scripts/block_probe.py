"""Probe of the persistent O/gate-up/down block (P2PT_DECODE_BLOCK): one
eager decode step of the small config, then the k_block counters read back
from the workspace (queue head, exits, per-phase arrivals, wait time-outs).
After a completed launch the counters are zero and the time-outs count the
dependency waits that gave up.

    P2PT_DECODE_BLOCK=256 P2PT_DECODE_BLOCK_WAIT=4096 python scripts/block_probe.py
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2p_llm_tunnel_amd import ops  # noqa: E402
from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama  # noqa: E402


def main():
    m = TinyLlama("small", device="cuda", max_batch=1, seed=11, fused=True)
    dec = m.fused_decoder()
    lib = ops.lib()
    lib.p2pt_llama_block_ctr_offset.argtypes = [ctypes.POINTER(ops.LlamaDims)]
    lib.p2pt_llama_block_ctr_offset.restype = ctypes.c_size_t
    off = lib.p2pt_llama_block_ctr_offset(ctypes.byref(dec.dims))
    tok = torch.randint(0, m.cfg.vocab, (1,), device="cuda")
    for step in range(3):
        pos = torch.full((1,), 10 + step, dtype=torch.int32, device="cuda")
        t0 = time.perf_counter()
        m.decode_step(tok, pos, (10 + step, 10 + step))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        c = dec.ws[off:off + 33 * 4].view(torch.int32).cpu().tolist()
        print(f"step {step}: {dt * 1e3:.2f} ms; queue {c[0]} exits {c[1]} arrivals {c[8:16]} {c[16:24]} {c[24:32]} "
              f"wait time-outs {c[32]}", flush=True)


if __name__ == "__main__":
    main()
