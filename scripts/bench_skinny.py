#!/usr/bin/env python3
"""Skinny-GEMM (decode projection) microbenchmark on one GPU.

    python scripts/bench_skinny.py [--reps 200]

For each decode-shaped projection (M rows <= 16; weights [N, K] bf16) and each
waves-per-block / column-subtile choice, times `reps` back-to-back launches of
decode_fused.hip's k_skinny (plain store epilogue) with HIP events and prints
µs per launch and the weight-stream bandwidth. Reference: a device-to-device
copy of the same weight tensor (read + write) for the achievable HBM rate.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2p_llm_tunnel_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--m", type=int, default=8)
    ap.add_argument("--attn", action="store_true", help="time the decode attention kernel instead")
    a = ap.parse_args()
    if a.attn:
        return attn(a)
    lib = ops.lib()
    vp, i = ctypes.c_void_p, ctypes.c_int
    lib.p2pt_skinny_bench.argtypes = [vp, vp, vp, i, i, i, i, i, i, vp]
    lib.p2pt_skinny_bench.restype = ctypes.c_int
    shapes = {"qkv_small": (3072, 2048), "o_small": (2048, 2048), "gate_up_small": (11264, 2048),
              "down_small": (2048, 5632), "lm_head": (32000, 2048), "o_tiny": (1024, 1024)}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rows = []
    for name, (N, K) in shapes.items():
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(a.m, K, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(a.m, N, device="cuda", dtype=torch.bfloat16)
        cp = torch.empty_like(w)
        for _ in range(3):
            cp.copy_(w)
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(20):
            cp.copy_(w)
        ev1.record()
        torch.cuda.synchronize()
        copy_us = ev0.elapsed_time(ev1) * 1e3 / 20
        for nw in (4, 8, 16):
            for tn in (1, 2):
                if N % (16 * tn):
                    continue
                st = torch.cuda.current_stream().cuda_stream
                args = (x.data_ptr(), w.data_ptr(), out.data_ptr(), a.m, N, K, nw, tn)
                if lib.p2pt_skinny_bench(*args, 5, st):
                    continue
                torch.cuda.synchronize()
                ev0.record()
                lib.p2pt_skinny_bench(*args, a.reps, st)
                ev1.record()
                torch.cuda.synchronize()
                us = ev0.elapsed_time(ev1) * 1e3 / a.reps
                ref = (x.float() @ w.float().T)
                err = (out.float() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
                rows.append({"shape": name, "N": N, "K": K, "M": a.m, "nw": nw, "tn": tn, "us": round(us, 2),
                             "TBps": round(N * K * 2 / us / 1e6, 2), "copy_us": round(copy_us, 2),
                             "copy_TBps_rw": round(2 * N * K * 2 / copy_us / 1e6, 2), "rel_err": round(err, 5)})
                print(json.dumps(rows[-1]), flush=True)


def attn(a):
    """Decode attention alone: K/V bytes per launch vs time, over batch and context."""
    lib = ops.lib()
    vp, i = ctypes.c_void_p, ctypes.c_int
    lib.p2pt_attn_bench.argtypes = [vp, vp, vp, vp, i, i, i, i, i, i, vp, vp, vp, vp, i, vp]
    lib.p2pt_attn_bench.restype = ctypes.c_int
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    H, Hkv, Smax = 16, 4, 4096
    for D in (128, 64):
        for B in (1, 8, 16):
            kc = torch.randn(B, Smax, Hkv, D, device="cuda", dtype=torch.bfloat16)
            vc = torch.randn_like(kc)
            q = torch.randn(B, H * D, device="cuda", dtype=torch.bfloat16)
            out = torch.empty_like(q)
            part_o = torch.empty(16 * H * (Smax // 64) * D, device="cuda", dtype=torch.float32)
            part_ml = torch.empty(16 * H * (Smax // 64) * 2, device="cuda", dtype=torch.float32)
            ctr = torch.zeros(16 * H, device="cuda", dtype=torch.int32)
            for ctx, ml in ((64, Smax), (64, 64), (256, Smax), (1024, Smax), (1024, 1024), (4000, Smax)):
                pos = torch.full((B,), ctx - 1, device="cuda", dtype=torch.int32)
                st = torch.cuda.current_stream().cuda_stream
                args = (q.data_ptr(), kc.data_ptr(), vc.data_ptr(), pos.data_ptr(), B, H, Hkv, D, Smax, ml,
                        part_o.data_ptr(), part_ml.data_ptr(), ctr.data_ptr(), out.data_ptr())
                assert lib.p2pt_attn_bench(*args, 3, st) == 0
                torch.cuda.synchronize()
                ev0.record()
                lib.p2pt_attn_bench(*args, a.reps, st)
                ev1.record()
                torch.cuda.synchronize()
                us = ev0.elapsed_time(ev1) * 1e3 / a.reps
                kv = B * ctx * Hkv * D * 2 * 2
                # reference for the last launch
                qf = q.float().view(B, Hkv, H // Hkv, D) / D ** 0.5
                kf = kc[:, :ctx].float().permute(0, 2, 1, 3)
                vf = vc[:, :ctx].float().permute(0, 2, 1, 3)
                p = torch.softmax(qf @ kf.transpose(-1, -2), -1)
                ref = (p @ vf).reshape(B, H * D)
                err = (out.float() - ref).abs().max().item()
                print(json.dumps({"attn_D": D, "B": B, "ctx": ctx, "max_len": ml, "us": round(us, 2), "kv_MB": round(kv / 1e6, 2),
                                  "TBps": round(kv / us / 1e6, 2), "max_abs_err": round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
