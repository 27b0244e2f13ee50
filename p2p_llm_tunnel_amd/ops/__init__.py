"""Python front-end for the gfx950 HIP kernels (``kernels.hip``).

The kernels are compiled in-tree into ``_hip_ops.so`` (see ``build.py``) and
called through ctypes on the current torch stream. Every wrapper validates
shapes, dtypes, devices and contiguity on the host *before* launching, so a
mismatched tensor raises instead of faulting the GPU. There is no silent
PyTorch fallback: if the library is missing on a GPU host, ``lib()`` raises.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class LlamaDims(ctypes.Structure):
    """Mirror of ``LlamaDims`` in decode_fused.hip."""
    _fields_ = [(n, ctypes.c_int) for n in ("vocab", "dim", "n_layers", "H", "Hkv", "D", "ffn", "max_seq",
                                           "max_batch")] + [("eps", ctypes.c_float), ("theta", ctypes.c_float)]


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        # P2PT_HIP_OPS_LIB: another in-tree build of the same kernels (A/B runs on one box).
        path = os.path.join(HERE, os.environ.get("P2PT_HIP_OPS_LIB", "_hip_ops.so"))
        if not os.path.exists(path):
            from . import build as _b
            _b.build()
        _LIB = ctypes.CDLL(path)
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        _LIB.p2pt_rmsnorm.argtypes = [vp, vp, vp, vp, vp, i, i, f, vp]
        _LIB.p2pt_silu_mul.argtypes = [vp, vp, i, i, vp]
        _LIB.p2pt_rope_qkv_cache.argtypes = [vp, vp, vp, vp, vp, i, i, i, i, i, f, vp]
        _LIB.p2pt_decode_attention.argtypes = [vp, vp, vp, vp, vp, vp, i, i, i, i, i, i, i, f, vp]
        _LIB.p2pt_argmax.argtypes = [vp, vp, i, i, vp]
        _LIB.p2pt_skinny_gemm.argtypes = [vp, vp, vp, i, i, i, vp]
        _LIB.p2pt_sample.argtypes = [vp, vp, vp, i, i, i, vp]
        _LIB.p2pt_llama_ws_bytes.argtypes = [ctypes.POINTER(LlamaDims)]
        _LIB.p2pt_llama_ws_bytes.restype = ctypes.c_size_t
        _LIB.p2pt_llama_decode.argtypes = [ctypes.POINTER(LlamaDims), ctypes.POINTER(vp), vp, vp, vp, vp, vp, i, i,
                                           i, vp, ctypes.c_size_t, vp, vp, vp]
        for fn in ("p2pt_rmsnorm", "p2pt_silu_mul", "p2pt_rope_qkv_cache", "p2pt_decode_attention", "p2pt_argmax",
                   "p2pt_skinny_gemm", "p2pt_llama_decode", "p2pt_sample"):
            getattr(_LIB, fn).restype = ctypes.c_int
    return _LIB



MAX_ROWS = 64  # token rows per fused step (decode_fused.hip kMaxM)

def loaded_path() -> str:
    lib()
    return os.path.join(HERE, "_hip_ops.so")


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _check(t: torch.Tensor, dtype, name: str, device=None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name} must be on a HIP device")
    if device is not None and t.device != device:
        raise ValueError(f"{name} on {t.device}, expected {device}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _ok(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what}: HIP launch failed (hipError {rc})")


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-6, residual: torch.Tensor | None = None):
    """out = rmsnorm(x [+ residual]) * weight. With a residual, returns (out, x + residual)."""
    _check(x, torch.bfloat16, "x")
    _check(weight, torch.bfloat16, "weight", x.device)
    hidden = x.shape[-1]
    if weight.shape != (hidden,):
        raise ValueError(f"weight shape {tuple(weight.shape)} != ({hidden},)")
    if hidden % 8 or hidden > 16384:
        raise ValueError("hidden must be a multiple of 8 and <= 16384")
    rows = x.numel() // hidden
    out = torch.empty_like(x)
    res_out = None
    if residual is not None:
        _check(residual, torch.bfloat16, "residual", x.device)
        if residual.shape != x.shape:
            raise ValueError("residual shape mismatch")
        res_out = torch.empty_like(x)
    _ok(lib().p2pt_rmsnorm(_p(x), _p(residual), _p(res_out), _p(weight), _p(out), rows, hidden, eps, _stream(x)),
        "rmsnorm")
    return out if residual is None else (out, res_out)


def silu_mul(gate_up: torch.Tensor) -> torch.Tensor:
    """[..., 2F] -> silu(gate) * up, [..., F]."""
    _check(gate_up, torch.bfloat16, "gate_up")
    two_f = gate_up.shape[-1]
    if two_f % 16:
        raise ValueError("last dim must be 2*F with F % 8 == 0")
    F = two_f // 2
    rows = gate_up.numel() // two_f
    out = torch.empty(*gate_up.shape[:-1], F, dtype=gate_up.dtype, device=gate_up.device)
    _ok(lib().p2pt_silu_mul(_p(gate_up), _p(out), rows, F, _stream(gate_up)), "silu_mul")
    return out


def rope_qkv_cache(qkv: torch.Tensor, pos: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                   n_heads: int, n_kv_heads: int, head_dim: int, theta: float = 10000.0,
                   pos_range: tuple[int, int] | None = None) -> torch.Tensor:
    """Apply RoPE to q and k of one new token per sequence and append k, v to the caches.

    qkv: [B, (H + 2*Hkv) * D]; pos: int32 [B]; caches: [B, Smax, Hkv, D]. Returns q [B, H, D].
    ``pos_range`` = host-known (min, max) of ``pos``; without it the bounds are
    read back from the device (a sync) before launch.
    """
    _check(qkv, torch.bfloat16, "qkv")
    _check(pos, torch.int32, "pos", qkv.device)
    _check(k_cache, torch.bfloat16, "k_cache", qkv.device)
    _check(v_cache, torch.bfloat16, "v_cache", qkv.device)
    B = qkv.shape[0]
    if qkv.shape != (B, (n_heads + 2 * n_kv_heads) * head_dim):
        raise ValueError(f"qkv shape {tuple(qkv.shape)} inconsistent with heads")
    if pos.shape != (B,):
        raise ValueError("pos must be [B]")
    Smax = k_cache.shape[1]
    if k_cache.shape != (B, Smax, n_kv_heads, head_dim) or v_cache.shape != k_cache.shape:
        raise ValueError(f"cache shape {tuple(k_cache.shape)} != ({B}, Smax, {n_kv_heads}, {head_dim})")
    if n_heads % n_kv_heads or head_dim % 2:
        raise ValueError("bad head config")
    pmin, pmax = pos_range if pos_range is not None else (int(pos.min().item()), int(pos.max().item()))
    if pmin < 0 or pmax >= Smax:
        raise ValueError(f"positions out of cache range [0, {Smax})")
    q = torch.empty(B, n_heads, head_dim, dtype=qkv.dtype, device=qkv.device)
    _ok(lib().p2pt_rope_qkv_cache(_p(qkv), _p(pos), _p(q), _p(k_cache), _p(v_cache), B, n_heads, n_kv_heads,
                                  head_dim, Smax, theta, _stream(qkv)), "rope_qkv_cache")
    return q


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, lens: torch.Tensor,
                     chunk: int = 64, max_len: int | None = None, scale: float | None = None) -> torch.Tensor:
    """Single-token GQA attention over the KV cache. q: [B, H, D]; lens: int32 [B] (>= 1).

    The sequence is split into `chunk`-token pieces, one workgroup each
    (B * Hkv * ceil(max_len / chunk) workgroups), so even batch-1 decode
    fills the 256 CUs. Splits past a sequence's length exit immediately, which
    lets a captured graph use max_len = cache capacity for every step.
    """
    _check(q, torch.bfloat16, "q")
    _check(k_cache, torch.bfloat16, "k_cache", q.device)
    _check(v_cache, torch.bfloat16, "v_cache", q.device)
    _check(lens, torch.int32, "lens", q.device)
    B, H, D = q.shape
    Smax, Hkv = k_cache.shape[1], k_cache.shape[2]
    if k_cache.shape != (B, Smax, Hkv, D) or v_cache.shape != k_cache.shape:
        raise ValueError("cache shape mismatch")
    if D not in (64, 128):
        raise ValueError("head_dim must be 64 or 128")
    if H % Hkv or H // Hkv > 8:
        raise ValueError("n_heads / n_kv_heads must be an integer <= 8")
    if lens.shape != (B,):
        raise ValueError("lens must be [B]")
    if max_len is None:
        max_len = int(lens.max().item())
        if int(lens.min().item()) < 1:
            raise ValueError("every sequence needs at least one cached token")
    if max_len > Smax:
        raise ValueError("lens exceed cache capacity")
    nsplit = max(1, math.ceil(max_len / chunk))
    ws = torch.empty(B * H * nsplit * (D + 2), dtype=torch.float32, device=q.device)
    out = torch.empty_like(q)
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    _ok(lib().p2pt_decode_attention(_p(q), _p(k_cache), _p(v_cache), _p(lens), _p(out), _p(ws), B, H, Hkv, D, Smax,
                                    nsplit, chunk, scale, _stream(q)), "decode_attention")
    return out


def argmax(logits: torch.Tensor) -> torch.Tensor:
    """Row-wise argmax (first index on ties) of bf16 logits [B, V] -> int64 [B]."""
    _check(logits, torch.bfloat16, "logits")
    if logits.dim() != 2:
        raise ValueError("logits must be [B, V]")
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.int64, device=logits.device)
    _ok(lib().p2pt_argmax(_p(logits), _p(out), B, V, _stream(logits)), "argmax")
    return out


def sample_(logits: torch.Tensor, ids: torch.Tensor, params: torch.Tensor) -> torch.Tensor:
    """In-place stochastic sampling (sample.hip): rows of bf16 ``logits`` [B, V]
    whose temperature is > 0 get ``ids[b]`` replaced by a draw from
    softmax(logits / T) after top-k and top-p filtering; greedy rows (T <= 0)
    keep the id already there. ``params``: int64 [5, >= B] (contiguous; column
    b for row b) — float32 bits of T, top_k (<= 0 off), float32 bits of top_p
    (>= 1 off), seed, counter (see ``pack_sampling``)."""
    _check(logits, torch.bfloat16, "logits")
    _check(ids, torch.int64, "ids", logits.device)
    _check(params, torch.int64, "params", logits.device)
    if logits.dim() != 2 or ids.shape != (logits.shape[0],) or params.dim() != 2 or params.shape[0] != 5:
        raise ValueError("need logits [B, V], ids [B], params [5, >= B]")
    B, V = logits.shape
    if params.shape[1] < B:
        raise ValueError("params need a column per row")
    _ok(lib().p2pt_sample(_p(logits), _p(ids), _p(params), B, params.shape[1], V, _stream(logits)), "sample")
    return ids


def f32_bits(x: float) -> int:
    """The float32 bit pattern of x as a non-negative int (the sampler's params encoding)."""
    import struct
    return struct.unpack("<I", struct.pack("<f", float(x)))[0]


def pack_sampling(temperature: float, top_k: int, top_p: float, seed: int, counter: int) -> list[int]:
    """One params column for ``sample_``."""
    return [f32_bits(temperature), int(top_k), f32_bits(top_p), int(seed) & 0x7FFFFFFFFFFFFFFF,
            int(counter) & 0x7FFFFFFFFFFFFFFF]


def skinny_gemm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """bf16(x @ w.T) for a few rows on MFMA (decode-shaped GEMM). x: [M<=64, K]; w: [N, K]."""
    _check(x, torch.bfloat16, "x")
    _check(w, torch.bfloat16, "w", x.device)
    if x.dim() != 2 or w.dim() != 2 or x.shape[1] != w.shape[1]:
        raise ValueError("shapes must be x [M, K], w [N, K]")
    M, K = x.shape
    N = w.shape[0]
    if not 1 <= M <= MAX_ROWS or N % 32 or K % 32:
        raise ValueError(f"need 1 <= M <= {MAX_ROWS}, N % 32 == 0, K % 32 == 0")
    out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    _ok(lib().p2pt_skinny_gemm(_p(x), _p(w), _p(out), M, N, K, _stream(x)), "skinny_gemm")
    return out


class FusedLlamaDecoder:
    """Host handle for the fused decode step (decode_fused.hip): 5 kernels per layer + 2.

    Holds the weight pointer table and a zero-initialised workspace; ``step``
    validates the per-call tensors and launches on the current stream (capturable
    into a hipGraph: no host sync, no allocation).
    """

    def __init__(self, dims: LlamaDims, weights: list, k_cache: torch.Tensor, v_cache: torch.Tensor):
        self.dims = dims
        dev = k_cache.device
        for i, t in enumerate(weights):
            _check(t, torch.bfloat16, f"weight[{i}]", dev)
        L, Bmax, S, Hkv, D = k_cache.shape
        if (L, Bmax, S, Hkv, D) != (dims.n_layers, dims.max_batch, dims.max_seq, dims.Hkv, dims.D):
            raise ValueError("cache shape does not match dims")
        _check(k_cache, torch.bfloat16, "k_cache", dev)
        _check(v_cache, torch.bfloat16, "v_cache", dev)
        if len(weights) != 3 + 6 * dims.n_layers:
            raise ValueError("weight table: embed, final_norm, lm_head, then 6 per layer "
                             "(wqkv, w_gate_up and lm_head with the preceding norm weight folded in)")
        nbytes = lib().p2pt_llama_ws_bytes(ctypes.byref(dims))
        if nbytes == 0:
            raise ValueError("model dims not supported by the fused decode kernels")
        self.weights = weights  # keep alive
        self._wptr = (ctypes.c_void_p * len(weights))(*[t.data_ptr() for t in weights])
        self.ws = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        self.k_cache, self.v_cache = k_cache, v_cache
        self.device = dev

    def step(self, tokens: torch.Tensor, pos: torch.Tensor, max_len: int, logits: torch.Tensor,
             ids: torch.Tensor, slots: torch.Tensor | None = None, emit_rows: int = 0) -> None:
        """One step over B <= 64 token rows (16-row MFMA tiles). Row b is token
        ``tokens[b]`` at cache position ``pos[b]`` of cache slot ``slots[b]``
        (default: slot b). Rows of one slot at consecutive positions are a prefill
        chunk (causal within the step). Only rows [0, emit_rows) get logits and
        ids (0: all): the LM head skips prefill rows that sample nothing."""
        d = self.dims
        _check(tokens, torch.int64, "tokens", self.device)
        _check(pos, torch.int32, "pos", self.device)
        _check(logits, torch.bfloat16, "logits", self.device)
        _check(ids, torch.int64, "ids", self.device)
        B = tokens.shape[0]
        if slots is not None:
            _check(slots, torch.int32, "slots", self.device)
            if slots.shape != (B,):
                raise ValueError("slots must be [B]")
        limit = MAX_ROWS if slots is not None else min(MAX_ROWS, d.max_batch)
        if not 0 <= emit_rows <= B:
            raise ValueError("emit_rows must be in 0..B")
        if not 1 <= B <= limit or pos.shape != (B,) or ids.shape != (B,):
            raise ValueError(f"rows must be 1..{limit} with matching pos/ids")
        if logits.shape != (B, d.vocab):
            raise ValueError("logits must be [B, vocab]")
        if not 1 <= max_len <= d.max_seq:
            raise ValueError("max_len out of range")
        _ok(lib().p2pt_llama_decode(ctypes.byref(d), self._wptr, _p(self.k_cache), _p(self.v_cache), _p(tokens),
                                    _p(pos), _p(slots), B, emit_rows, max_len, _p(self.ws), self.ws.numel(), _p(logits),
                                    _p(ids), _stream(tokens)), "llama_decode")
