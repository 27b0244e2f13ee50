"""Helper for tests/test_gpu_model.py (not a test module): runs T fused decode
steps of a random-init model and saves the last logits, ids and caches, so a
test can compare decode variants that are chosen by environment variables read
once per process (e.g. P2PT_DECODE_BLOCK, the persistent O/gate-up/down kernel).

    python tests/gpu_decode_run.py CFG B T OUT.pt [--graph]
"""
import sys

import torch


def main():
    cfg, B, T, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    graph = "--graph" in sys.argv[5:]
    sys.path.insert(0, __file__.rsplit("/tests/", 1)[0])
    from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama
    m = TinyLlama(cfg, device="cuda", max_batch=B, seed=11, fused=True)
    torch.manual_seed(5)
    seqs = torch.randint(0, m.cfg.vocab, (B, T), device="cuda")
    if graph:
        m.capture_graph(rows=B)
    ids = logits = None
    for p in range(T):
        pos = torch.full((B,), p, dtype=torch.int32, device="cuda")
        if graph:
            ids, logits = m.graph_step(seqs[:, p], pos, return_logits=True)
        else:
            ids, logits = m.decode_step(seqs[:, p], pos, (p, p), return_logits=True)
        if p % 10 == 0:
            torch.cuda.synchronize()
            print(f"{cfg} B={B} step {p}", flush=True)
    torch.cuda.synchronize()
    torch.save({"ids": ids.cpu(), "logits": logits.float().cpu(), "k": m.k_cache[:, :B, :T].float().cpu(),
                "ref": m.reference_logits(seqs).float().cpu()}, out)


if __name__ == "__main__":
    main()
