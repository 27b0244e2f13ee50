"""Sampler diagnostics on the GPU box: chi-square p-values of the on-device
sampler against the fp32 reference over several seeds per (T, k, p) — under a
correct sampler they are uniform on (0, 1) — plus one row's logits and draws
saved for an exact host-side replay of the hash/Gumbel-max."""
import json
import sys

import numpy as np
import torch
from scipy.stats import chi2

sys.path.insert(0, ".")
from p2p_llm_tunnel_amd import ops  # noqa: E402
from tests.test_gpu_ops import _draws, _ref_probs  # noqa: E402

torch.manual_seed(11)
V = 1000
row = (torch.randn(V, device="cuda") * 2.0).to(torch.bfloat16)
out = {}
for T, k, p in [(0.8, 0, 1.0), (1.0, 20, 1.0), (0.7, 0, 0.9), (1.2, 50, 0.8), (1.0, 0, 0.5)]:
    probs = _ref_probs(row, T, k, p).double().cpu()
    pv = []
    for seed in range(1, 21):
        got = _draws(ops, row, T, k, p, n_launch=100, seed=seed * 7919).cpu()
        n = got.numel()
        counts = torch.bincount(got, minlength=V).double()
        exp = probs * n
        big = exp >= 5
        stat = ((counts[big] - exp[big]) ** 2 / exp[big]).sum().item()
        dof = int(big.sum().item()) - 1
        re, ro = exp[~big].sum().item(), counts[~big].sum().item()
        if re >= 5:
            stat += (ro - re) ** 2 / re
            dof += 1
        pv.append(float(chi2.sf(stat, dof)))
    out[f"T={T} k={k} p={p}"] = {"pvalues": [round(x, 4) for x in pv], "min": min(pv), "mean": float(np.mean(pv))}
    print(f"T={T} k={k} p={p}: mean p {np.mean(pv):.3f} min {min(pv):.4f}", flush=True)
d = _draws(ops, row, 1.0, 20, 1.0, n_launch=4, seed=1234).cpu().numpy()
np.savez("gpurun_out/sample_diag.npz", row=row.float().cpu().numpy(), draws=d)
json.dump(out, open("gpurun_out/sample_diag.json", "w"), indent=1)
