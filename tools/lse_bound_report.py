#!/usr/bin/env python3
"""Measured max |decoded_bits(GPU) - reference| / (2 E) over the exact-LSE / soft-SC golden fixtures, E =
the oracle's forward error bound (oracle.sc_decode_lse_bound / sc_decode_soft_bound).  Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from neural_polar_decoder_amd import PolarCode  # noqa: E402

out = {}
for N, K in [(16, 8), (32, 16), (64, 32), (128, 64)]:
    d = np.load(os.path.join(ROOT, "tests", "golden", f"lse_{N}_{K}.npz"))
    code = PolarCode(int(np.log2(N)), K, F=np.setdiff1d(np.arange(N), d["info"]))
    worst, mx, n = 0.0, 0.0, 0
    for s in np.unique(d["snr"]):
        m = d["snr"] == s
        h, b = code.sc_decode(torch.from_numpy(d["y"][m]).cuda(), float(s), hard_decision=False, return_bits=True)
        h, b = h.cpu().numpy(), b.cpu().numpy()
        E = O.sc_decode_lse_bound(d["y"][m], float(s), d["info"])[1]
        rows = (h == d["msg_hat_soft"][m]).all(1)
        g = d["bits_soft"][m][rows]
        fin = ~np.isnan(g)
        err = np.abs(b[rows][fin].astype(np.float64) - g[fin])
        worst = max(worst, float((err / np.maximum(2 * E[rows][fin], 1e-300)).max(initial=0)))
        mx = max(mx, float(err.max(initial=0)))
        n += int(fin.sum())
    out[f"lse_{N}_{K}"] = {"max_ratio": worst, "max_abs": mx, "entries": n}
print(json.dumps(out))
