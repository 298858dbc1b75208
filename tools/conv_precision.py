#!/usr/bin/env python3
"""Conv-model precision study (round 4, as tools/gru_precision.py for the GRU): logit error of every implementation
of convNet's forward against the float64 restatement (oracle.conv_forward), on the configs[4] shape and on the
trained conv fixture.

    python tools/conv_precision.py [--n5 1024] [--nt 8192] [--out FILE]

Implementations:
  * "reference" -- the reference's arithmetic (models.py:742-767: Conv1d + GELU blocks, residuals, flatten c*N + l,
                   Linear + GELU, Linear + GELU, Linear, LayerNorm(eps 1e-6)) as torch fp32 ops on the CPU;
  * "fp32"      -- the HIP fp32 path the bench times (conv_layer_kernel / fc_kernel, v_mfma_f32_32x32x2_f32);
  * "fp16x3"    -- the split path (conv_ws16_kernel / conv_split_ws_kernel / fc_split_wsp_kernel, hi + lo fp16, three products).
Decision flips are counted against the float64 decisions (sign of the logit)."""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as Fn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import conv_weights_from_seed  # noqa: E402
from oracle import oracle as O  # noqa: E402

PCT = [50.0, 99.0, 99.9, 100.0]


def reference_forward(y, sd):
    """models.py:742-767 in torch fp32 on the CPU (the ATen calls nn.Conv1d / nn.GELU / nn.Linear / nn.LayerNorm make)."""
    t = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in sd.items()}
    x = torch.from_numpy(np.asarray(y, np.float32))[:, None, :]

    def conv(name, x, pad, dil):
        return Fn.gelu(Fn.conv1d(x, t[name + ".weight"], t.get(name + ".bias"), padding=pad, dilation=dil))

    spec = O.CONV_SPEC
    with torch.no_grad():
        x2 = conv(spec[1][0], conv(spec[0][0], x, spec[0][1], spec[0][2]), spec[1][1], spec[1][2])
        x3 = conv(spec[3][0], conv(spec[2][0], x2, spec[2][1], spec[2][2]), spec[3][1], spec[3][2]) + x2
        x4 = conv(spec[5][0], conv(spec[4][0], x3, spec[4][1], spec[4][2]), spec[5][1], spec[5][2]) + x3
        x5 = conv(spec[7][0], conv(spec[6][0], x4, spec[6][1], spec[6][2]), spec[7][1], spec[7][2]) + x4
        x6 = conv(spec[9][0], conv(spec[8][0], x5, spec[8][1], spec[8][2]), spec[9][1], spec[9][2])
        h = x6.reshape(x6.shape[0], -1)
        h = Fn.gelu(Fn.linear(h, t["layersFin.0.weight"], t["layersFin.0.bias"]))
        h = Fn.gelu(Fn.linear(h, t["layersFin.2.weight"], t["layersFin.2.bias"]))
        h = Fn.linear(h, t["layersFin.4.weight"], t["layersFin.4.bias"])
        h = Fn.layer_norm(h, (h.shape[1],), t["layer_norm.weight"], t["layer_norm.bias"], eps=1e-6)
    return h.numpy()


def hip_forward(y, sd, E, N, precision):
    from neural_polar_decoder_amd.models import convNet
    cfg = argparse.Namespace(embed_dim=E, max_len=N, N=N, dont_use_bias=False, dropout=0.0)
    net = convNet(cfg, precision=precision)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    lg, _ = net.eval().logits(torch.from_numpy(y).to("cuda:0"))
    return lg.cpu().numpy()


def stats(lg, ref64):
    err = np.abs(lg.astype(np.float64) - ref64).ravel()
    q = np.percentile(err, PCT)
    flips = (np.sign(lg) != np.sign(ref64)) & (np.abs(ref64) > 0)
    return {"p50": float(q[0]), "p99": float(q[1]), "p99.9": float(q[2]), "max": float(q[3]),
            "mean": float(err.mean()), "bit_flips": int(flips.sum()), "cw_flips": int(flips.any(1).sum())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n5", type=int, default=512, help="configs[4] words (embed 128, N 256, seeded weights)")
    ap.add_argument("--nt", type=int, default=8192, help="trained embed-16 fixture words")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rng = np.random.default_rng(2024)
    cases = []
    d5 = np.load(os.path.join(ROOT, "tests", "golden", "conv_c5_256.npz"))
    sd5 = conv_weights_from_seed(int(d5["embed"]), int(d5["N"]), int(d5["seed"]))
    y5 = (np.where(rng.random((a.n5, 256)) < 0.5, -1.0, 1.0) + 0.7 * rng.standard_normal((a.n5, 256))).astype(np.float32)
    cases.append(("configs[4] embed 128 N 256 seeded, 1 dB-like words", sd5, int(d5["embed"]), 256, y5))
    tp = os.path.join(ROOT, "tests", "golden", "trained_conv_64_22.npz")
    if os.path.exists(tp):
        dt = np.load(tp)
        sdt = {k[2:]: np.asarray(dt[k]) for k in dt.files if k.startswith("w.")}
        yt = (np.where(rng.random((a.nt, 64)) < 0.5, -1.0, 1.0) + 0.8 * rng.standard_normal((a.nt, 64))).astype(np.float32)
        cases.append(("trained_conv_64_22 (embed 16, N 64)", sdt, int(dt["embed"]), 64, yt))
    out = {"source": "tools/conv_precision.py: |logit - float64 oracle| over all positions; flips = sign differences",
           "cases": {}}
    for name, sd, E, N, y in cases:
        ref64 = np.concatenate([O.conv_forward(y[i:i + 256], sd, out_dtype=np.float64) for i in range(0, len(y), 256)])
        row = {"words": int(len(y)), "reference": stats(reference_forward(y, sd), ref64)}
        for prec in ("fp32", "fp16x3"):
            row[prec] = stats(hip_forward(y, sd, E, N, prec), ref64)
        out["cases"][name] = row
        print(name, json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
