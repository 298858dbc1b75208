#!/usr/bin/env python3
"""Measured max |logits(GPU) - reference| of the fused convNet on its golden fixtures and vs the oracle
(tests/test_conv_gpu.py's tolerance is set from these).  Prints one JSON line."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import conv_weights_from_seed  # noqa: E402
from neural_polar_decoder_amd.models import convNet  # noqa: E402
from oracle import oracle as O  # noqa: E402


def net_from(sd, embed, N):
    net = convNet(argparse.Namespace(embed_dim=embed, max_len=N, N=N, dont_use_bias=False, dropout=0.0))
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return net.eval()


out = {}
d = np.load(os.path.join(ROOT, "tests", "golden", "conv_small_64.npz"))
sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
net = net_from(sd, int(d["embed"]), int(d["N"]))
lg = net.logits(torch.from_numpy(d["y"]).cuda())[0].cpu().numpy()
out["small_64_vs_reference"] = float(np.abs(lg - d["logits"]).max())
y = np.random.default_rng(1).standard_normal((4096 + 77, 64)).astype(np.float32)
lg = net.logits(torch.from_numpy(y).cuda())[0].cpu().numpy()[::37]
out["small_64_vs_oracle"] = float(np.abs(lg - O.conv_forward(y[::37], sd)).max())
d = np.load(os.path.join(ROOT, "tests", "golden", "conv_c5_256.npz"))
sd = conv_weights_from_seed(int(d["embed"]), int(d["N"]), int(d["seed"]))
net = net_from(sd, int(d["embed"]), int(d["N"]))
lg = net.logits(torch.from_numpy(d["y"]).cuda())[0].cpu().numpy()
out["c5_256_vs_reference"] = float(np.abs(lg - d["logits"]).max())
out["c5_logit_abs_max"] = float(np.abs(d["logits"]).max())
print(json.dumps(out))
