"""A/B the register-resident and LDS-resident soft-SC kernels at N <= 64 on extreme received words, and
print, for the N = 128 fixture row that differs from the reference, the first leaf where the GPU differs."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402

for N in (32, 64):
    code = reference_polar_code(N, N // 2)
    rows = []
    for v in (-1.0, 1.0, -0.5, 2.0):
        rows.append(np.full(N, v, np.float32))
    rng = np.random.default_rng(1)
    rows += [(rng.choice([-1.0, 1.0], N) * 3).astype(np.float32) for _ in range(60)]
    y = torch.from_numpy(np.stack(rows)).cuda()
    prior = rng.standard_normal(N).astype(np.float32)
    for snr in (0.0, 2.0, 4.0, 6.0, 10.0):
        os.environ.pop("NPD_SOFT_LDS", None)
        _, b1 = code.sc_decode_soft(y, snr, priors=prior, hard_decision=False, return_bits=True)
        os.environ["NPD_SOFT_LDS"] = "1"
        _, b2 = code.sc_decode_soft(y, snr, priors=prior, hard_decision=False, return_bits=True)
        b1, b2 = b1.cpu().numpy(), b2.cpu().numpy()
        same = np.array_equal(np.nan_to_num(b1, nan=7.0), np.nan_to_num(b2, nan=7.0))
        print(N, snr, "reg == lds:", same, "nan reg", int(np.isnan(b1).sum()), "nan lds", int(np.isnan(b2).sum()))
