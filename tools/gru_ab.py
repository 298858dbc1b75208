"""A/B of the F <= 64 GRU kernel's workgroup size (NPD_GRU_WAVES=4 vs 8) at configs[2]: Polar(64,32),
hidden 64, 2 layers, 2^20 codewords.  Run once per setting (the choice is read once per process)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402
from neural_polar_decoder_amd.montecarlo import seeded_crisp  # noqa: E402

code = reference_polar_code(64, 32)
net, dec = seeded_crisp(code, 64, 2, seed=0, device="cuda")
_, _, y = code.mc_generate(1 << 20, 2.0, 1234, 0, 0, want_msg=False)
d0 = dec.decode(net, False, y)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(3):
    dec.decode(net, False, y)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 3
print(json.dumps({"waves": os.environ.get("NPD_GRU_WAVES", "default"), "ms": ms, "cw_s": (1 << 20) / ms * 1e3,
                  "frac": 4751360 * (1 << 20) / (ms / 1e3) / 1e12 / 157.3,
                  "checksum": float(d0.sum().item())}))
