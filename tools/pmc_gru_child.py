"""Child program for PMC passes on the F = 64 CRISP GRU kernels (rocprofv3 --pmc ... -- python3 tools/pmc_gru_child.py):
2^18 Polar(64,32) words at 2 dB, fp32 and fp16x3 paths, 3 launches each."""
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402
from neural_polar_decoder_amd.montecarlo import seeded_crisp  # noqa: E402

code = reference_polar_code(64, 32)
_, _, y = code.mc_generate(1 << 18, 2.0, 1234, 0, 0, want_msg=False)
for prec in ("fp32", "fp16x3"):
    net, dec = seeded_crisp(code, 64, 2, seed=0, device="cuda", precision=prec)
    for _ in range(3):
        dec.decode(net, False, y)
torch.cuda.synchronize()
