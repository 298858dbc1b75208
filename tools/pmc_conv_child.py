"""PMC child for the fp16x3 conv model: two forwards of one 4096-codeword chunk of configs[4] (Polar(256,128) convNet
embed 128, seeded weights) on cuda:0.  Used by tools/gpu_pmc_k.sh (PMC_CHILD=tools/pmc_conv_child.py)."""
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402
from neural_polar_decoder_amd.montecarlo import seeded_conv  # noqa: E402

net = seeded_conv(256, 128, seed=0, device="cuda")
net.precision = "fp16x3"
code = reference_polar_code(256, 128)
_, _, y = code.mc_generate(4096, 1.0, 7, 0, 0, device="cuda", want_msg=False)
for _ in range(2):
    net.logits(y)
torch.cuda.synchronize()
print("ok", flush=True)
