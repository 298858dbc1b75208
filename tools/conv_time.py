"""configs[4] conv forward time, fp32 vs fp16x3 (Polar(256,128) convNet embed 128, 8192 codewords, cuda:0), and the
fp16x3 logits' max difference from fp32's.  python tools/conv_time.py [reps]"""
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402
from neural_polar_decoder_amd.montecarlo import seeded_conv  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
net = seeded_conv(256, 128, seed=0, device="cuda")
code = reference_polar_code(256, 128)
_, _, y = code.mc_generate(8192, 1.0, 7, 0, 0, device="cuda", want_msg=False)
out = {}
for rep in range(reps):
    for prec in ("fp32", "fp16x3"):
        net.precision = prec
        lg, _ = net.logits(y)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            net.logits(y)
        e.record()
        torch.cuda.synchronize()
        out[prec] = lg
        print(f"{prec:7s} {s.elapsed_time(e) / 5:8.3f} ms per 8192", flush=True)
print(f"max |logit fp16x3 - fp32| {(out['fp16x3'] - out['fp32']).abs().max().item():.2e}", flush=True)
