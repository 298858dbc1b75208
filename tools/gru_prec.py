"""GRU decode time per 2^20 Polar(64,32) words for each precision path (cuda:0): python tools/gru_prec.py"""
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402
from neural_polar_decoder_amd.montecarlo import seeded_crisp  # noqa: E402

code = reference_polar_code(64, 32)
_, _, y = code.mc_generate(1 << 20, 2.0, 1234, 0, 0, want_msg=False)
ref = None
for prec in ("fp32", "fp16x3", "bf16x3", "bf16"):
    net, dec = seeded_crisp(code, 64, 2, seed=0, device="cuda", precision=prec)
    d, lg = dec.decode(net, False, y, return_logits=True)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        dec.decode(net, False, y)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 3
    extra = ""
    if ref is None:
        ref = (d, lg)
    else:
        same = (d == ref[0]).all(1)
        extra = f" cw agree {same.float().mean().item():.6f} max |dlogit| {(lg[same] - ref[1][same]).abs().max().item():.2e}"
    print(f"{prec:7s} {ms:7.2f} ms  {(1 << 20) / ms * 1e3:.3e} cw/s{extra}", flush=True)
