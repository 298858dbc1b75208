"""Child program for PMC passes on the secondary kernels (rocprofv3 --pmc ... -- python3 tools/pmc_kernels.py):
SC-List L = 4 at Polar(256,128) (2^16 words, 1 dB) and Polar(64,32) (2^18, 2 dB), exact-LSE SC soft / hard at
Polar(64,32) (2^18, 2 dB), PAC(128,64) SC streaming decode with msg_hat and its fused Monte-Carlo sweep
(2^20 words).  Each is launched 3 times."""
import argparse
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import PAC, reference_polar_code  # noqa: E402


def main():
    dev = "cuda:0"
    cnt = torch.zeros(8, 2, dtype=torch.int64, device=dev)
    c256 = reference_polar_code(256, 128)
    _, _, y256 = c256.mc_generate(1 << 16, 1.0, 1, 0, 0, device=dev, want_msg=False)
    c64 = reference_polar_code(64, 32)
    _, _, y64 = c64.mc_generate(1 << 18, 2.0, 1, 0, 0, device=dev, want_msg=False)
    pac = PAC(argparse.Namespace(target_K=64), 128, 64, 91)
    _, _, yp = pac.mc_generate(1 << 20, 2.0, 1, 2, 0, device=dev, want_msg=False)
    hat = torch.empty(1 << 20, 64, device=dev)
    for _ in range(3):
        c256.scl_decode_mc(y256, 1.0, 4, 1, 0, cnt[0])
        c64.scl_decode_mc(y64, 2.0, 4, 1, 0, cnt[1])
        c64.sc_decode(y64, 2.0, hard_decision=False)
        c64.sc_decode(y64, 2.0, hard_decision=True)
        pac.sc_decode_mc(yp, 2.0, 1, 0, cnt[2], msg_hat=hat)
        pac.sc_mc_sweep_fused(1 << 20, [2.0], 1, 0, cnt[3:4], snr_index0=2)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
