"""Child program for PMC passes on the PAC(128,64) SC decode (rocprofv3 --pmc ... -- python3 tools/pmc_pac.py):
the bench's pac_sc configuration -- 2^20 words at 2 dB, msg_hat written, compile-time frozen set -- launched 3
times, then Polar(128,64) SC decode (same kernel family, run-time frozen set) 3 times."""
import argparse
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import PAC, reference_polar_code  # noqa: E402


def main():
    dev = "cuda:0"
    cnt = torch.zeros(8, 2, dtype=torch.int64, device=dev)
    pac = PAC(argparse.Namespace(target_K=64), 128, 64, 91)
    _, _, yp = pac.mc_generate(1 << 20, 2.0, 1, 2, 0, device=dev, want_msg=False)
    hat = torch.empty(1 << 20, 64, device=dev)
    c128 = reference_polar_code(128, 64)
    _, _, y128 = c128.mc_generate(1 << 20, 2.0, 1, 0, 0, device=dev, want_msg=False)
    hat128 = torch.empty(1 << 20, 64, device=dev)
    for _ in range(3):
        pac.sc_decode_mc(yp, 2.0, 1, 0, cnt[0], msg_hat=hat)
    for _ in range(3):
        c128.sc_decode_mc(y128, 2.0, 1, 0, cnt[1], msg_hat=hat128)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
