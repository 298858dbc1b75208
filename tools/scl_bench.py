"""Quick SC-List throughput sweep (codewords/s) on cuda:0: python tools/scl_bench.py"""
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402


def main():
    dev = "cuda:0"
    for N, K, B, snr in [(64, 32, 1 << 18, 2.0), (256, 128, 1 << 16, 1.0), (128, 64, 1 << 16, 1.0)]:
        code = reference_polar_code(N, K)
        _, _, y = code.mc_generate(B, snr, seed=1, device=dev, want_msg=False)
        cnt = torch.zeros(2, dtype=torch.int64, device=dev)
        for L in (1, 2, 4, 8):
            code.scl_decode_mc(y, snr, L, 1, 0, cnt)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                code.scl_decode_mc(y, snr, L, 1, 0, cnt)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 3
            print(f"N={N} K={K} L={L}: {ms:.3f} ms  {B / ms * 1e3:.3e} cw/s", flush=True)


if __name__ == "__main__":
    main()
