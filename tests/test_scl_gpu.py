"""GPU parity of the SC-List decoder (npd_scl_decode / PolarCode.scl_decode) against the reference's
golden vectors (PolarCode.scl_decode, polar.py:793-876) and the C++ oracle (oracle/npd_oracle_scl.cpp).

Bar: bit-exact msg_hat and chosen-path leaf LLRs.  The kernel and the oracle both sum the final ML
distance sequentially in fp32; the reference sums with torch's vectorised reduction, so a codeword whose
two best list candidates differ by less than that rounding could choose differently (none in the
fixtures, whose tie-heavy rows have exactly representable distances)."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SCL_FIXTURES = ["scl_64_32_L4", "scl_32_16_L4", "scl_16_8_L2", "scl_64_32_L8", "scl_32_16_L1", "scl_32_16_L3",
                "scl_8_4_L4", "scl_128_64_L4", "scl_256_128_L4", "scl_128_64_L8"]


def polar_for(N, info):
    from neural_polar_decoder_amd import PolarCode
    F = np.array(sorted(set(range(N)) - set(int(i) for i in info)))
    return PolarCode(int(np.log2(N)), len(info), F=F)


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.mark.parametrize("name", SCL_FIXTURES)
def test_scl_decode_golden(name):
    d = golden(f"{name}.npz")
    N = d["y"].shape[1]
    code = polar_for(N, d["info"])
    for s in np.unique(d["snr"]):
        m = d["snr"] == s
        leaf, hat = code.scl_decode(t(d["y"][m]), float(s), int(d["L"]))
        assert np.array_equal(hat.cpu().numpy(), d["msg_hat"][m]), (name, s)
        assert np.array_equal(leaf.cpu().numpy(), d["leaf"][m]), (name, s)


@pytest.mark.parametrize("N,K", [(64, 32), (32, 16), (16, 8), (8, 4), (64, 22), (128, 64), (256, 128), (256, 200)])
@pytest.mark.parametrize("L", [1, 2, 3, 4, 5, 8])
def test_scl_vs_oracle_random(oracle, N, K, L):
    """Ragged batches (not a multiple of the 64/G codewords of a wave tile) vs the oracle."""
    from neural_polar_decoder_amd import reference_polar_code
    code = reference_polar_code(N, K)
    rng = np.random.default_rng(N * 100 + K + L)
    B = 777
    for snr in (0.0, 2.0):
        _, _, y = code.mc_generate(B, snr, seed=int(rng.integers(1 << 30)), snr_index=0, want_msg=False)
        leaf, hat = code.scl_decode(y, snr, L)
        ol, oh, _ = oracle.scl_decode(y.cpu().numpy(), snr, code.info_positions, L)
        assert np.array_equal(hat.cpu().numpy(), oh), (N, K, L, snr)
        assert np.array_equal(leaf.cpu().numpy(), ol), (N, K, L, snr)


def test_scl_tie_heavy_vs_oracle(oracle):
    """Grid-valued y: many metric ties at the pruning boundary, exercising the in-kernel nth_element."""
    from neural_polar_decoder_amd import reference_polar_code
    rng = np.random.default_rng(11)
    grid = np.array([-1.5, -1.0, -0.5, 0.0, 0.5, 1.0, 1.5], np.float32)
    for N, K, L in [(64, 32, 4), (32, 16, 8), (16, 8, 3), (64, 32, 2), (128, 64, 4), (256, 128, 4), (256, 128, 8)]:
        code = reference_polar_code(N, K)
        y = grid[rng.integers(0, grid.size, (1000, N))]
        _, hat = code.scl_decode(t(y), 1.0, L, want_llrs=False)
        _, oh, _ = oracle.scl_decode(y, 1.0, code.info_positions, L)
        assert np.array_equal(hat.cpu().numpy(), oh), (N, K, L)


@pytest.mark.parametrize("N,K,L", [(64, 32, 2), (64, 32, 4), (64, 32, 8), (256, 128, 4), (256, 200, 2), (128, 64, 8)])
def test_scl_decode_mc_counters_exact(oracle, N, K, L):
    """Fused error counting (message bits regenerated from Philox in the kernel; K > 128 uses a second
    Philox block) equals the oracle's count on the oracle's own decisions."""
    from neural_polar_decoder_amd import reference_polar_code
    code = reference_polar_code(N, K)
    B, seed, off = 3000 if N <= 64 else 1000, 9, 4242
    for si, snr in enumerate([1.0, 3.0]):
        msg, _, y = code.mc_generate(B, snr, seed, si, off)
        cnt = torch.zeros(2, dtype=torch.int64, device=DEV)
        hat = torch.empty(B, K, device=DEV)
        code.scl_decode_mc(y, snr, L, seed, off, cnt, msg_hat=hat)
        _, oh, _ = oracle.scl_decode(y.cpu().numpy(), snr, code.info_positions, L)
        assert np.array_equal(hat.cpu().numpy(), oh)
        assert cnt.cpu().tolist() == list(oracle.count_errors(msg.cpu().numpy(), oh))


def test_scl_list_gain_and_noiseless():
    """Full-size properties: noiseless words decode exactly; at 2 dB SCL-4 beats SC on the same words."""
    from neural_polar_decoder_amd import reference_polar_code
    code = reference_polar_code(64, 32)
    B = 1 << 18
    msg, x, y = code.mc_generate(B, 2.0, seed=3, want_x=True)
    _, hat = code.scl_decode(x, 2.0, 4, want_llrs=False)
    assert torch.equal(hat, msg)
    c_sc = torch.zeros(2, dtype=torch.int64, device=DEV)
    c_l4 = torch.zeros(2, dtype=torch.int64, device=DEV)
    code.sc_decode_mc(y, 2.0, 3, 0, c_sc)
    code.scl_decode_mc(y, 2.0, 4, 3, 0, c_l4)
    bler_sc, bler_l4 = c_sc[1].item() / B, c_l4[1].item() / B
    assert bler_l4 < 0.8 * bler_sc, (bler_sc, bler_l4)


def test_scl_long_noiseless_and_list_gain():
    """N = 256 (the C5 eval loop's SC-List, run_models.py:329): noiseless words decode exactly, and L = 4
    beats SC on the same received words."""
    from neural_polar_decoder_amd import reference_polar_code
    code = reference_polar_code(256, 128)
    B = 1 << 14
    msg, x, y = code.mc_generate(B, 1.5, seed=7, want_x=True)
    _, hat = code.scl_decode(x, 1.5, 4, want_llrs=False)
    assert torch.equal(hat, msg)
    c_sc = torch.zeros(2, dtype=torch.int64, device=DEV)
    c_l4 = torch.zeros(2, dtype=torch.int64, device=DEV)
    code.sc_decode_mc(y, 1.5, 7, 0, c_sc)
    code.scl_decode_mc(y, 1.5, 4, 7, 0, c_l4)
    assert c_l4[1].item() < 0.8 * c_sc[1].item(), (c_sc.tolist(), c_l4.tolist())


def test_scl_montecarlo_shard_invariance():
    from neural_polar_decoder_amd import reference_polar_code
    from neural_polar_decoder_amd.montecarlo import SCLMonteCarlo
    code = reference_polar_code(64, 32)
    one = SCLMonteCarlo(code, 4, [1.0, 2.0], 30_001, 8192, seed=5, rank=0, world=1).run()
    parts = [SCLMonteCarlo(code, 4, [1.0, 2.0], 30_001, 8192, seed=5, rank=r, world=2).run() for r in range(2)]
    assert [sum(p.block_errors[i] for p in parts) for i in range(2)] == one.block_errors
    assert [sum(p.bit_errors[i] for p in parts) for i in range(2)] == one.bit_errors
