"""npd_gru_decode_count_sweep (RNN_decoder.decode_count_sweep): the eval loop's GRU half over an SNR sweep
(rnn_all.py:853-880) in one launch, errors counted in the decision epilogue.

Bar: bit-exact against the unfused sequence it replaces -- per segment RNN_decoder.decode (the same kernel) followed by
errors_ber / errors_bler's count of decoded[:, cols] against msg (npd_count_errors_cols): identical counters, and
identical decisions when `decoded` is requested.  Ragged batches (B not a multiple of the 16-codeword tile), reverse
order, unsorted columns, PAC(128,64), and the per-segment path of handles the fused kernel does not cover (fp32)."""
import numpy as np
import pytest
import torch

from conftest import trained_fixture

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def trained_net(name, precision, reverse=False):
    from neural_polar_decoder_amd.rnn import RNN_Model, RNN_decoder
    d = trained_fixture(name)
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    net = RNN_Model("GRU", N + 2, F, 1, L, N, 0, 0).to(DEV).eval()
    net.load_state_dict({k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")})
    return net, RNN_decoder("y_input", N, d["info"], onehot=True, reverse_order=reverse, precision=precision), d


def words(code, snrs, B, seed=11):
    ys, msg = [], None
    for si, s in enumerate(snrs):
        m, _, y = code.mc_generate(B, s, seed, si, 0, device=DEV)
        msg = m if msg is None else msg
        ys.append(y)
    return msg, torch.stack(ys).contiguous()


def unfused(net, dec, y, msg, cols):
    from neural_polar_decoder_amd.utils import count_errors
    c = torch.zeros(y.shape[0], 2, dtype=torch.int64, device=DEV)
    outs = []
    for s in range(y.shape[0]):
        d = dec.decode(net, False, y[s])
        count_errors(msg, d, c[s], cols=cols)
        outs.append(d)
    return c, torch.stack(outs)


@pytest.mark.parametrize("precision", ["fp16x3", "fp32"])
@pytest.mark.parametrize("B", [16 * 700 + 5, 4096])
def test_sweep_counts_equal_unfused(precision, B):
    from neural_polar_decoder_amd import reference_polar_code
    net, dec, d = trained_net("trained_crisp_32_16", precision)
    code = reference_polar_code(int(d["N"]), int(d["K"]))
    info = np.asarray(code.info_positions)
    assert np.array_equal(info, d["info"])
    msg, y = words(code, [0.0, 1.0, 2.0, 3.0, 4.0], B)
    ref_c, ref_d = unfused(net, dec, y, msg, info)
    c = torch.zeros(5, 2, dtype=torch.int64, device=DEV)
    dec.decode_count_sweep(net, y, msg, c)
    assert torch.equal(c.cpu(), ref_c.cpu()), (c.cpu(), ref_c.cpu())
    assert int(ref_c[:, 1].sum()) > 0  # a decoding net: errors at every SNR, so the counts are not vacuous
    out = torch.full_like(ref_d, 7.0)
    c2 = torch.zeros(5, 2, dtype=torch.int64, device=DEV)
    dec.decode_count_sweep(net, y, msg, c2, decoded=out)
    assert torch.equal(c2.cpu(), ref_c.cpu())
    assert torch.equal(out.cpu(), ref_d.cpu())


def test_sweep_unsorted_cols_and_reverse():
    """cols in any order (msg column k <-> position cols[k]) and reverse-order decoding."""
    from neural_polar_decoder_amd import reference_polar_code
    net, dec, d = trained_net("trained_crisp_32_16", "fp16x3", reverse=True)
    code = reference_polar_code(32, 16)
    msg, y = words(code, [1.0, 3.0], 3000)
    perm = np.random.default_rng(5).permutation(16)
    cols = np.asarray(code.info_positions)[perm]
    msgp = msg[:, torch.from_numpy(perm).to(DEV)].contiguous()
    ref_c, _ = unfused(net, dec, y, msgp, cols)
    c = torch.zeros(2, 2, dtype=torch.int64, device=DEV)
    dec.decode_count_sweep(net, y, msgp, c, cols=cols)
    assert torch.equal(c.cpu(), ref_c.cpu())


def test_sweep_pac_128_64():
    """configs[3]'s shape (N = 128: four K blocks of the y projection), seeded weights, counted against the PAC
    message (cols = the information set B)."""
    import argparse
    from neural_polar_decoder_amd import PAC
    from neural_polar_decoder_amd.montecarlo import seeded_crisp
    code = PAC(argparse.Namespace(target_K=64), 128, 64, 91)
    net, dec = seeded_crisp(code, 64, 2, seed=0, device=DEV, precision="fp16x3")
    msg, y = words(code, [0.0, 4.0], 2048 + 9)
    ref_c, _ = unfused(net, dec, y, msg, code.B)
    c = torch.zeros(2, 2, dtype=torch.int64, device=DEV)
    dec.decode_count_sweep(net, y, msg, c, cols=code.B)
    assert torch.equal(c.cpu(), ref_c.cpu())


def test_sweep_rejects_bad_shapes():
    from neural_polar_decoder_amd import reference_polar_code
    net, dec, d = trained_net("trained_crisp_32_16", "fp16x3")
    code = reference_polar_code(32, 16)
    msg, y = words(code, [1.0], 64)
    c = torch.zeros(1, 2, dtype=torch.int64, device=DEV)
    with pytest.raises(ValueError):
        dec.decode_count_sweep(net, y[0], msg, c)          # not (n_snr, B, N)
    with pytest.raises(ValueError):
        dec.decode_count_sweep(net, y, msg[:, :8], c)      # msg columns != cols
    with pytest.raises(ValueError):
        dec.decode_count_sweep(net, torch.cat([y, y]), msg, c)  # counters too small for 2 segments


def test_sweep_non_pm1_messages():
    """count_errors_kernel compares rint(msg) with rint(decision); the fused count keeps that rule for messages outside
    {-1, +1} (0 / 1 messages, other integers): the 2-bit codes map -1, +1, 0 and 'other' (never equal to a decision)."""
    from neural_polar_decoder_amd import reference_polar_code
    net, dec, d = trained_net("trained_crisp_32_16", "fp16x3")
    code = reference_polar_code(32, 16)
    _, y = words(code, [1.0, 2.0], 2000 + 3)
    g = torch.Generator(device="cpu").manual_seed(3)
    vals = torch.tensor([-1.0, 1.0, 0.0, 2.0, -3.0, 0.4, -0.6])
    msg = vals[torch.randint(0, len(vals), (y.shape[1], 16), generator=g)].to(DEV)
    ref_c, _ = unfused(net, dec, y, msg, np.asarray(code.info_positions))
    c = torch.zeros(2, 2, dtype=torch.int64, device=DEV)
    dec.decode_count_sweep(net, y, msg, c)
    assert torch.equal(c.cpu(), ref_c.cpu())


@pytest.mark.parametrize("kind", ["polar", "pac"])
def test_montecarlo_driver_sweep_equals_per_point(kind):
    """GRUMonteCarlo.count_sweep (one npd_gru_decode_count_sweep launch per batch, the messages generated once) gives
    the counters of the per-SNR-point path (generate with message, decode, count) on the same Philox streams."""
    import argparse
    from neural_polar_decoder_amd import PAC
    from neural_polar_decoder_amd.montecarlo import GRUMonteCarlo, MonteCarlo, seeded_crisp
    if kind == "pac":
        code = PAC(argparse.Namespace(target_K=64), 128, 64, 91)
        net, dec = seeded_crisp(code, 64, 2, seed=1, device=DEV, precision="fp16x3")
    else:
        net, dec, d = trained_net("trained_crisp_32_16", "fp16x3")
        from neural_polar_decoder_amd import reference_polar_code
        code = reference_polar_code(32, 16)
    mc = GRUMonteCarlo(code, net, dec, [0.0, 2.0, 4.0], 5000, 2048, seed=5, rank=0, world=1, device=DEV)
    a = mc.new_counters()
    b = mc.new_counters()
    for off in range(0, 5000, 2048):
        n = min(2048, 5000 - off)
        mc.count_sweep(off, n, a)
        MonteCarlo.count_sweep(mc, off, n, b)
    assert torch.equal(a.cpu(), b.cpu()) and int(a[:, 0].sum()) > 0
