"""Reference on-disk formats: standard test sets (run_models.py:797-803) and checkpoints
(rnn_all.py:1474-1615).  CPU tests cover loading (weights_only, no code execution); GPU tests cover
evaluation through the kernels."""
import argparse

import numpy as np
import pytest
import torch

from conftest import golden


def ref_args(**kw):
    d = dict(code="Polar", rate_profile="polar", N=64, K=32, target_K=32, g=91, rnn_type="GRU",
             decoding_type="y_input", rnn_feature_size=64, rnn_depth=2, onehot=True, reverse_order=False,
             use_ynn=False, out_linear_depth=1, activation="selu", dropout=0.0, use_skip=False,
             bidirectional=False, use_layernorm=False, model="conv", embed_dim=16, max_len=64,
             dont_use_bias=False)
    d.update(kw)
    return argparse.Namespace(**d)


class Evil:
    """Stands for any non-allow-listed class inside a checkpoint."""


def gru_state(d):
    return {k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")}


def test_checkpoint_roundtrip_weights_only(tmp_path):
    from neural_polar_decoder_amd.datasets import load_checkpoint, rnn_from_checkpoint
    d = golden("gru_polar_64_32.npz")
    path = tmp_path / "model_final.pt"
    torch.save({"net": gru_state(d), "step": 100, "args": ref_args()}, path)
    ck = load_checkpoint(str(path))
    assert ck["step"] == 100 and ck["args"].rnn_feature_size == 64
    net, dec, code = rnn_from_checkpoint(ck, device="cpu")
    for k, v in gru_state(d).items():
        assert torch.equal(net.state_dict()[k], v)
    assert np.array_equal(code.info_positions, d["info"])
    assert dec.onehot and dec.N == 64


def test_checkpoint_refuses_pickled_code(tmp_path):
    """A checkpoint carrying an arbitrary class is refused by the weights-only loader."""
    from neural_polar_decoder_amd.datasets import load_checkpoint
    path = tmp_path / "bad.pt"
    torch.save({"net": {}, "args": Evil()}, path)
    with pytest.raises(Exception):
        load_checkpoint(str(path))


def test_standard_set_roundtrip(tmp_path):
    from neural_polar_decoder_amd.datasets import load_standard, polar_test_path, save_standard
    msg = 1 - 2 * torch.randint(0, 2, (64, 32)).float()
    rec = {0.0: torch.randn(64, 64), 2.0: torch.randn(64, 64)}
    p = polar_test_path(64, 32, root=str(tmp_path))
    save_standard(p, {"msg": msg, "rec": rec, "snr": [0.0, 2.0]})
    m, r, s = load_standard(p)
    assert torch.equal(m, msg) and s == [0.0, 2.0] and torch.equal(r[2.0], rec[2.0])


@pytest.mark.gpu
def test_evaluate_standard_matches_montecarlo():
    """SC on a generated standard set == the sharded MC driver on the same Philox streams; the
    checkpoint-built GRU decodes identically to the directly-built one."""
    from neural_polar_decoder_amd import reference_polar_code
    from neural_polar_decoder_amd.datasets import evaluate_standard, make_standard, rnn_from_checkpoint
    from neural_polar_decoder_amd.montecarlo import SCMonteCarlo
    code = reference_polar_code(64, 32)
    data = make_standard(code, [1.0, 3.0], 8192, seed=77)
    d = golden("gru_polar_64_32.npz")
    net, dec, _ = rnn_from_checkpoint({"net": gru_state(d), "args": ref_args()}, device="cuda:0")
    res = evaluate_standard(code, data["msg"], data["rec"], 4096, list_size=4, gru=(net, dec))
    mc = SCMonteCarlo(code, [1.0, 3.0], 8192, 8192, seed=77).run()
    assert res["SC"]["bler"] == mc.bler and res["SC"]["ber"] == mc.ber
    assert all(l <= s for l, s in zip(res["SCL"]["bler"], res["SC"]["bler"]))
    assert len(res["RNN"]["ber"]) == 2
