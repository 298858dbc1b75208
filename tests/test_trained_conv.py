"""The oracle's convNet restatement at trained-model margins (CPU): logits of oracle.conv_forward on the trained conv
fixture's words (tests/golden/gen_trained_conv.py: run_alt.sh-shaped n2c curriculum with the reference's own
run_models.py, embed 16, Polar(64,22)) against the reference's convNet.forward logits (within 1e-4) and its
decisions; the fixture's provenance (curriculum) and that the net decodes (reference BLER < 0.5 at >= 2 SNR points)."""
import hashlib
import os
import sys

import numpy as np
import pytest
import torch

from conftest import trained_fixture

NAMES = ["trained_conv_64_22", "trained_conv_64_22_e128"]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_conv_trained_fixture(oracle, name):
    d = trained_fixture(name)
    N, K = int(d["N"]), int(d["K"])
    sd = {k[2:]: np.asarray(d[k]) for k in d.files if k.startswith("w.")}
    info = d["info"]
    for si in range(len(d["snr"])):
        torch.manual_seed(int(d["seed_dec"]) + si)
        msg = 1.0 - 2.0 * (torch.rand(int(d["n_dec"]), K) < 0.5).float()
        x = torch.from_numpy(oracle.encode_plotkin(msg.numpy(), N, info))
        y = (x + 10 ** (-float(d["snr"][si]) / 20) * torch.randn(x.shape, dtype=torch.float)).numpy()
        assert hashlib.sha256(np.ascontiguousarray(y).tobytes()).hexdigest() == bytes(d[f"y_digest_{si}"]).decode()
        m = d[f"logits_{si}"].shape[0]
        lg = oracle.conv_forward(y[:m], sd)
        # the reference's own fp32 logits sit up to 3.1e-5 from the float64 ones on these words (trained weights:
        # LayerNorm of a larger-magnitude FC output); the bar for any fp32-class implementation is 1e-4
        assert np.abs(lg - d[f"logits_{si}"]).max() < 1e-4
        ref = np.where(np.unpackbits(d[f"dec_bits_{si}"], axis=1)[:m, :K] == 1, -1.0, 1.0)
        sure = np.abs(d[f"logits_{si}"][:, info]) > 1e-4
        assert np.array_equal(np.sign(lg[:, info])[sure], ref[sure])
    ref_bler = np.asarray(d["mc_blk_err"], float) / int(d["mc_n"])
    assert (ref_bler < 0.5).sum() >= 2, ref_bler
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import importlib.util
    spec = importlib.util.spec_from_file_location("gtc", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                      "golden", "gen_trained_conv.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    cur = g.CASES[name]["curriculum"]
    if cur is None:  # GPU-trained (tests/golden/train_conv_gpu.py holds its curriculum)
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
        import train_conv_gpu
        cur = train_conv_gpu.CASE["curriculum"]
    assert [tuple(int(v) for v in r) for r in d["curriculum"]] == [tuple(r) for r in cur]
