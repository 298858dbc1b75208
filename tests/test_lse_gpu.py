"""GPU parity of the exact-LSE SC decoder (npd_sc_decode_lse / PolarCode.sc_decode) and the soft-output
SC decoder (sc_decode_soft) against the reference's golden vectors (polar.py:209-358) and the C oracle
(oracle/npd_oracle_lse.c).

Tolerance, by analysis: exp/log/tanh are the device libm (OCML) on the GPU, glibc in the oracle and Sleef
in torch's CPU path, each within 2 ulp.  The oracle propagates a first-order forward error bound E through
the same recursion (oracle.sc_decode_lse_bound / sc_decode_soft_bound: exact sensitivities of the boxplus,
of g = u a + b, of tanh(L/2) and of the partial-sum products, plus each operation's rounding), so two
implementations of the model differ by at most 2 E per decoded_bits entry.  Soft partial sums multiply
LLRs of magnitude ~1e2 (g = u a + b), so E reaches ~1e-2 on ill-conditioned entries -- the drifts up to
~0.06 seen before were such entries.  Bars:
  * decisions: a decision may differ only where its LLR (the oracle's) is within 2 E_L of zero -- checked
    for the first disagreement of each codeword in sc_decode (later ones follow from it through the
    partial sums) and for every disagreement in sc_decode_soft (whose decisions feed nothing);
  * values: hard decoded_bits bit-exact on agreeing codewords; EVERY finite soft decoded_bits entry within
    2 E of the reference (max |diff| / 2E is reported); same NaN positions wherever the leaf's bound is
    finite (a leaf whose computation met an inf/NaN -- crafted words whose LLRs approach exp's overflow --
    may be finite in one implementation and NaN in the other: an ulp decides whether exp overflows).
Measured on MI355X (tools/lse_bound_report.py): max |diff| / 2E = 0.125 on every lse_* fixture (the
oracle-vs-torch figure is the same), max |diff| 1.4e-4 (N = 128).
"""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
LSE_CASES = [(16, 8), (32, 16), (64, 32), (128, 64)]


def polar_for(N, info):
    from neural_polar_decoder_amd import PolarCode
    F = np.array(sorted(set(range(N)) - set(int(i) for i in info)))
    return PolarCode(int(np.log2(N)), len(info), F=F)


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def check(hat, bits, ref_hat, ref_bits, hard, what, bd):
    """bd = bound(...): the oracle's forward error bounds on the same words.  Decisions: every codeword's
    first disagreeing information bit (sc_decode: later ones follow from it through the partial sums) --
    every one for sc_decode_soft, whose decisions feed nothing -- must sit where the decision LLR is
    within 2 E of zero.  Values: on codewords whose decisions agree (all codewords for sc_decode_soft),
    hard decoded_bits bit-exact, soft ones within 2 E per entry, same NaN positions; those codewords are at least
    95 % of the batch (a coarse floor: the bound, not the floor, is the parity criterion)."""
    from oracle import oracle as O
    bad = O.unexplained_disagreements(hat, ref_hat, bd["info"], bd["leaf"], bd["eleaf"], bd["feedback"])
    assert not bad, (what, "decision flips the bound does not explain (row, k, L, E)", bad[:5])
    if ref_bits is not None:
        rows = (hat == ref_hat).all(axis=1) if bd["feedback"] else np.ones(hat.shape[0], bool)
        # coarse sanity floor beside the bound: the codewords left out of the value check below stay few
        assert rows.mean() >= 0.95, (what, "codewords with identical decisions", float(rows.mean()))
        # finiteness may differ only at leaves whose computation met an inf/NaN (the bound is then not
        # finite): there an ulp of difference decides whether exp overflows (crafted |LLR| >> 1 words)
        nb, nr = np.isnan(bits[rows]), np.isnan(ref_bits[rows])
        assert np.all((nb == nr) | ~np.isfinite(bd["eleaf"][rows])), what
        fin = ~nb & ~nr
        if hard:
            if bd["feedback"]:
                assert np.array_equal(bits[rows][fin], ref_bits[rows][fin]), what
            else:  # sign(L): may differ exactly where L is within 2 E of zero (checked above)
                same = bits[rows][fin] == ref_bits[rows][fin]
                assert np.all(same | (np.abs(bd["leaf"][rows][fin]) <= 2 * bd["eleaf"][rows][fin])), what
        else:
            err = np.abs(bits[rows][fin].astype(np.float64) - ref_bits[rows][fin])
            bound = 2.0 * bd["E"][rows][fin]
            ratio = err / np.maximum(bound, 1e-300)
            assert np.all(err <= bound), (what, "max |diff| / 2E", float(ratio.max(initial=0.0)),
                                          "max |diff|", float(err.max(initial=0.0)))


def lse_bound(y, snr, info, hard):
    from oracle import oracle as O
    _, E, leaf, eleaf = O.sc_decode_lse_bound(y, snr, info, hard, leaves=True)
    return {"E": E, "leaf": leaf, "eleaf": eleaf, "info": np.sort(np.asarray(info)), "feedback": True}


def soft_bound(y, snr, info, prior, hard):
    from oracle import oracle as O
    _, E, leaf, eleaf = O.sc_decode_soft_bound(y, snr, hard, prior, leaves=True)
    return {"E": E, "leaf": leaf, "eleaf": eleaf, "info": np.sort(np.asarray(info)), "feedback": False}


def stack(parts, d):
    """Per-SNR bound dicts -> one dict in the fixture's row order."""
    out = {k: np.empty((d["y"].shape[0],) + parts[0][1][k].shape[1:], parts[0][1][k].dtype)
           for k in ("E", "leaf", "eleaf")}
    for m, b in parts:
        for k in out:
            out[k][m] = b[k]
    out["info"], out["feedback"] = parts[0][1]["info"], parts[0][1]["feedback"]
    return out


@pytest.mark.parametrize("N,K", LSE_CASES)
def test_sc_decode_lse_golden(N, K):
    d = golden(f"lse_{N}_{K}.npz")
    code = polar_for(N, d["info"])
    for tag, hard in (("hard", True), ("soft", False)):
        hat = np.empty_like(d[f"msg_hat_{tag}"])
        bits = np.empty_like(d[f"bits_{tag}"])
        parts = []
        for s in np.unique(d["snr"]):
            m = d["snr"] == s
            h, b = code.sc_decode(t(d["y"][m]), float(s), hard_decision=hard, return_bits=True)
            hat[m], bits[m] = h.cpu().numpy(), b.cpu().numpy()
            parts.append((m, lse_bound(d["y"][m], float(s), d["info"], hard)))
        check(hat, bits, d[f"msg_hat_{tag}"], d[f"bits_{tag}"], hard, (N, tag), stack(parts, d))


def test_sc_decode_lse_args_default_is_soft():
    """hard_decision comes from args like the reference (argparse default False -> soft tanh)."""
    import argparse
    d = golden("lse_32_16.npz")
    code = polar_for(32, d["info"])
    m = d["snr"] == 1.0
    soft = code.sc_decode(t(d["y"][m]), 1.0).cpu().numpy()
    assert (soft == d["msg_hat_soft"][m]).mean() >= 0.999
    code.args = argparse.Namespace(hard_decision=True)
    hard = code.sc_decode(t(d["y"][m]), 1.0).cpu().numpy()
    assert (hard == d["msg_hat_hard"][m]).mean() >= 0.999


@pytest.mark.parametrize("N,K", [(4, 2), (8, 4), (64, 32), (128, 64), (256, 128), (64, 1), (64, 22)])
def test_sc_decode_lse_vs_oracle_random(oracle, N, K):
    """Ragged batches (64-codeword tile tails), lengths 4..256, both decision modes, the reference's
    'polar' rate profile.  Not rate-1 codes: there leaf 0's LLR is the boxplus of all N channel LLRs,
    ~1e-8 after catastrophic cancellation in log(1+e^(x+y)) - x - log(1+e^(y-x)), so its sign -- and
    every later SC decision -- is rounding noise of the reference formula itself (tools/dbg_lse.py)."""
    from neural_polar_decoder_amd.codes import polar_info_positions
    info = polar_info_positions(N, K)
    code = polar_for(N, info)
    rng = np.random.default_rng(N * 7 + K)
    for B in (1, 65, 1000):
        y = (rng.standard_normal((B, N)) * 0.8 + (1 - 2 * (rng.random((B, N)) < 0.5))).astype(np.float32)
        for hard in (True, False):
            h, b = code.sc_decode(t(y), 2.5, hard_decision=hard, return_bits=True)
            oh, ob = oracle.sc_decode_lse(y, 2.5, info, hard)
            check(h.cpu().numpy(), b.cpu().numpy(), oh, ob, hard, (N, K, B, hard), lse_bound(y, 2.5, info, hard))


def test_sc_decode_lse_full_size_properties(oracle):
    """B = 2^20, Polar(64,32): noiseless words decode to the message exactly (both modes) when the LLR
    scale keeps every partial LLR below exp's overflow (decoded at the -5 dB scale; at 2 dB the
    reference's own arithmetic overflows to inf/NaN on clean words and loses ~1 % of bits); a 2^14 sample
    of noisy words matches the oracle; the soft-decision BER at 2 dB is near the reference's measured
    figure for this decoder (0.051; the oracle gives 0.0485 on 2e4 codewords)."""
    from neural_polar_decoder_amd import reference_polar_code
    from neural_polar_decoder_amd.utils import count_errors
    code = reference_polar_code(64, 32)
    B = 1 << 20
    msg, x, y = code.mc_generate(B, 2.0, seed=21, snr_index=0, cw_offset=0, want_x=True)
    for hard in (True, False):
        assert torch.equal(code.sc_decode(x, -5.0, hard_decision=hard), msg), hard
    cnt = count_errors(msg, code.sc_decode(y, 2.0, hard_decision=False))
    ber = cnt[0].item() / (B * 32)
    assert 0.04 < ber < 0.062, ber
    ys = y[: 1 << 14]
    for hard in (True, False):
        oh, _ = oracle.sc_decode_lse(ys.cpu().numpy(), 2.0, code.info_positions, hard)
        h = code.sc_decode(ys, 2.0, hard_decision=hard).cpu().numpy()
        check(h, None, oh, None, hard, hard, lse_bound(ys.cpu().numpy(), 2.0, code.info_positions, hard))


@pytest.mark.parametrize("N,K", [(8, 4), (32, 16), (64, 32), (128, 64)])
def test_register_and_lds_variants_agree(monkeypatch, N, K):
    """N <= 128 runs the register-resident kernel; NPD_LSE_LDS=1 forces the LDS-resident one (used for
    N = 256).  Same fp32 operation sequence -> identical bits in both decision modes."""
    from neural_polar_decoder_amd import reference_polar_code
    code = reference_polar_code(N, K)
    _, _, y = code.mc_generate(3001, 1.0, seed=9, want_msg=False)
    for hard in (True, False):
        h1, b1 = code.sc_decode(y, 1.0, hard_decision=hard, return_bits=True)
        monkeypatch.setenv("NPD_LSE_LDS", "1")
        h2, b2 = code.sc_decode(y, 1.0, hard_decision=hard, return_bits=True)
        monkeypatch.delenv("NPD_LSE_LDS")
        assert torch.equal(h1, h2) and torch.equal(torch.nan_to_num(b1, nan=7.0), torch.nan_to_num(b2, nan=7.0))


def test_lse_montecarlo_driver_and_cli(capsys):
    """LSEMonteCarlo: shard invariance (3 simulated ranks == 1) and the CLI's --lse output."""
    from neural_polar_decoder_amd import reference_polar_code
    from neural_polar_decoder_amd.montecarlo import LSEMonteCarlo, _main
    code = reference_polar_code(64, 32)
    one = LSEMonteCarlo(code, [1.0, 2.0], 50_001, 20_000, seed=3, rank=0, world=1).run()
    parts = [LSEMonteCarlo(code, [1.0, 2.0], 50_001, 20_000, seed=3, rank=r, world=3).run() for r in range(3)]
    assert [sum(p.bit_errors[i] for p in parts) for i in range(2)] == one.bit_errors
    assert 0.04 < one.ber[1] < 0.062
    _main(["--test_size", "8192", "--batch_size", "4096", "--lse", "--snr_points", "2"])
    assert "BERs of exact-LSE SC decoding" in capsys.readouterr().out



@pytest.mark.parametrize("N,K", [(16, 8), (32, 16), (64, 32), (128, 64), (256, 128)])
def test_sc_decode_soft_golden(N, K):
    """PolarCode.sc_decode_soft (polar.py:281-358) vs the reference's vectors, with the fixture's priors
    ('pr') and without ('p0': frozen bits are decoded like information bits, so leaf 0's LLR is the
    boxplus of all N channel LLRs, cancellation-dominated; its sign flips only within the bound)."""
    d = golden(f"lse_soft_{N}_{K}.npz")
    code = polar_for(N, d["info"])
    for hard in (True, False):
        for ptag in ("p0", "pr"):
            tag = ("hard" if hard else "soft") + "_" + ptag
            hat = np.empty_like(d[f"msg_hat_{tag}"])
            bits = np.empty_like(d[f"bits_{tag}"])
            parts = []
            for s in np.unique(d["snr"]):
                m = d["snr"] == s
                pr = None if ptag == "p0" else d["prior"]
                h, b = code.sc_decode_soft(t(d["y"][m]), float(s), priors=pr, hard_decision=hard, return_bits=True)
                hat[m], bits[m] = h.cpu().numpy(), b.cpu().numpy()
                parts.append((m, soft_bound(d["y"][m], float(s), d["info"], pr, hard)))
            check(hat, bits, d[f"msg_hat_{tag}"], d[f"bits_{tag}"], hard, (N, tag), stack(parts, d))


def test_sc_decode_soft_vs_oracle_random(oracle):
    """Random words, ragged batches, priors from the frozen set (+20) plus noise, N = 8..64."""
    from neural_polar_decoder_amd.codes import polar_info_positions
    for N, K in [(8, 4), (32, 16), (64, 32), (64, 22), (128, 64), (256, 128)]:
        info = polar_info_positions(N, K)
        code = polar_for(N, info)
        rng = np.random.default_rng(N + 3 * K)
        prior = np.zeros(N, np.float32)
        prior[np.setdiff1d(np.arange(N), info)] = 20.0
        prior += rng.standard_normal(N).astype(np.float32)
        for B in (1, 65, 1000):
            y = (rng.standard_normal((B, N)) * 0.8 + (1 - 2 * (rng.random((B, N)) < 0.5))).astype(np.float32)
            for hard in (True, False):
                h, b = code.sc_decode_soft(t(y), 2.5, priors=prior, hard_decision=hard, return_bits=True)
                oh, ob = oracle.sc_decode_soft(y, 2.5, info, hard, prior)
                check(h.cpu().numpy(), b.cpu().numpy(), oh, ob, hard, (N, K, B, hard), soft_bound(y, 2.5, info, prior, hard))


def soft_new_bound(y, snr, info, prior):
    from oracle import oracle as O
    _, E, leaf, eleaf = O.sc_decode_soft_bound(y, snr, True, prior, leaves=True, twice=True)
    return {"E": E, "leaf": leaf, "eleaf": eleaf, "info": np.sort(np.asarray(info)), "feedback": False}


@pytest.mark.parametrize("N,K", [(16, 8), (32, 16), (64, 32), (128, 64), (256, 128)])
def test_sc_decode_soft_new_golden(N, K):
    """PolarCode.sc_decode_soft_new (polar.py:485-607) vs the reference's vectors: decoded_bits (its return
    value) and u_hat = sign of every stored leaf.  Its decisions feed nothing (the partial sums are the leaf
    LLRs), so every disagreement must sit where the stored leaf LLR is within 2 E of zero."""
    d = golden(f"soft_new_{N}_{K}.npz")
    code = polar_for(N, d["info"])
    for ptag in ("p0", "pr"):
        pr = None if ptag == "p0" else d["prior"]
        hat = np.empty_like(d[f"msg_hat_{ptag}"])
        u = np.empty_like(d[f"leaf_{ptag}"])
        parts = []
        for s in np.unique(d["snr"]):
            m = d["snr"] == s
            h, uh = code.sc_decode_soft_new(t(d["y"][m]), float(s), priors=pr, return_u_hat=True)
            hat[m], u[m] = h.cpu().numpy(), uh.cpu().numpy()
            parts.append((m, soft_new_bound(d["y"][m], float(s), d["info"], pr)))
        check(hat, u, d[f"msg_hat_{ptag}"], np.sign(d[f"leaf_{ptag}"]), True, (N, ptag), stack(parts, d))


def test_sc_decode_soft_new_vs_oracle_random(oracle):
    """Ragged batches, N = 8..256, priors None and frozen-heavy; also host-tensor input (staged to the GPU,
    result back on the host) and the (B,K) return shape."""
    from neural_polar_decoder_amd.codes import polar_info_positions
    for N, K in [(8, 4), (32, 16), (64, 32), (128, 64), (256, 128)]:
        info = polar_info_positions(N, K)
        code = polar_for(N, info)
        rng = np.random.default_rng(5 * N + K)
        prior = np.zeros(N, np.float32)
        prior[np.setdiff1d(np.arange(N), info)] = 20.0
        prior += rng.standard_normal(N).astype(np.float32)
        for B in (1, 65, 700):
            y = (rng.standard_normal((B, N)) * 0.8 + (1 - 2 * (rng.random((B, N)) < 0.5))).astype(np.float32)
            for pr in (None, prior):
                h, u = code.sc_decode_soft_new(t(y), 2.5, priors=pr, return_u_hat=True)
                oh, leaf = oracle.sc_decode_soft_new(y, 2.5, info, pr)
                check(h.cpu().numpy(), u.cpu().numpy(), oh, np.sign(leaf), True, (N, K, B, pr is None),
                      soft_new_bound(y, 2.5, info, pr))
        hc = code.sc_decode_soft_new(torch.from_numpy(y), 2.5, priors=torch.from_numpy(prior))
        assert hc.device.type == "cpu" and hc.shape == (y.shape[0], K)
        assert torch.equal(hc, code.sc_decode_soft_new(t(y), 2.5, priors=prior).cpu())


def test_sc_decode_soft_new_register_and_lds_agree(monkeypatch):
    """N <= 64 runs the register-resident kernel, NPD_SOFT_LDS=1 the LDS one: identical bits."""
    from neural_polar_decoder_amd import reference_polar_code
    for N, K in [(16, 8), (64, 32)]:
        code = reference_polar_code(N, K)
        _, _, y = code.mc_generate(2001, 1.0, seed=4, want_msg=False)
        pr = np.linspace(-3, 3, N).astype(np.float32)
        h1, u1 = code.sc_decode_soft_new(y, 1.0, priors=pr, return_u_hat=True)
        monkeypatch.setenv("NPD_SOFT_LDS", "1")
        h2, u2 = code.sc_decode_soft_new(y, 1.0, priors=pr, return_u_hat=True)
        monkeypatch.delenv("NPD_SOFT_LDS")
        assert torch.equal(h1, h2) and torch.equal(u1, u2)
