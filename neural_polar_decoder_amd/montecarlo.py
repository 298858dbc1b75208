"""BER/BLER Monte-Carlo evaluation, sharded over GPUs.

The reference's eval loops (run_models.py:297-371 ``testXformer``, rnn_all.py:821-961
``polar_RNN_full_test``) draw a message batch, encode, pass it through AWGN at every SNR of
``linspace(start, end, points)`` (run_models.py:1329-1333), decode, and average per-batch
``errors_ber`` / ``errors_bler`` over equal-sized batches (== pooled counts).

Here every codeword has a global index g; its message bits and channel noise are Philox streams keyed
by (seed, g) and (seed, SNR index, g), so a run is identical for any number of ranks.  Rank r
decodes the contiguous index range ``shard_range(total, r, world)``; counters stay on the device
({bit errors, block errors} per SNR, uint64) and are summed by ONE all-reduce at the end (RCCL over
xGMI with the ``nccl`` backend; gloo on CPU tests).  No data-path collective exists.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys

import numpy as np
import torch


def snr_range(start: float, end: float, points: int):
    """run_models.py:1329-1333 / rnn_all.py:1765-1769."""
    if points == 1:
        return [start]
    step = (end - start) * 1.0 / (points - 1)
    return [step * i + start for i in range(points)]


def shard_range(total: int, rank: int, world: int):
    """Contiguous, balanced partition of [0, total) over `world` ranks -> (start, count)."""
    base, rem = divmod(int(total), int(world))
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


@dataclasses.dataclass
class MCResult:
    snrs: list
    bit_errors: list
    block_errors: list
    codewords: int
    K: int

    @property
    def ber(self):
        return [b / (self.codewords * self.K) for b in self.bit_errors]

    @property
    def bler(self):
        return [b / self.codewords for b in self.block_errors]

    def as_dict(self):
        return {"snr": self.snrs, "ber": self.ber, "bler": self.bler, "bit_errors": self.bit_errors,
                "block_errors": self.block_errors, "codewords": self.codewords, "K": self.K}


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


class MonteCarlo:
    """Sharded MC driver.  Subclasses provide ``count_batch(si, snr, cw_offset, n, counters_row)``."""

    def __init__(self, K: int, snrs, total_cw: int, batch: int, seed: int = 1234, rank=None, world=None, device=None):
        d = _dist()
        self.rank = d.get_rank() if (rank is None and d) else (rank or 0)
        self.world = d.get_world_size() if (world is None and d) else (world or 1)
        self.K = K
        self.snrs = [float(s) for s in snrs]
        self.total = int(total_cw)
        self.batch = int(batch)
        self.seed = int(seed)
        self.device = device

    def new_counters(self):
        return torch.zeros(len(self.snrs), 2, dtype=torch.int64, device=self.device)

    def count_batch(self, si, snr, cw_offset, n, counters_row):  # pragma: no cover - abstract
        raise NotImplementedError

    def count_sweep(self, cw_offset, n, counters):
        """All SNR points of one batch; the default runs count_batch per SNR."""
        for si, snr in enumerate(self.snrs):
            self.count_batch(si, snr, cw_offset, n, counters[si])

    def run(self) -> MCResult:
        start, count = shard_range(self.total, self.rank, self.world)
        counters = self.new_counters()
        for off in range(0, count, self.batch):
            n = min(self.batch, count - off)
            self.count_sweep(start + off, n, counters)
        d = _dist()
        if d is not None and self.world > 1:
            d.all_reduce(counters)  # the one collective of the run
        c = counters.cpu().numpy()
        return MCResult(self.snrs, [int(v) for v in c[:, 0]], [int(v) for v in c[:, 1]], self.total, self.K)


class SCMonteCarlo(MonteCarlo):
    """Polar / PAC SC decoding: fused generate (npd_mc_generate) + decode-and-count (npd_sc_decode_mc)."""

    def __init__(self, code, snrs, total_cw, batch, seed=1234, rank=None, world=None, device=None, fused=True):
        device = torch.device(device or "cuda")
        super().__init__(code.K, snrs, total_cw, batch, seed, rank, world, device)
        self.code = code
        self._y = None
        # generation fused into the decode kernel (npd_sc_mc_sweep_fused), y never stored: the codes the fused
        # kernels cover (code.fused_mc_supported, the same rule as the C ABI's)
        self.fused = (bool(fused) and hasattr(code, "sc_mc_sweep_fused") and len(self.snrs) <= 16
                      and getattr(code, "fused_mc_supported", lambda: False)())

    def count_batch(self, si, snr, cw_offset, n, counters_row):
        _, _, y = self.code.mc_generate(n, snr, self.seed, si, cw_offset, device=self.device, want_msg=False)
        self.code.sc_decode_mc(y, snr, self.seed, cw_offset, counters_row)

    def count_sweep(self, cw_offset, n, counters):
        if self.fused:
            self.code.sc_mc_sweep_fused(n, self.snrs, self.seed, cw_offset, counters)
            return
        if not hasattr(self.code, "sc_decode_mc_sweep") or len(self.snrs) > 16:
            return super().count_sweep(cw_offset, n, counters)
        # Polar: every SNR point of the batch in one decode launch (npd_sc_decode_mc_sweep)
        if self._y is None or self._y.shape[1] != n:
            self._y = torch.empty(len(self.snrs), n, self.code.N, dtype=torch.float32, device=self.device)
        y = self._y
        for si, snr in enumerate(self.snrs):
            self.code.mc_generate(n, snr, self.seed, si, cw_offset, want_msg=False, out=y[si])
        self.code.sc_decode_mc_sweep(y, self.snrs, self.seed, cw_offset, counters)


class SCLMonteCarlo(SCMonteCarlo):
    """Polar SC-List decoding (polar.py:793-876, run_models.py:327-331): fused generate +
    npd_scl_decode_mc (decode and count in one launch)."""

    def __init__(self, code, list_size, snrs, total_cw, batch, seed=1234, rank=None, world=None, device=None):
        super().__init__(code, snrs, total_cw, batch, seed, rank, world, device, fused=False)
        self.list_size = int(list_size)

    def count_batch(self, si, snr, cw_offset, n, counters_row):
        _, _, y = self.code.mc_generate(n, snr, self.seed, si, cw_offset, device=self.device, want_msg=False)
        self.code.scl_decode_mc(y, snr, self.list_size, self.seed, cw_offset, counters_row)

    def count_sweep(self, cw_offset, n, counters):
        return MonteCarlo.count_sweep(self, cw_offset, n, counters)


class LSEMonteCarlo(SCMonteCarlo):
    """Exact-LSE SC decoding (PolarCode.sc_decode, polar.py:209-279; hard or soft decisions): fused
    generate + npd_sc_decode_lse + device error counting."""

    def __init__(self, code, snrs, total_cw, batch, seed=1234, hard_decision=False, rank=None, world=None,
                 device=None):
        super().__init__(code, snrs, total_cw, batch, seed, rank, world, device, fused=False)
        self.hard_decision = bool(hard_decision)

    def count_batch(self, si, snr, cw_offset, n, counters_row):
        from .utils import count_errors
        msg, _, y = self.code.mc_generate(n, snr, self.seed, si, cw_offset, device=self.device, want_msg=True)
        count_errors(msg, self.code.sc_decode(y, snr, hard_decision=self.hard_decision), counters_row)

    def count_sweep(self, cw_offset, n, counters):
        return MonteCarlo.count_sweep(self, cw_offset, n, counters)


class DecoderMonteCarlo(MonteCarlo):
    """A neural decoder's Monte-Carlo: fused generation (npd_mc_generate, message kept), the decoder's
    (n, N) decisions, and decisions[:, info] counted against the message on the device
    (errors_ber / errors_bler semantics, utils.py:17-51).  Subclasses provide ``decisions(y)``."""

    def __init__(self, code, snrs, total_cw, batch, seed=1234, rank=None, world=None, device=None):
        device = torch.device(device or "cuda")
        super().__init__(code.K, snrs, total_cw, batch, seed, rank, world, device)
        self.code = code
        info = getattr(code, "info_positions", None)
        self.info_np = np.asarray(info if info is not None else code.B, dtype=np.int64)
        self.info = torch.as_tensor(self.info_np, device=device)

    def generate(self, si, snr, cw_offset, n):
        msg, _, y = self.code.mc_generate(n, snr, self.seed, si, cw_offset, device=self.device, want_msg=True)
        return msg, y

    def decisions(self, y):  # pragma: no cover - abstract
        raise NotImplementedError

    def count(self, msg, dec, counters_row):
        """msg (n,K) vs the decisions' information columns dec[:, info] (n,N), not gathered."""
        from .utils import count_errors
        count_errors(msg, dec, counters_row, cols=self.info_np)

    def count_batch(self, si, snr, cw_offset, n, counters_row):
        msg, y = self.generate(si, snr, cw_offset, n)
        self.count(msg, self.decisions(y), counters_row)


class GRUMonteCarlo(DecoderMonteCarlo):
    """CRISP GRU decoding (rnn_all.py:874-878 Polar; rnn_all.py:679-700 PAC): decoded[:, info] vs the
    message."""

    def __init__(self, code, net, decoder, snrs, total_cw, batch, seed=1234, rank=None, world=None, device=None):
        super().__init__(code, snrs, total_cw, batch, seed, rank, world, device)
        self.net, self.decoder = net, decoder

    def decisions(self, y):
        return self.decoder.decode(self.net, False, y)

    def count_sweep(self, cw_offset, n, counters):
        """Every SNR point of the batch in one decode-and-count launch (npd_gru_decode_count_sweep, rnn_all.py:853-880)
        for y_input nets without the y-MLP; the messages are the same for every point (keyed by codeword)."""
        if self.decoder.decoding_type != "y_input" or getattr(self.net, "y_depth", 0) > 0:
            return super().count_sweep(cw_offset, n, counters)
        y = torch.empty(len(self.snrs), n, self.code.N, dtype=torch.float32, device=self.device)
        msg = None
        for si, snr in enumerate(self.snrs):
            m, _, _ = self.code.mc_generate(n, snr, self.seed, si, cw_offset, want_msg=msg is None, out=y[si])
            msg = m if msg is None else msg
        self.decoder.decode_count_sweep(self.net, y, msg, counters, cols=self.info_np)


class ConvMonteCarlo(DecoderMonteCarlo):
    """convNet decoding (run_models.py:333-337, testXformer): sign of the LayerNorm output at the info
    positions vs the message."""

    def __init__(self, code, net, snrs, total_cw, batch, seed=1234, rank=None, world=None, device=None):
        super().__init__(code, snrs, total_cw, batch, seed, rank, world, device)
        self.net = net

    def decisions(self, y):
        return self.net.logits(y)[1]


def seeded_crisp(code, feature_size=64, depth=2, seed=0, device="cuda", onehot=True, precision="fp32"):
    """(net, RNN_decoder) with PyTorch-default-initialised weights under torch.manual_seed(seed): the
    reference ships no trained checkpoint (rnn_all.py:294-398 architecture, y_input + onehot)."""
    from .rnn import RNN_Model, RNN_decoder
    N = code.N
    torch.manual_seed(seed)
    net = RNN_Model("GRU", N + 1 + int(onehot), feature_size, 1, depth, N, 0, 0).to(device).eval()
    info = getattr(code, "info_positions", None)
    dec = RNN_decoder("y_input", N, np.asarray(info if info is not None else code.B), onehot=onehot,
                      precision=precision)
    return net, dec


def seeded_conv(N, embed_dim=128, seed=0, device="cuda"):
    """convNet (models.py:691-772) with PyTorch-default-initialised weights under torch.manual_seed(seed)."""
    from .models import convNet
    torch.manual_seed(seed)
    cfg = argparse.Namespace(embed_dim=embed_dim, max_len=N, N=N, dont_use_bias=False, dropout=0.0)
    return convNet(cfg).to(device).eval()


def _main(argv=None):
    ap = argparse.ArgumentParser(description="MI355X BER/BLER Monte-Carlo (SC, SC-List, exact-LSE SC, CRISP GRU, "
                                             "convNet decoders)")
    ap.add_argument("--code", choices=["polar", "pac"], default="polar")
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--K", type=int, default=32)
    ap.add_argument("--rate_profile", default="polar")
    ap.add_argument("--target_K", type=int, default=None)
    ap.add_argument("--g", type=int, default=None, help="PAC polynomial (default: the reference scripts' choice for N, "
                                                         "codes.pac_default_g: 53 at N = 32, 91 from N = 64)")
    ap.add_argument("--test_snr_start", type=float, default=0.0)
    ap.add_argument("--test_snr_end", type=float, default=4.0)
    ap.add_argument("--snr_points", type=int, default=5)
    ap.add_argument("--test_size", type=int, default=1 << 20)
    ap.add_argument("--batch_size", type=int, default=1 << 20)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--list_size", type=int, default=None, help="also run SC-List with this list size (Polar)")
    ap.add_argument("--lse", action="store_true", help="also run the exact-LSE sc_decode (Polar, polar.py:209)")
    ap.add_argument("--hard_decision", action="store_true", help="exact-LSE SC with sign decisions (else tanh)")
    ap.add_argument("--crisp", action="store_true", help="also run the CRISP GRU decoder (rnn_all.py:874)")
    ap.add_argument("--crisp_checkpoint", default=None, help="rnn_all.py checkpoint ({'net', 'args'}) for --crisp")
    ap.add_argument("--rnn_feature_size", type=int, default=64, help="--crisp without checkpoint: hidden size")
    ap.add_argument("--rnn_depth", type=int, default=2, help="--crisp without checkpoint: GRU layers")
    ap.add_argument("--conv", action="store_true", help="also run the convNet decoder (run_models.py:333)")
    ap.add_argument("--conv_checkpoint", default=None, help="run_models.py checkpoint ({'xformer', 'args'}) for --conv")
    ap.add_argument("--embed_dim", type=int, default=128, help="--conv without checkpoint: channels")
    ap.add_argument("--init_seed", type=int, default=0, help="torch seed of the untrained (seeded) decoder weights")
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from .codes import pac_default_g, polar_info_positions
    from .pac_code import PAC
    if a.g is None:
        a.g = pac_default_g(a.N)
    from .polar import PolarCode
    if a.code == "polar":
        info = polar_info_positions(a.N, a.K, a.rate_profile, a.target_K)
        F = np.setdiff1d(np.arange(a.N), info)
        code = PolarCode(int(np.log2(a.N)), a.K, F=F)
    else:
        code = PAC(argparse.Namespace(target_K=a.target_K or a.K), a.N, a.K, a.g)
    snrs = snr_range(a.test_snr_start, a.test_snr_end, a.snr_points)
    res = SCMonteCarlo(code, snrs, a.test_size, a.batch_size, a.seed).run()
    scl = None
    if a.list_size:
        if a.code != "polar":
            raise SystemExit("--list_size: SC-List is defined for Polar codes only (polar.py:793)")
        scl = SCLMonteCarlo(code, a.list_size, snrs, a.test_size, a.batch_size, a.seed).run()
    lse = None
    if a.lse:
        if a.code != "polar":
            raise SystemExit("--lse: the exact-LSE sc_decode is defined for Polar codes only (polar.py:209)")
        lse = LSEMonteCarlo(code, snrs, a.test_size, a.batch_size, a.seed, hard_decision=a.hard_decision).run()
    crisp = None
    if a.crisp:
        if a.crisp_checkpoint:
            from .datasets import rnn_from_checkpoint
            net, dec, ccode = rnn_from_checkpoint(a.crisp_checkpoint)
            if ccode.N != a.N or ccode.K != a.K:
                raise SystemExit("--crisp_checkpoint was trained for a different (N, K)")
            # messages are generated and counted on `code`; the checkpoint's decoder reads its own info set
            # (args.rate_profile), so the two codes must be the same code, not just the same (N, K)
            cinfo = np.asarray(getattr(ccode, "info_positions", None) if a.code == "polar" else ccode.B)
            info = np.asarray(code.info_positions if a.code == "polar" else code.B)
            if not np.array_equal(np.sort(cinfo), np.sort(info)):
                raise SystemExit("--crisp_checkpoint's information set (its rate profile) differs from the CLI code's "
                                 "(--rate_profile/--target_K)")
            if a.code == "pac" and getattr(ccode, "g", a.g) != a.g:
                raise SystemExit("--crisp_checkpoint's PAC convolution polynomial differs from --g")
        else:
            net, dec = seeded_crisp(code, a.rnn_feature_size, a.rnn_depth, a.init_seed)
        crisp = GRUMonteCarlo(code, net, dec, snrs, a.test_size, a.batch_size, a.seed).run()
    conv = None
    if a.conv:
        if a.conv_checkpoint:
            from .datasets import convnet_from_checkpoint
            cnet = convnet_from_checkpoint(a.conv_checkpoint)
        else:
            cnet = seeded_conv(a.N, a.embed_dim, a.init_seed)
        conv = ConvMonteCarlo(code, cnet, snrs, a.test_size, a.batch_size, a.seed).run()
    if _dist() is None or _dist().get_rank() == 0:
        print("Test SNRs : ", snrs)
        if crisp is not None:
            print("BERs of RNN: {0}".format(crisp.ber))
        if conv is not None:
            print("BERs of Xformer: {0}".format(conv.ber))
        print("BERs of SC decoding: {0}".format(res.ber))
        print("BLERs of SC decoding: {0}".format(res.bler))
        rec = {"sc": res.as_dict()}
        if scl is not None:
            print("BERs of SCL decoding: {0}".format(scl.ber))
            print("BLERs of SCL decoding: {0}".format(scl.bler))
            rec["scl"] = dict(scl.as_dict(), list_size=a.list_size)
        if lse is not None:
            print("BERs of exact-LSE SC decoding: {0}".format(lse.ber))
            print("BLERs of exact-LSE SC decoding: {0}".format(lse.bler))
            rec["sc_lse"] = dict(lse.as_dict(), hard_decision=a.hard_decision)
        if crisp is not None:
            print("BLERs of RNN: {0}".format(crisp.bler))
            rec["crisp_gru"] = crisp.as_dict()
        if conv is not None:
            print("BLERs of Xformer: {0}".format(conv.bler))
            rec["conv"] = conv.as_dict()
        print(json.dumps(rec))
    return res


if __name__ == "__main__":
    sys.exit(0 if _main() else 1)
