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

    def __init__(self, code, snrs, total_cw, batch, seed=1234, rank=None, world=None, device=None):
        device = torch.device(device or "cuda")
        super().__init__(code.K, snrs, total_cw, batch, seed, rank, world, device)
        self.code = code
        self._y = None

    def count_batch(self, si, snr, cw_offset, n, counters_row):
        _, _, y = self.code.mc_generate(n, snr, self.seed, si, cw_offset, device=self.device, want_msg=False)
        self.code.sc_decode_mc(y, snr, self.seed, cw_offset, counters_row)

    def count_sweep(self, cw_offset, n, counters):
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
        super().__init__(code, snrs, total_cw, batch, seed, rank, world, device)
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
        super().__init__(code, snrs, total_cw, batch, seed, rank, world, device)
        self.hard_decision = bool(hard_decision)

    def count_batch(self, si, snr, cw_offset, n, counters_row):
        from .utils import count_errors
        msg, _, y = self.code.mc_generate(n, snr, self.seed, si, cw_offset, device=self.device, want_msg=True)
        count_errors(msg, self.code.sc_decode(y, snr, hard_decision=self.hard_decision), counters_row)

    def count_sweep(self, cw_offset, n, counters):
        return MonteCarlo.count_sweep(self, cw_offset, n, counters)


class GRUMonteCarlo(MonteCarlo):
    """CRISP GRU decoding (rnn_all.py:874-878): decoded[:, info] vs the message, counted on device."""

    def __init__(self, code, net, decoder, snrs, total_cw, batch, seed=1234, rank=None, world=None, device=None):
        device = torch.device(device or "cuda")
        super().__init__(code.K, snrs, total_cw, batch, seed, rank, world, device)
        self.code, self.net, self.decoder = code, net, decoder
        info = getattr(code, "info_positions", None)
        self.info = torch.as_tensor(np.asarray(info if info is not None else code.B), device=device)

    def count_batch(self, si, snr, cw_offset, n, counters_row):
        from .utils import count_errors
        msg, _, y = self.code.mc_generate(n, snr, self.seed, si, cw_offset, device=self.device, want_msg=True)
        dec = self.decoder.decode(self.net, False, y)
        count_errors(msg, dec.index_select(1, self.info), counters_row)


def _main(argv=None):
    ap = argparse.ArgumentParser(description="MI355X BER/BLER Monte-Carlo (SC decoding)")
    ap.add_argument("--code", choices=["polar", "pac"], default="polar")
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--K", type=int, default=32)
    ap.add_argument("--rate_profile", default="polar")
    ap.add_argument("--target_K", type=int, default=None)
    ap.add_argument("--g", type=int, default=91)
    ap.add_argument("--test_snr_start", type=float, default=0.0)
    ap.add_argument("--test_snr_end", type=float, default=4.0)
    ap.add_argument("--snr_points", type=int, default=5)
    ap.add_argument("--test_size", type=int, default=1 << 20)
    ap.add_argument("--batch_size", type=int, default=1 << 20)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--list_size", type=int, default=None, help="also run SC-List with this list size (Polar)")
    ap.add_argument("--lse", action="store_true", help="also run the exact-LSE sc_decode (Polar, polar.py:209)")
    ap.add_argument("--hard_decision", action="store_true", help="exact-LSE SC with sign decisions (else tanh)")
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from .codes import polar_info_positions
    from .pac_code import PAC
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
    if _dist() is None or _dist().get_rank() == 0:
        print("Test SNRs : ", snrs)
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
        print(json.dumps(rec))
    return res


if __name__ == "__main__":
    sys.exit(0 if _main() else 1)
