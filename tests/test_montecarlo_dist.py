"""CPU (gloo, world_size 2): the Monte-Carlo sharding + single counter all-reduce give exactly the
single-process result.  The per-batch decoder here is the CPU oracle (fused Philox msg -> encode ->
AWGN -> SC -> count), standing in for the GPU kernels the driver calls on the MI355X."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT


class OracleMC:
    @staticmethod
    def make(N, K, snrs, total, batch, seed, rank=None, world=None):
        from neural_polar_decoder_amd.codes import polar_info_positions
        from neural_polar_decoder_amd.montecarlo import MonteCarlo
        from oracle import oracle as O
        info = polar_info_positions(N, K)

        class _MC(MonteCarlo):
            def count_batch(self, si, snr, cw_offset, n, row):
                be, bl = O.mc_sc(n, N, info, snr, self.seed, si, cw_offset)
                row[0] += be
                row[1] += bl

        return _MC(K, snrs, total, batch, seed, rank, world, device="cpu")


def test_shard_range_partition():
    from neural_polar_decoder_amd.montecarlo import shard_range
    for total in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            parts = [shard_range(total, r, world) for r in range(world)]
            assert sum(c for _, c in parts) == total
            pos = 0
            for s, c in parts:
                assert s == pos
                pos += c


def test_snr_range_matches_reference_formula():
    from neural_polar_decoder_amd.montecarlo import snr_range
    assert snr_range(-2.0, 4.0, 7) == [-2.0, -1.0, 0.0, 1.0, 2.0, 3.0, 4.0]
    assert snr_range(0.0, 4.0, 1) == [0.0]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    O.set_num_threads(2)
    res = OracleMC.make(64, 32, [0.0, 2.0], 3000, 512, 99).run()
    q.put((rank, res.bit_errors, res.block_errors))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_equals_single_process(world):
    from oracle import oracle as O
    O.set_num_threads(2)
    single = OracleMC.make(64, 32, [0.0, 2.0], 3000, 512, 99, rank=0, world=1).run()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, be, bl in out:  # every rank holds the reduced totals
        assert be == single.bit_errors and bl == single.block_errors, (rank, be, single.bit_errors)
