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


@pytest.mark.parametrize("world", [2, 3])  # 3: shards of unequal size (3000 words)
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


# ------------------------------------------------------------------ neural decoders (CRISP GRU, convNet)
def _oracle_decoder_mc(kind, rank=None, world=None):
    """GRUMonteCarlo / ConvMonteCarlo with the per-batch device work (generation, decode, count)
    replaced by the CPU oracle; sharding, info-column selection and the counter all-reduce are the
    drivers' own."""
    import argparse
    from neural_polar_decoder_amd import PAC, reference_polar_code
    from neural_polar_decoder_amd.montecarlo import ConvMonteCarlo, GRUMonteCarlo, MonteCarlo, seeded_conv, seeded_crisp
    from oracle import oracle as O
    if kind == "gru_pac":
        code = PAC(argparse.Namespace(target_K=64), 128, 64, 91)
    else:
        code = reference_polar_code(64, 32)
    info = np.asarray(getattr(code, "info_positions", None) if kind != "gru_pac" else code.B)
    if kind.startswith("gru"):
        net, dec = seeded_crisp(code, feature_size=32, depth=2, seed=3, device="cpu")
        sd = {k: v.detach().numpy() for k, v in net.state_dict().items()}
        base = GRUMonteCarlo
        args = (code, net, dec)

        def decide(y):
            return O.gru_decode(y, sd, code.N, 32, 2, info, onehot=True)
    else:
        net = seeded_conv(64, embed_dim=16, seed=3, device="cpu")
        sd = {k: v.detach().numpy() for k, v in net.state_dict().items()}
        base = ConvMonteCarlo
        args = (code, net)

        def decide(y):
            return np.sign(O.conv_forward(y, sd))

    class _MC(base):
        def generate(self, si, snr, cw_offset, n):
            msg = O.gen_msg(n, code.K, self.seed, cw_offset)
            x = O.pac_encode(msg, code.N, info) if kind == "gru_pac" else O.encode_plotkin(msg, code.N, info)
            return torch.from_numpy(msg), torch.from_numpy(O.awgn(x, snr, self.seed, si, cw_offset))

        def decisions(self, y):
            return torch.from_numpy(np.ascontiguousarray(decide(y.numpy()), dtype=np.float32))

        def count(self, msg, dec, row):
            be, bl = O.count_errors(msg.numpy(), np.ascontiguousarray(dec.numpy()[:, self.info_np]))
            row[0] += be
            row[1] += bl

        def count_sweep(self, cw_offset, n, counters):
            # the per-SNR-point path (GRUMonteCarlo's one-launch sweep is a device kernel: test_gru_sweep_gpu.py)
            MonteCarlo.count_sweep(self, cw_offset, n, counters)

    return _MC(*args, [0.0, 3.0], 300, 64, 77, rank=rank, world=world, device="cpu")


def _decoder_worker(rank, world, port, kind, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    res = _oracle_decoder_mc(kind).run()
    q.put((rank, res.bit_errors, res.block_errors))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["gru_polar", "gru_pac", "conv"])
def test_gloo_decoder_montecarlo_sharded(kind):
    """world 2 over gloo == one process, for the CRISP GRU (Polar(64,32), PAC(128,64)) and convNet
    Monte-Carlo drivers (the configs[3] / configs[4] multi-GPU legs)."""
    single = _oracle_decoder_mc(kind, rank=0, world=1).run()
    assert sum(single.block_errors) > 0  # seeded, untrained weights: errors occur
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_decoder_worker, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, be, bl in out:
        assert be == single.bit_errors and bl == single.block_errors, (kind, rank, be, single.bit_errors)
