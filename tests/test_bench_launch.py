"""bench.py's launcher contract on CPU: ``--gpus N`` without a launcher starts N ranks through
torch.distributed.run (the parent never touches the GPU), and a launcher world size that differs from
--gpus is refused before any GPU call."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run(args, env=None, timeout=180):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=timeout, cwd=ROOT)


def test_self_launch_starts_n_ranks():
    r = _run(["--gpus", "2", "--launch-probe"])
    assert r.returncode == 0, r.stderr[-2000:]
    seen = sorted(json.loads(l)["rank"] for l in r.stdout.splitlines() if l.startswith("{"))
    worlds = {json.loads(l)["world"] for l in r.stdout.splitlines() if l.startswith("{")}
    assert seen == [0, 1] and worlds == {2}, r.stdout


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "4", "--launch-probe"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_single_rank_default():
    r = _run(["--launch-probe"])
    assert r.returncode == 0 and json.loads(r.stdout.strip().splitlines()[-1]) == {"rank": 0, "world": 1}


@pytest.mark.gpu
def test_two_ranks_on_one_gpu_rehearsal():
    """The N > 1 bench path end to end on one MI355X (the driver's 8-GPU scaling run uses it over RCCL): two ranks
    launched by bench.py itself, both on cuda:0 over gloo (NPD_BENCH_SHARE_GPU / NPD_BENCH_BACKEND), weak scaling --
    rank 0 prints one line whose value counts both ranks' codewords, with per-rank times and a 2-rank world."""
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "65536", "--no-traffic", "--no-cpu-baseline",
              "--no-gru", "--no-pac", "--no-conv", "--no-scl", "--no-lse", "--no-mc",
              "--full-json", os.path.join(ROOT, "gpurun_out", "bench_full_2rank.json")],
             env={"NPD_BENCH_BACKEND": "gloo", "NPD_BENCH_SHARE_GPU": "1"}, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    d = lines[0]
    assert d["n_gpus"] == 2 and d["world_size_rccl"] == 2 and len(d["rank_ms_per_step"]) == 2
    assert d["value"] > 0 and abs(d["value"] * d["ms_per_step"] / 1e3 - 2 * 5 * 65536) < 1e-3 * 2 * 5 * 65536
    assert d["configs_summary"]["1_sc_decode"]["ber_match_0.05dB"] is not None
