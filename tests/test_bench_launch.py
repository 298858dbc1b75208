"""bench.py's launcher contract on CPU: ``--gpus N`` without a launcher starts N ranks through
torch.distributed.run (the parent never touches the GPU), and a launcher world size that differs from
--gpus is refused before any GPU call."""
import json
import os
import subprocess
import sys

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
