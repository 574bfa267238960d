"""bench.py's launcher contract (CPU): `--gpus N` without a launcher starts N
ranks itself, a WORLD_SIZE that disagrees with --gpus is an error, and a host
with fewer GPUs than ranks fails loudly instead of measuring one GPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "HM_BENCH_DRY")}
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True, timeout=300)


def test_gpus_n_spawns_n_ranks():
    r = _run(["--gpus", "3"], HM_BENCH_DRY="1")
    assert r.returncode == 0, r.stderr
    ranks = sorted(json.loads(x)["rank"] for x in r.stdout.split("\n") if x.startswith("{"))
    assert ranks == [0, 1, 2]


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2"], WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE=4 but --gpus 2" in r.stderr


def test_too_few_gpus_is_an_error():
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has the GPUs")
    r = _run(["--gpus", "2"])
    assert r.returncode == 2
    assert "needs 2 visible GPUs" in r.stderr
