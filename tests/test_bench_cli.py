"""bench.py's multi-GPU contract (BASELINE.json configs[3]).

`python bench.py --gpus N` is the driver's form for every N.  It must either run N ranks, one
per GPU, and print a line with n_gpus = N and N per_gpu entries, or exit non-zero -- never a
silent one-GPU line.  CPU cases check the refusals; GPU cases run the launcher for real: with
two GPUs on two devices, and on any box as the one-GPU rehearsal (NETC_BENCH_DEVICE=0: both
ranks on device 0, gloo for the timing collectives), which drives the same child launch.
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=120):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=ROOT)


def _gpus():
    import torch

    return torch.cuda.device_count()


def test_gpus_more_than_visible_exits_nonzero():
    if _gpus() >= 2:
        pytest.skip("two GPUs visible: the refusal case cannot be provoked here")
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1"])
    assert r.returncode != 0
    assert '"n_gpus"' not in r.stdout
    assert "GPU(s) visible" in r.stderr


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_gpus_zero_rejected():
    r = _run(["--gpus", "0"])
    assert r.returncode == 2


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def _check_line(line, n):
    assert line["n_gpus"] == n
    assert len(line["per_gpu"]) == n
    assert line["verified"]["ranks_verified"] == n and line["verified"]["all_ranks_ok"]
    sh = line["c4_shards"]
    assert sh is not None and len(sh["per_gpu"]) == n and sh["verified_all_ranks"]
    assert line["value"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_gpus_distinct_devices():
    if _gpus() < 2:
        pytest.skip("needs two GPUs")
    r = _run(["--gpus", "2", "--steps", "5", "--warmup", "2", "--c5-gib", "0", "--cpu-seconds", "0",
              "--no-copy-ceiling"], timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    _check_line(line, 2)
    assert line["config"]["devices"] == "one GPU per rank"


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_launcher_rehearsal_one_gpu():
    """The child-launch path on a one-GPU box: `python bench.py --gpus 2` with both ranks on
    device 0 (the rehearsal switch only skips the device count and pins the device)."""
    r = _run(["--gpus", "2", "--steps", "5", "--warmup", "2", "--c5-gib", "0", "--cpu-seconds", "0",
              "--no-copy-ceiling"], {"NETC_BENCH_DEVICE": "0", "NETC_BENCH_BACKEND": "gloo"}, timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    _check_line(line, 2)
    assert line["config"]["devices"].startswith("rehearsal")
