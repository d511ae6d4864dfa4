"""bench.py under torch.distributed.run on the CPU (gloo): the driver's multi-rank contract (one JSON line from rank 0,
whole-job aggregate) for DP replicas and for TP replicas (--tp 2: the 70B TP=8 serving shape, here at TP=2 on the
tiny model), without GPUs."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "bench.py"), "--gpus", "2",
           "--device", "cpu", "--model", "tiny", "--streams", "3", "--steps", "1", "--warmup", "1",
           "--num-predict", "24", "--single-stream", "2", "--no-graphs", "--max-model-len", "384"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.slow
@pytest.mark.parametrize("tp,sp", [(1, False), (2, False), (2, True)])
def test_bench_two_ranks(tp, sp):
    r = _run((["--tp", str(tp)] if tp > 1 else []) + (["--sequence-parallel"] if sp else []))
    assert r["n_gpus"] == 2 and r["steps"] == 1 and r["value"] > 0
    if tp == 1:
        assert r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 6
        assert r["verdicts_valid"] == "6/6"
    else:
        assert r["config"]["parallelism"] == "tp2" and r["config"]["global_batch"] == 3
        assert r["verdicts_valid"] == "3/3" and "TP=2" in r["metric"]


def _run_plain(gpus_args, env_extra=None, timeout=600):
    model = "tiny70" if "--tp" in gpus_args else "tiny"
    cmd = [sys.executable, os.path.join(REPO, "bench.py")] + gpus_args + [
        "--device", "cpu", "--model", model, "--streams", "3", "--steps", "1", "--warmup", "1",
        "--num-predict", "24", "--single-stream", "2", "--no-graphs", "--max-model-len", "384"]
    env = dict(os.environ, OMP_NUM_THREADS="2", **(env_extra or {}))
    env.pop("WORLD_SIZE", None) if not env_extra or "WORLD_SIZE" not in env_extra else None
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=REPO)


@pytest.mark.slow
def test_bench_gpus_flag_self_launches():
    """`python bench.py --gpus 2` with no launcher runs 2 ranks (--gpus was ignored) and reports both
    replicas' chains."""
    out = _run_plain(["--gpus", "2"])
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2" and r["verdicts_valid"] == "6/6"


def test_bench_gpus_mismatch_is_an_error():
    out = _run_plain(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, timeout=300)
    assert out.returncode != 0 and "disagrees with WORLD_SIZE" in out.stderr


@pytest.mark.slow
def test_bench_tp8_70b_geometry_self_launch():
    """The 70B TP=8 serving shape at its real degree: `bench.py --gpus 8 --tp 8` on the tiny70 preset (64 q / 8 KV
    heads: one KV head per rank; 16032-row vocab shards), 8 gloo ranks in one lockstep TP group."""
    out = _run_plain(["--gpus", "8", "--tp", "8"], timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 8 and r["config"]["parallelism"] == "tp8" and r["config"]["model"] == "tiny70"
    assert r["verdicts_valid"] == "3/3" and "TP=8" in r["metric"]
