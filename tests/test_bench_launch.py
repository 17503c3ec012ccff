"""bench.py's rank layout (the driver's `python bench.py --gpus N` contract): with no launcher,
`--gpus N` starts N ranks itself as a child torch.distributed.run, and a launcher whose WORLD_SIZE
differs from --gpus is an error.  CPU tests use --launch-check (gloo, no GPU); the GPU test runs the
real bench loop at a small size with two ranks sharing the box's one GPU over gloo."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
_LAUNCH_VARS = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                "TORCHELASTIC_RUN_ID", "GROUP_RANK", "ROLE_RANK")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in _LAUNCH_VARS}
    env.update(extra)
    return env


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH, *args], env=env, capture_output=True, text=True, timeout=timeout,
                          cwd=ROOT)


def test_gpus_two_starts_two_ranks_without_a_launcher():
    r = _run(["--gpus", "2", "--launch-check"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout            # rank 0's line only, relayed once
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_joined"] == 2
    assert "starting 2 ranks" in r.stderr


def test_gpus_one_stays_in_process():
    r = _run(["--launch-check"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    assert line["n_gpus"] == 1 and "starting" not in r.stderr


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "4", "--launch-check"], _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "--gpus 4 but WORLD_SIZE=2" in r.stderr
    assert not _json_lines(r.stdout)


def test_launcher_with_matching_world_size():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
                        "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", BENCH, "--gpus", "3", "--launch-check"],
                       env=_env(), capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    assert line["n_gpus"] == 3 and line["ranks_joined"] == 3


@pytest.mark.gpu
def test_gpu_bench_two_ranks_self_launched():
    """The real bench loop through the self-launch path: 2 ranks on the box's one GPU (gloo exchange,
    a rehearsal of the driver's N-GPU run), small frame, no side lines."""
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--width", "320", "--height", "240",
              "--no-pass-types", "--no-pipeline", "--no-e2e", "--no-cpu-baseline"],
             _env(DPE_BENCH_BACKEND="gloo"), timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = _json_lines(r.stdout)
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["exchange"]["world"] == 2 and line["exchange"]["backend"] == "gloo"
    assert "rehearsal" in line["config"]["parallelism"]
