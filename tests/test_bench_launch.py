"""bench.py's rank launch (reference: eval_inference_model.sh:29-36 starts
`num_gpus` extraction processes): `--gpus N` without a launcher starts N rank
processes; under a launcher it must agree with WORLD_SIZE.  CPU only -- the
hidden --stub-extractor runs the same launch and gather logic over gloo with a
numpy stand-in for the forward."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env_kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_kw)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          cwd=ROOT, capture_output=True, text=True, timeout=180)


def _line(r):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout      # rank 0 alone prints
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_n_spawns_n_ranks(n):
    line = _line(_run(["--gpus", str(n), "--steps", "3", "--stub-extractor"]))
    assert line["n_gpus"] == n and line["ranks_ran"] == n


def test_gpus_1_runs_in_process():
    line = _line(_run(["--gpus", "1", "--steps", "2", "--stub-extractor"]))
    assert line["n_gpus"] == 1 and line["ranks_ran"] == 1


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "4", "--steps", "1", "--stub-extractor"], WORLD_SIZE="2", RANK="0",
             LOCAL_RANK="0")
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_launch_failure_propagates():
    r = _run(["--gpus", "2", "--steps", "1", "--stub-extractor", "--frames", "-5"])
    assert r.returncode != 0


def test_one_failing_rank_stops_the_others():
    """A rank that dies (here: rank 1 of 2 before the rendezvous completes) must
    not leave rank 0 blocked in the collective: the launcher stops it and exits
    non-zero, well inside the test's time limit."""
    import time
    t0 = time.perf_counter()
    r = _run(["--gpus", "2", "--steps", "1", "--stub-extractor"], VOXEMB_STUB_FAIL_RANK="1")
    assert r.returncode != 0
    assert time.perf_counter() - t0 < 120
