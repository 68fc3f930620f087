"""bench.py's rank launcher (`--gpus N` without WORLD_SIZE) and its refusals, on the CPU.

The driver runs `python bench.py --gpus N ...` (and `torchrun ... bench.py --gpus N`): the first form
must start N rank processes itself, the second must agree with --gpus. The ranks here run the hidden
`--launcher-selftest` mode, which reports the rendezvous environment and exits before any torch
import, so no GPU is involved."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=120)


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_under_test", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("n", [2, 3, 8])
def test_launcher_starts_n_ranks_with_their_environment(n):
    r = _run(["--gpus", str(n), "--launcher-selftest", "ok"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout                      # the contract: rank 0's ONE JSON line
    envs = {0: json.loads(lines[0])}
    for ln in r.stderr.splitlines():
        if ln.startswith("[rank ") and ln[ln.index("]") + 2:].startswith("{"):
            rk = int(ln[len("[rank "):ln.index("]")])
            envs[rk] = json.loads(ln[ln.index("]") + 2:])
    assert sorted(envs) == list(range(n))
    ports = {e["MASTER_PORT"] for e in envs.values()}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for rk, e in envs.items():
        assert e["RANK"] == e["LOCAL_RANK"] == str(rk)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == str(n)
        assert e["MASTER_ADDR"] == "127.0.0.1"


def test_launcher_fails_when_a_rank_fails():
    r = _run(["--gpus", "3", "--launcher-selftest", "fail1"])
    assert r.returncode != 0
    assert "rank 1 exited 3 after stage 'start'" in r.stderr
    assert r.stdout.strip() == ""                          # no JSON line from a failed world


def test_launcher_names_a_hung_rank_and_its_last_stage():
    """a rank that hangs (here rank 1 after "process group up", while rank 0 waits
    in the closing barrier) is killed at --launch-timeout — by default below the driver's 600-s limit —
    and named with the last stage marker it printed; the launcher exits non-zero with no JSON line,
    and every rank's markers were forwarded to stderr as they arrived."""
    import time
    t0 = time.monotonic()
    r = _run(["--gpus", "2", "--launcher-selftest", "hang1", "--launch-timeout", "4"])
    assert time.monotonic() - t0 < 60
    assert r.returncode != 0 and r.stdout.strip() == ""
    assert "timeout after 4 s: rank 1 hung after stage 'process group up'" in r.stderr, r.stderr
    assert "rank 0: last stage 'warm-up done'" in r.stderr and "[still running]" in r.stderr, r.stderr
    assert "[rank 1] bench-stage rank=1 stage=process group up" in r.stderr, r.stderr
    b = _bench_module()
    assert b.parse_stage("bench-stage rank=3 stage=timed region done t=12.5s") == (3, "timed region done")
    assert b.parse_stage("something else") is None


def test_launch_timeout_default_is_below_the_drivers_limit():
    import argparse
    import sys as _sys
    b = _bench_module()
    argv, _sys.argv = _sys.argv, ["bench.py"]
    try:
        args = b.parse()
    finally:
        _sys.argv = argv
    assert isinstance(args, argparse.Namespace) and 0 < args.launch_timeout < 600


@pytest.mark.parametrize("ws,gpus", [("2", 4), ("1", 8), ("8", 1)])
def test_world_size_mismatch_is_refused(ws, gpus):
    r = _run(["--gpus", str(gpus)], env_extra={"WORLD_SIZE": ws, "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "refusing" in r.stderr


def test_world_check_and_rank_environments_units():
    b = _bench_module()
    assert b.world_check(1, {}) == "rank"
    assert b.world_check(4, {}) == "launch"
    assert b.world_check(4, {"WORLD_SIZE": "4"}) == "rank"
    with pytest.raises(SystemExit):
        b.world_check(4, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        b.world_check(0, {})
    envs = b.rank_environments(4, 12345, base={"PATH": "/bin", "OMP_NUM_THREADS": "16"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["PATH"] == "/bin" and e["OMP_NUM_THREADS"] == "16" and e["MASTER_PORT"] == "12345" for e in envs)


def test_single_rank_without_gpu_fails_loudly():
    """A rank that finds no device (this container) exits non-zero instead of folding or falling back."""
    r = _run(["--gpus", "1", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--pmc", "off"])
    assert r.returncode != 0
    assert "refusing to fold" in r.stderr or "GPU" in r.stderr
