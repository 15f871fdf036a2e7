"""bench.py's own multi-rank launcher (CPU: --dry-run stops every rank before GPU initialisation).

``python bench.py --gpus N`` without torch.distributed.run in front must start N ranks itself (one process per
GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), relay rank 0's JSON line and fail
when a rank fails; under a launcher, --gpus must equal WORLD_SIZE."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=120):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=e, timeout=timeout)


def test_launcher_spawns_n_ranks():
    r = _run(["--gpus", "3", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # only rank 0's line reaches stdout
    d = json.loads(lines[0])
    assert d["dry_run"] and d["n_gpus"] == 3 and d["rank"] == 0
    for rank in range(3):
        assert f"[rank {rank}/3] dry run: local rank {rank}, master 127.0.0.1:" in r.stderr
    assert "[launcher] started 3 ranks" in r.stderr


def test_launcher_fails_when_a_rank_fails():
    r = _run(["--gpus", "2", "--dry-run"], env={"SMG_BENCH_FAIL_RANK": "1"})
    assert r.returncode != 0
    assert "rank 1 exited with" in r.stderr


def test_gpus_must_match_world_size_under_a_launcher():
    r = _run(["--gpus", "1", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "one rank per GPU" in r.stderr
    r = _run(["--gpus", "2", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1",
                                                "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "1"})
    assert r.returncode == 0 and r.stdout.strip() == ""  # rank 1 prints nothing on stdout
