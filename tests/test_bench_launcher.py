"""bench.py as the N-rank launcher (CPU, no GPU touched): `python bench.py --gpus N`
outside torch.distributed.run starts N rank processes with distinct RANK /
LOCAL_RANK, WORLD_SIZE = N and a 127.0.0.1 rendezvous, and refuses a --gpus that
disagrees with an inherited WORLD_SIZE."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_starts_n_ranks(n):
    p = run(["--gpus", str(n), "--dry-run", "--workload", "C3"])
    assert p.returncode == 0, p.stderr
    lines = [json.loads(s) for s in p.stdout.splitlines() if s.strip()]
    assert sorted(d["rank"] for d in lines) == list(range(n))
    assert sorted(d["local_rank"] for d in lines) == list(range(n))
    assert all(d["world"] == n and d["ranks_in_group"] == n for d in lines)  # one gloo group of N
    assert all(d["workload"] == "C3" and d["master"].startswith("127.0.0.1:") for d in lines)
    assert len({d["master"] for d in lines}) == 1


def test_single_rank_needs_no_launcher():
    p = run(["--dry-run"])
    assert p.returncode == 0, p.stderr
    (d,) = [json.loads(s) for s in p.stdout.splitlines() if s.strip()]
    assert d["world"] == 1 and d["rank"] == 0


def test_gpus_must_match_inherited_world():
    p = run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr


def test_failing_rank_fails_the_launch():
    # an unknown workload makes every rank exit non-zero at argument parsing
    p = run(["--gpus", "2", "--dry-run", "--tune", "NO_SUCH_KNOB=1"])
    assert p.returncode != 0
