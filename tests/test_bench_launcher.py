"""bench.py's own N-rank launcher (no torchrun), CPU rehearsal with gloo:
``python bench.py --gpus 2`` really runs two ranks, both scaling modes shard
the global batch, and every item sees the same inputs and parameters as in a
single-process run (the per-item digests are equal).  The GPU form of this
check (outputs, not inputs) is tests/test_gpu_parity.py::test_bench_two_ranks_*."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
COMMON = ["--dry-run", "--dist-backend", "gloo", "--size", "160", "--backgrounds", "3", "--no-cpu-baseline"]


def _run(args, tmp_path, name, env_extra=None):
    out = tmp_path / f"{name}.json"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, str(ROOT / "bench.py")] + COMMON + args + ["--dump-digests", str(out)],
                       capture_output=True, text=True, timeout=240, env=env, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0]), json.loads(out.read_text())


@pytest.mark.parametrize("workload", ["pipe5", "rotflip"])
def test_two_rank_launcher_matches_single_process(tmp_path, workload):
    one, d1 = _run(["--gpus", "1", "--batch", "6", "--workload", workload], tmp_path, "one")
    assert one["n_gpus"] == 1 and one["items"] == 6
    strong, d2 = _run(["--gpus", "2", "--batch", "6", "--scaling", "strong", "--workload", workload],
                      tmp_path, "strong")
    assert strong["n_gpus"] == 2 and strong["global_batch"] == 6 and strong["scaling"] == "strong"
    assert d2 == d1
    weak, d3 = _run(["--gpus", "2", "--batch", "3", "--workload", workload], tmp_path, "weak")
    assert weak["n_gpus"] == 2 and weak["global_batch"] == 6 and weak["scaling"] == "weak"
    assert d3 == d1


def test_rank_count_mismatch_fails_loudly(tmp_path):
    env = {k: v for k, v in os.environ.items()}
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"] + COMMON,
                       capture_output=True, text=True, timeout=120, env=env, cwd=str(ROOT))
    assert p.returncode != 0 and "--gpus 2 but 1 rank" in p.stderr
