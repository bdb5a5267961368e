"""bench.py's multi-rank launch path on the CPU (no GPU call): `bench.py --gpus N` without an
external launcher spawns N ranks itself with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT (the fan-out StorageClient.inl:74-159 does per request, here once per job), and the
ranks rendezvous over gloo.  --launch-check stops after the rendezvous."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--launch-check"], env=env,
                       capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0's line only
    d = json.loads(lines[0])
    assert d["launch_check"] == "ok" and d["world"] == n and d["rank_sum"] == n * (n - 1) // 2
