"""CPU: `bench.py --gpus N` outside torch.distributed.run starts its own N rank processes (children, never exec)
and the ranks run the gloo control plane (unique-id hand-off, all-gather of verdict words, MIN reduction); the
CPU dry run replaces the GPU verify with the oracle. VERDICT r1 item 1: the driver may run
`python bench.py --gpus 8` directly."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("gpus", [2, 3])
def test_bench_self_launch_dry_run(gpus):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dry-run",
                          "--records-per-gpu", "1000", "--msg-len", "77"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, out.stdout  # exactly one JSON line, from rank 0
    r = json.loads(lines[0])
    assert r["dry_run"] and r["n_gpus"] == gpus and r["verdict_match"] == 1.0 and r["unique_id_shared"]
    assert 0 < r["valid"] < r["records"]
    # the N > 1 line separates per-rank kernel time, collective time and the slowest rank
    m = r["multi_gpu"]
    for k in ("kernel_ms_per_rank", "verify_only_ms_per_rank", "gather_only_ms_per_rank"):
        assert len(m[k]) == gpus and all(x >= 0 for x in m[k]), k
    assert m["ranks"] == gpus and 0 <= m["max_rank"] < gpus
    assert m["kernel_ms_max"] == max(m["kernel_ms_per_rank"]) == m["kernel_ms_per_rank"][m["max_rank"]]
    assert m["kernel_ms_min"] <= m["kernel_ms_max"] and m["gather_words_per_rank"] > 0


@pytest.mark.parametrize("fail_rank", [1, 0])
def test_bench_self_launch_stops_all_ranks_when_one_dies(fail_rank):
    """a rank that exits early (here before the gloo rendezvous, so its peers would block in it)
    makes the launcher stop the other ranks and exit non-zero within seconds, not at the driver's time limit."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID")}
    env["AT2V_BENCH_FAIL_RANK"] = str(fail_rank)
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--dry-run",
                          "--records-per-gpu", "1000"], capture_output=True, text=True, timeout=120, env=env)
    dt = time.time() - t0
    assert out.returncode != 0
    assert dt < 30, dt
    assert f"rank {fail_rank} exited with status" in out.stderr
    assert "injected failure" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.strip()]  # no result line
