"""`bench.py --gpus N` as the driver runs it (no outer torch.distributed.run): the script starts
N rank processes itself and rank 0's JSON line reports the whole job (SURVEY.md §8(e);
reference exchange: a2c.py:324-336).  Rehearsed with 2 ranks sharing cuda:0 and gloo
collectives (FJSP_BENCH_BACKEND=gloo); the 8-GPU driver run uses one GPU per rank and RCCL."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = dict(os.environ, FJSP_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", *args], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]        # one JSON line: rank 0's
    return json.loads(lines[0])


def test_bench_gpus2_step_workload():
    d = _bench("--steps", "2", "--warmup", "1", "--batch-steps", "128", "--chunk", "128", "--no-cpu-baseline",
               "--no-step-mode", "--no-chunk-compare")
    assert d["n_gpus"] == 2
    assert d["config"]["global_envs"] == 8192
    assert d["config"]["env_steps_per_bench_step"] == 2 * 4096 * 128
    assert d["value"] > 0 and d["scaling"] == "weak"


def test_bench_gpus2_a2c_gather():
    d = _bench("--workload", "a2c", "--exchange", "gather", "--steps", "1", "--warmup", "1")
    assert d["n_gpus"] == 2
    assert d["config"]["global_envs"] == 8192
    assert d["config"]["exchange"] == "gather"
    a = d["a2c"]
    assert a["exchange_bytes_per_rank_per_batch"] == 256 * 4096 * 258 + 4096 * 4
    assert a["n_gpus"] == 2 and a["value"] > 0


def test_bench_gpus2_a2c_shard():
    d = _bench("--workload", "a2c", "--steps", "1", "--warmup", "1")     # the a2c default exchange
    assert d["n_gpus"] == 2 and d["config"]["exchange"] == "shard"
    a = d["a2c"]
    rec = a["shard_records"]
    assert not rec["fallback"] and rec["samples"] == 256 * 4096
    # the records sent to the other rank, plus the 2.7 MB gradient all_reduce: far below the slab
    assert 0 < a["exchange_bytes_per_rank_per_batch"] < 256 * 4096 * 258
    assert a["n_gpus"] == 2 and a["value"] > 0
    # the stats batch's stages, max over ranks, and every rank's record traffic
    stages = ("gae", "adv_stats", "combine", "exchange", "own", "all_reduce", "clip_adam")
    assert set(a["update_stage_ms"]) == {"learn"} | {"shard_" + k for k in stages}
    assert len(a["shard_bytes_sent_by_rank"]) == 2 and all(b > 0 for b in a["shard_bytes_sent_by_rank"])
    assert all(len(v) == 2 for v in a["shard_records_received_by_rank"].values())
