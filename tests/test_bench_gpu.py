"""bench.py on a GPU box: ``--gpus N`` really runs N ranks (rehearsed as gloo ranks sharing cuda:0,
through the graphed step sequence with host-staged collectives), or fails fast when the node has
fewer GPUs.  Reference: ``experiments/huge_batch_size.py:358-363`` (one process per GPU)."""

import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_two_ranks_shared_gpu_gloo():
    """Two rank processes (self-launched), one JSON line with n_gpus 2, the alternative strategy timed
    too, and the cross-rank checks clean: the same global batches everywhere (es) and bit-identical
    replicas (dp, 2 model chunks of 4 models on 2048 rows -- the shape whose engines pick a split-K
    gradient on their own)."""
    r = _bench("--gpus", "2", "--shared-gpu", "--dist-backend", "gloo", "--steps", "20", "--warmup", "5",
               "--no-eval", "--settle-ms", "0", "--ring-rows", "131072", "--parallelism", "es")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "es2" and rec["config"]["global_batch"] == 4096
    col = rec["collectives"]
    assert col["process_group"] == {"backend": "gloo", "ranks": 2}
    assert "gloo" in col["path"] and col["fallback"] is None
    assert [d["rank"] for d in col["rank_devices"]] == [0, 1]
    assert col["consistency"]["max_abs_spread"] == 0.0
    alt = rec["alt_parallelism"]
    assert alt["parallelism"] == "dp2" and "error" not in alt, alt
    assert alt["value"] > 0 and "gloo" in alt["collective_path"]
    assert alt["consistency"]["max_abs_delta"] == 0.0
    cal = rec["comm_calibration"]  # the node's own collective rates, timed before the mode was chosen
    assert cal["backend"] == "gloo" and cal["all_gather"]["bytes_per_rank"] == 2048 * 512 * 2
    assert cal["all_reduce"]["bus_GBps"] > 0


def test_bench_more_gpus_than_present_fails_fast():
    have = torch.cuda.device_count()
    r = _bench("--gpus", str(have + 1), "--steps", "2", "--warmup", "1", timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "GPU(s)" in r.stderr and not r.stdout.strip()
