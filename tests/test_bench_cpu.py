"""bench.py's launcher contract on the CPU: ``--gpus N`` runs N ranks or fails fast, never silently one."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_check_world_rejects_mismatches(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("RANK", raising=False)
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 1)
    assert bench.check_world(bench.parse(["--gpus", "1"])) is None
    assert "has 1 GPU" in bench.check_world(bench.parse(["--gpus", "2"]))
    assert bench.check_world(bench.parse(["--gpus", "2", "--shared-gpu"])) is None
    assert "--gpus must be" in bench.check_world(bench.parse(["--gpus", "0"]))
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 8)
    assert "WORLD_SIZE=4" in bench.check_world(bench.parse(["--gpus", "2"]))
    assert bench.check_world(bench.parse(["--gpus", "4"])) is None


def test_main_fails_fast_without_enough_gpus(monkeypatch):
    """More GPUs asked for than the node has: non-zero before any GPU work or launch."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("RANK", raising=False)
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 1)
    launched = []
    monkeypatch.setattr(bench, "launch_ranks", lambda *a, **k: launched.append(a) or 0)
    assert bench.main(["--gpus", "2"]) == 3
    assert not launched
    # enough devices: the parent hands over to the launcher instead of running one GPU
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 8)
    assert bench.main(["--gpus", "8", "--steps", "3"]) == 0
    assert launched and launched[0][0] == 8 and "--steps" in launched[0][1]


PROBE = r'''
import json, os, sys
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
print("noise on stdout from rank", rank, flush=True)
if rank == 0:
    print(json.dumps({"metric": "probe", "n_gpus": world, "argv": sys.argv[1:]}), flush=True)
sys.exit(int(os.environ.get("PROBE_RC", "0")) if rank == world - 1 else 0)
'''


@pytest.mark.parametrize("rc", [0, 5])
def test_launch_ranks_forwards_rank0_json_and_worst_rc(tmp_path, rc, capfd, monkeypatch):
    """The launcher starts N torch.distributed.run ranks, forwards exactly rank 0's JSON line to stdout
    (other stdout goes to stderr) and returns non-zero when any rank fails."""
    script = tmp_path / "probe.py"
    script.write_text(PROBE)
    monkeypatch.setenv("PROBE_RC", str(rc))
    got = bench.launch_ranks(3, ["--gpus", "3", "--steps", "2"], script=str(script))
    out, err = capfd.readouterr()
    if rc == 0:
        assert got == 0
        lines = [ln for ln in out.splitlines() if ln.strip()]
        assert len(lines) == 1, out
        rec = json.loads(lines[0])
        assert rec["n_gpus"] == 3 and rec["argv"] == ["--gpus", "3", "--steps", "2"]
        assert "noise on stdout" in err
    else:
        assert got != 0


def _consistency_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import bench as b
    from sparse_coding__amd.parallel.dist import DistInfo

    dist.init_process_group("gloo", rank=rank, world_size=world)
    info = DistInfo(rank, world, rank, torch.device("cpu"), "gloo")
    same = [torch.arange(6, dtype=torch.float32)]
    diff = [torch.arange(6, dtype=torch.float32) + (0.5 if rank == 1 else 0.0)]
    out = {"same": b._replica_delta(same, info)["max_abs_delta"], "diff": b._replica_delta(diff, info)["max_abs_delta"],
           "bsame": b._batch_spread([torch.ones(2, 3)], info)["max_abs_spread"],
           "bdiff": b._batch_spread([torch.ones(2, 3) * (rank + 1)], info)["max_abs_spread"]}
    q.put((rank, out))
    dist.destroy_process_group()


def test_cross_rank_consistency_checks_gloo():
    """The bench's post-run checks: max |master - rank 0's| (dp / zero1) and the spread of global-batch
    checksums (es) are 0 for identical ranks and non-zero otherwise, on every rank."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_consistency_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        assert res[r]["same"] == 0.0 and res[r]["diff"] == 0.5
        assert res[r]["bsame"] == 0.0 and res[r]["bdiff"] > 0


HANG_PROBE = r'''
import json, os, sys
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
if "--dist-graph" not in sys.argv:
    # the in-graph run: rank 1's watchdog fires in the timed region (marker + exit 5, no JSON)
    if rank == 1:
        with open(os.path.join(os.environ["SC_BENCH_HANG_DIR"], "rank1.json"), "w") as f:
            json.dump({"rank": 1, "phase": "timed", "emitted": False}, f)
        sys.exit(5)
    sys.exit(0)
if rank == 0:
    print(json.dumps({"metric": "probe", "argv": sys.argv[1:]}), flush=True)
'''


def test_launch_ranks_relaunches_on_host_collectives_after_a_watchdog_hang(tmp_path, capfd):
    """A rank whose watchdog ended a hung in-graph phase (marker + HANG_RC, no result line) makes the
    launcher start FRESH ranks with --dist-graph 0 and the reason on record; their line is forwarded."""
    script = tmp_path / "hang.py"
    script.write_text(HANG_PROBE)
    got = bench.launch_ranks(2, ["--gpus", "2", "--steps", "2"], script=str(script))
    out, err = capfd.readouterr()
    assert got == 0, err
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out
    argv = json.loads(lines[0])["argv"]
    assert argv[:4] == ["--gpus", "2", "--steps", "2"]
    assert argv[argv.index("--dist-graph") + 1] == "0"
    assert "in-graph hang: timed (rank 1)" in argv[argv.index("--fallback-reason") + 1]
    # already on host collectives: a second hang is not retried
    assert bench._dist_graph_off(["--dist-graph", "0"]) and bench._dist_graph_off(["--dp-graph=0"])
    assert not bench._dist_graph_off(["--dist-graph", "1"]) and not bench._dist_graph_off([])


WD_PROBE = r'''
import json, os, sys, time
sys.path.insert(0, sys.argv[1])
import bench
class Info: rank, is_main = 0, True
wd = bench.Watchdog(Info(), True)
wd.arm("capture", 30.0)
wd.arm("first-replay", 0.2)    # re-armed: the capture limit no longer applies
wd.disarm()
time.sleep(0.5)                 # disarmed: nothing fires
wd.pending = {"metric": "probe", "value": 1.0}
wd.arm("alt-timed", 0.2)
time.sleep(30)
print("not reached")
'''


def test_watchdog_exits_with_marker_and_pending_record(tmp_path):
    """The watchdog ends a process whose armed phase overruns: exit HANG_RC, a marker naming the phase,
    and the pending (already measured) record on stdout; a disarmed or re-armed phase never fires."""
    script = tmp_path / "wd.py"
    script.write_text(WD_PROBE)
    env = dict(os.environ, SC_BENCH_HANG_DIR=str(tmp_path))
    p = subprocess.run([sys.executable, str(script), ROOT], capture_output=True, text=True, env=env, timeout=60)
    assert p.returncode == bench.HANG_RC, p.stderr
    assert "hung in phase 'alt-timed'" in p.stderr and "not reached" not in p.stdout
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["metric"] == "probe" and rec["watchdog"]["phase"] == "alt-timed"
    marker = json.loads((tmp_path / "rank0.json").read_text())
    assert marker == {"rank": 0, "phase": "alt-timed", "emitted": True}
