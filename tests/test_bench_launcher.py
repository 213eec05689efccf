"""bench.py's own multi-rank launch (`python bench.py --gpus N` outside torchrun)
on CPU: the parent starts N gloo ranks (bench.launch_ranks), they shard the
stream, gather it, take the max time over ranks, and rank 0 prints ONE JSON
line with n_gpus == N, a verified stream order and the CPU baseline.  The
--dry-run flag replaces the voting by the fields' generating keypoints (the
product path needs a GPU), everything around it is the real run's code."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", "--steps", "3", "--warmup", "1",
           "--per-step", "10", "--fields", "4", "--cpu-seconds", "1"] + list(extra)
    return subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_gpus_n_gloo(n):
    p = _run("--gpus", str(n))
    assert p.returncode == 0, p.stderr[-3000:]
    # one JSON line, from rank 0 only (gloo itself prints a connection note)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == n and line["dry_run"] is True
    assert line["stream_order_ok"] and line["stream_order_max_err_px"] == 0.0
    assert line["config"]["stream_images"] == n * 3 * 10
    assert line["cpu_baseline"]["value"] > 0          # rank 0 reports it at every N


def test_launcher_gpus_1_single_process():
    p = _run("--gpus", "1", "--skip-cpu")
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert line["n_gpus"] == 1 and line["stream_order_ok"]


def test_world_size_mismatch_fails():
    p = _run("--gpus", "2", "--skip-cpu", env_extra={"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE 1 != --gpus 2" in p.stderr


def test_failing_rank_stops_launch():
    # ranks that raise (an empty stream: nothing to stack) make the launcher
    # stop the others and return non-zero instead of waiting
    p = _run("--gpus", "2", "--skip-cpu", "--steps", "0")
    assert p.returncode != 0


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_launcher_two_ranks_on_the_device():
    """The real GPU path at N = 2 on a one-GPU box: bench.py starts two ranks
    that share cuda:0 over gloo (--share-device; RCCL refuses two ranks on one
    device) and run the headline stream, configs[3] and configs[4] legs,
    graph capture and replay included, through the sharded gather; one JSON
    line with n_gpus 2 and every gathered image in its stream slot."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--share-device", "--steps", "2",
           "--warmup", "1", "--per-step", "16", "--fields", "4", "--skip-e2e", "--skip-u1", "--skip-u4",
           "--skip-cpu"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=580)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["stream_order_ok"]
    assert line["config"]["stream_images"] == 2 * 2 * 16
    assert line["stream_config3"]["n_gpus"] == 2 and line["stream_config3"]["zeros_path_ok"]
    assert line["stream_config4"]["n_gpus"] == 2 and line["stream_config4"]["covariances_finite"]


def _cpuset(s):
    out = set()
    for part in s.split(","):
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_ranks_pinned_disjoint(n):
    """bench.pin_rank: every rank of `bench.py --gpus N` runs on its own CPUs
    (set before its first GPU call), disjoint from the other ranks', reported
    in the line as rank_cpus."""
    p = _run("--gpus", str(n), "--skip-cpu")
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    sets = [_cpuset(s) for s in line["rank_cpus"]]
    assert len(sets) == n and all(sets)
    for i in range(n):
        for j in range(i + 1, n):
            assert not (sets[i] & sets[j]), line["rank_cpus"]
    assert set().union(*sets) <= os.sched_getaffinity(0)
    assert line["rank_cpus_source"] == "even-split"      # no KFD topology in this container


def test_rank_cpu_sets_gpu_local():
    """rank_cpu_sets on a modelled 8-GPU node: GPUs 0-3 local to CPUs 0-63,
    GPUs 4-7 to 64-127, the process allowed every other CPU: each rank gets
    its own slice of its GPU's local CPUs."""
    import bench
    local = [set(range(0, 64))] * 4 + [set(range(64, 128))] * 4
    allowed = set(range(0, 128, 2))
    sets, src = bench.rank_cpu_sets(8, allowed, local)
    assert src == "gpu-local"
    for r in range(8):
        assert sets[r] and sets[r] <= local[r] & allowed and len(sets[r]) == 8
        for q in range(r):
            assert not (sets[r] & sets[q])
    # overlapping but unequal local sets: an even split of the allowed CPUs
    sets, src = bench.rank_cpu_sets(2, set(range(8)), [set(range(0, 6)), set(range(2, 8))])
    assert src == "even-split" and sets == [set(range(4)), set(range(4, 8))]
    # --share-device: every rank on GPU 0's local CPUs
    sets, src = bench.rank_cpu_sets(2, set(range(16)), [set(range(8))], share_device=True)
    assert src == "gpu-local" and sets == [set(range(4)), set(range(4, 8))]
    # fewer CPUs than ranks: no pinning
    assert bench.rank_cpu_sets(4, {0, 1}, None)[0] is None
