"""bench.py's own multi-GPU launch (`--gpus N` without torch.distributed.run): the launch plan, the
WORLD_SIZE mismatch exit and the child processes, on CPU (no GPU call is made by any of these)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(kw)
    return e


def test_launch_plan_one_gpu_runs_in_process():
    assert bench.launch_plan(1, _env()) is None


def test_launch_plan_spawns_one_rank_per_gpu():
    plan = bench.launch_plan(4, _env(), port=29517)
    assert [p["RANK"] for p in plan] == ["0", "1", "2", "3"]
    assert [p["LOCAL_RANK"] for p in plan] == ["0", "1", "2", "3"]
    assert all(p["WORLD_SIZE"] == "4" and p["MASTER_ADDR"] == "127.0.0.1" and p["MASTER_PORT"] == "29517"
               for p in plan)


def test_launch_plan_defers_to_a_matching_launcher():
    assert bench.launch_plan(8, _env(WORLD_SIZE="8", RANK="3", LOCAL_RANK="3")) is None


@pytest.mark.parametrize("gpus,ws", [(8, "1"), (2, "4"), (1, "2")])
def test_launch_plan_rejects_a_mismatched_world(gpus, ws):
    with pytest.raises(bench.LaunchError):
        bench.launch_plan(gpus, _env(WORLD_SIZE=ws))


def test_mismatch_exits_nonzero_before_any_gpu_work():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=_env(WORLD_SIZE="3"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2
    assert "disagrees" in r.stderr


def test_spawned_ranks_run_and_exit_cleanly():
    # every child gets WORLD_SIZE=2, so it runs main() itself: --help exits 0 before touching torch
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--help"],
                       env=_env(TCI_BENCH_DEVICES="2"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("usage:") == 2


def test_a_failing_rank_fails_the_launch():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-such-flag"],
                       env=_env(TCI_BENCH_DEVICES="2"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0


@pytest.mark.parametrize("gpus,visible,rehearsal,ok", [(8, 8, False, True), (8, 7, False, False), (2, 1, False, False),
                                                       (2, 1, True, True), (1, 0, False, False)])
def test_device_count_check(gpus, visible, rehearsal, ok):
    if ok:
        bench.check_devices(gpus, visible, rehearsal)
    else:
        with pytest.raises(bench.LaunchError):
            bench.check_devices(gpus, visible, rehearsal)


def test_too_few_devices_refused_before_any_rank_starts():
    # the parent counts devices (torch.cuda.device_count(): no HIP context) and exits 2; no child runs
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=_env(TCI_BENCH_DEVICES="4"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2
    assert "needs 8 visible GPU(s), found 4" in r.stderr
    assert "usage:" not in r.stdout


def test_no_gpu_refused_for_one_rank():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")], env=_env(TCI_BENCH_DEVICES="0"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2
    assert "needs 1 visible GPU(s), found 0" in r.stderr


@pytest.mark.parametrize("rank,world", [(0, 1), (0, 2), (0, 8), (1, 2), (3, 8)])
def test_cpu_baseline_is_in_the_line_at_every_world_size(monkeypatch, rank, world):
    """the CPU baseline legs run on rank 0 at any world size (not only N = 1), so
    every line of a 1/2/4/8-GPU scaling run carries `cpu_baseline` next to the GPU numbers; other
    ranks skip them. The legs themselves are stubbed here (the real ones are exercised on the GPU box)."""
    from types import SimpleNamespace

    monkeypatch.setattr(bench, "cpu_baseline", lambda *a, **k: {"value": 1.0, "unit": "SS evals/s"})
    monkeypatch.setattr(bench, "cpu_fit_config1", lambda *a, **k: {"value": 2.0})
    monkeypatch.setattr(bench, "cpu_baseline_synth", lambda cfg, *a, **k: {"value": float(cfg)})

    class C:
        n_cells = 3

    res = {}
    bench.cpu_legs(res, rank, world, SimpleNamespace(no_cpu_baseline=False, proposals=4, cpu_seconds=1.0), C(),
                   None, None, None, {4: {}, 5: {}})
    if rank == 0:
        assert set(res) == {"cpu_baseline", "cpu_fit_config1", "cpu_baseline_config4", "cpu_baseline_config5"}
        assert res["cpu_baseline"]["host"]["ranks_on_this_host"] == world
    else:
        assert res == {}
    res = {}
    bench.cpu_legs(res, rank, world, SimpleNamespace(no_cpu_baseline=True, proposals=4, cpu_seconds=1.0), C(),
                   None, None, None, {})
    assert res == {}
