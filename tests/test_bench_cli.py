"""bench.py's multi-GPU launch logic on the CPU (no GPU needed):

* one distinct GPU per rank, or a refusal; sharing only as a labelled rehearsal;
* `--gpus N` without a launcher spawns N rank processes (never an exec of a
  process that touched the GPU) and fails as a whole when a rank fails;
* `--gpus` must agree with a launcher's WORLD_SIZE.
"""
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_plan_device_one_gpu_per_rank():
    assert bench.plan_device(0, 8, 8, False) == (0, False)
    assert bench.plan_device(7, 8, 8, False) == (7, False)
    assert bench.plan_device(1, 2, 8, False) == (1, False)


def test_plan_device_refuses_shared_gpus_unless_rehearsal():
    with pytest.raises(SystemExit) as e:
        bench.plan_device(1, 2, 1, False)
    assert "GPU(s) visible" in str(e.value)
    assert bench.plan_device(1, 2, 1, True) == (0, True)
    assert bench.plan_device(5, 8, 4, True) == (1, True)
    with pytest.raises(SystemExit):
        bench.plan_device(0, 1, 0, True)  # no GPU at all


def test_gpus_must_match_launcher_world(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "4")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "2"])
    assert "WORLD_SIZE=4" in str(e.value)


def test_spawned_ranks_fail_together_without_gpu():
    """On a machine without a GPU every spawned rank refuses to run; the
    launcher returns a failure instead of hanging or reporting a number."""
    if os.environ.get("HIP_VISIBLE_DEVICES") is None:
        try:
            import torch

            if torch.cuda.device_count() > 0:
                pytest.skip("a GPU is visible here")
        except ImportError:
            pass
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu", "--traffic", "off",
                        "--quiet"], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0
    assert "needs a GPU" in p.stderr
    assert p.stdout.strip() == ""  # no JSON line from a failed run
    assert time.time() - t0 < 300


def test_summarize_reports_median_and_spread():
    w = bench.Workload("x", 1000, 32, [lambda: None], "k", "d")
    w.enqueue_s = 0.0
    r = bench.summarize(w, [2.0, 1.0, 4.0], [0.02, 0.01, 0.04], 10, 1000 * 10)
    assert r["value"] == 5000.0 and r["value_min"] == 2500.0 and r["value_max"] == 10000.0
    assert r["kernel_us"] == pytest.approx(20000.0)
    assert r["repeats"] == 3


def test_pmc_fields_and_limiter():
    f = bench.pmc_fields({"FETCH_SIZE": 100.0, "WRITE_SIZE": 50.0, "SQ_ACTIVE_INST_VALU": 1024.0,
                          "GRBM_GUI_ACTIVE": 8.0}, 250 * 1024.0)
    assert f["traffic"] == 250 * 1024.0 and f["traffic_over_algorithmic"] == 1.0
    assert f["valu_busy"] == 4.0
    assert bench.limiter(6000.0, 0.5) == "hbm"
    assert bench.limiter(3000.0, 0.9) == "valu"
