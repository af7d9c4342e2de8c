"""bench.py's multi-rank path on the GPU box (configs[4]'s split):

* `bench.py --gpus 2` with one visible GPU is refused (every rank needs a GPU
  of its own);
* the same run as a labelled rehearsal (--allow-shared-gpu) spawns 2 rank
  processes that each hash their own contiguous shard of the 1B keys through
  the product library: shards [0, 5e8) and [5e8, 1e9), disjoint and complete,
  outputs checked against the oracle on every rank, `n_gpus` = distinct GPUs,
  and the line carries each rank's device, kernel times and verdicts.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--only", "fixed16,shard1b", "--steps", "5", "--warmup", "2", "--repeats", "2", "--rotate", "2",
        "--keys16", "1000000", "--no-cpu", "--traffic", "off", "--no-host-inclusive", "--warmup-min-s", "0",
        "--quiet"]


def _env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}


def _run(extra, timeout=240):
    return subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2"] + ARGS + extra,
                          capture_output=True, text=True, timeout=timeout, env=_env(), cwd=ROOT)


def test_two_ranks_refused_on_one_gpu():
    if torch.cuda.device_count() >= 2:
        pytest.skip("two GPUs visible: nothing to refuse")
    p = _run([])
    assert p.returncode != 0
    assert "GPU(s) visible" in p.stderr
    assert p.stdout.strip() == ""


def test_two_rank_rehearsal_shards_configs4(tmp_path):
    detail = str(tmp_path / "detail.json")
    p = _run(["--allow-shared-gpu", "--detail-out", detail])
    assert p.returncode == 0, p.stderr[-3000:]
    out = p.stdout.strip().splitlines()
    assert len(out) == 1, out  # stdout is the JSON line alone (gloo's notices and the like go to stderr)
    assert len(out[0]) <= 4096  # what the driver's tail can hold
    line = json.loads(out[0])
    ndev = torch.cuda.device_count()
    assert line["ranks"] == 2
    assert line["n_gpus"] == min(2, ndev)
    assert line.get("rehearsal", False) == (ndev < 2)
    sh = line["secondary"]["shard1b"]
    assert sh["scaling"] == "strong"
    assert sh["shards"] == [[0, 500_000_000], [500_000_000, 1_000_000_000]]
    assert sh["verified"] is True
    assert line["verified"] is True
    # value = all ranks' keys / max-over-ranks time (the line rounds to 6 digits)
    assert line["value"] == pytest.approx(2 * 1_000_000 * 5 / (line["ms_per_step"] * 5 / 1e3), rel=1e-4)
    # the detail file the line names: per-rank evidence (device, own kernel times and verdicts, shards)
    assert line["detail"] == detail
    full = json.load(open(detail))
    assert full["secondary"]["shard1b"]["verified"]["samples_per_rank"] >= 20000
    pr = full["per_rank"]
    assert [p["rank"] for p in pr] == [0, 1]
    assert [p["device"] for p in pr] == [r % max(1, ndev) for r in range(2)]
    assert all(p["kernel_us"]["fixed16"] > 0 and p["kernel_us"]["shard1b"] > 0 for p in pr)
    assert all(p["verified"]["fixed16"] is True and p["verified"]["shard1b"] is True for p in pr)
    assert [p["shard"] for p in pr] == sh["shards"]
    assert set(line["slowest_over_fastest_rank"]) == {"fixed16", "shard1b"}
    assert all(v >= 1.0 for v in line["slowest_over_fastest_rank"].values())
    assert line["barrier_backend"] == "gloo"


def test_two_rank_rehearsal_under_torch_distributed_run():
    """The driver's launcher (`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`):
    the ranks come from the launcher's environment, not from bench.py's own spawn."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2"]
    p = subprocess.run(cmd + ARGS + ["--allow-shared-gpu"], capture_output=True, text=True, timeout=300, env=_env(),
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0's line only
    line = json.loads(lines[0])
    assert line["ranks"] == 2 and line["verified"] is True
    assert line["secondary"]["shard1b"]["shards"] == [[0, 500_000_000], [500_000_000, 1_000_000_000]]
    assert [r["rank"] for r in json.load(open(os.path.join(ROOT, line["detail"])))["per_rank"]] == [0, 1]
    assert line["barrier_backend"] == "gloo"
