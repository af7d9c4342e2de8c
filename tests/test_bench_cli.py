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
                          "GRBM_GUI_ACTIVE": 8.0, "SQ_WAIT_ANY": 30.0, "SQ_WAVE_CYCLES": 100.0}, 250 * 1024.0,
                         fetch_factor=2.0, valu_sat=[2.0, 4.0])
    assert f["traffic"] == 250 * 1024.0 and f["traffic_over_algorithmic"] == 1.0
    assert f["traffic_from"].startswith("FETCH_SIZE")
    # the per-size request counts win when present: 32/64/128-B requests, exact bytes
    g = bench.pmc_fields({"FETCH_SIZE": 100.0, "WRITE_SIZE": 50.0, "TCC_EA0_RDREQ_32B_sum": 2.0,
                          "TCC_EA0_RDREQ_64B_sum": 1.0, "TCC_EA0_RDREQ_128B_sum": 1600.0}, 1.0)
    assert g["read_bytes"] == 32 * 2 + 64 + 128 * 1600 and g["traffic"] == g["read_bytes"] + 50 * 1024.0
    assert g["traffic_fetch_calibrated"] == 250 * 1024.0
    assert f["valu_busy"] == 4.0 and f["valu_busy_range"] == [1.0, 2.0]
    assert f["wait_frac"] == 0.3
    assert bench.limiter(0.95, 0.5) == "hbm"
    assert bench.limiter(0.5, 0.9) == "valu"
    assert bench.limiter(None, 0.9).startswith("unknown")


def test_rank_envs_for_eight_gpus():
    envs = bench.rank_envs(8, 29500, base={"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == [str(r) for r in range(8)]
    assert [e["LOCAL_RANK"] for e in envs] == [str(r) for r in range(8)]
    assert all(e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "8" and e["MASTER_ADDR"] == "127.0.0.1"
               and e["MASTER_PORT"] == "29500" and e["PATH"] == "/bin" for e in envs)
    # every rank its own GPU on an 8-GPU node
    assert [bench.plan_device(r, 8, 8, False) for r in range(8)] == [(r, False) for r in range(8)]


def test_grid_threads_match_the_launchers():
    assert bench.grid_threads("fixed16", 10_000_000) == 10_000_128
    assert bench.grid_threads("fixed256", 100) == 128
    assert bench.grid_threads("var", 100_000_000) == 781_250 * 128  # 1 562 500 tiles, two per workgroup
    assert bench.grid_threads("var", 65) == 128
    assert bench.grid_threads("tabpart", 1024) == 1024 * 512
    assert bench.grid_threads("winorder", 10_000_000) == 2442 * 256  # one 256-thread workgroup per 4096 keys
    assert bench.grid_threads("ceil_read16", 64) == 256
    assert bench.grid_threads("ceil_read16w1", 128) == 128
    assert bench.grid_threads("ceil_copynt", 10_000_000) == 10_000_128


def test_parse_pmc_rows_keys_on_kernel_and_grid():
    rows = [{"Kernel_Name": "void shfhb::k_fixed16<0>(...)", "Grid_Size": "256", "Counter_Name": "FETCH_SIZE",
             "Counter_Value": "10"},
            {"Kernel_Name": "void shfhb::k_fixed16<0>(...)", "Grid_Size": "512", "Counter_Name": "FETCH_SIZE",
             "Counter_Value": "99"},
            {"Kernel_Name": "shfhb::(anonymous namespace)::k_ceil_copy(...)", "Grid_Size": "256",
             "Counter_Name": "FETCH_SIZE", "Counter_Value": "5"},
            {"Kernel_Name": "void shfhb::(anonymous namespace)::k_ceil_copyv<1>(...)", "Grid_Size": "256",
             "Counter_Name": "FETCH_SIZE", "Counter_Value": "7"}]
    v = bench.parse_pmc_rows(rows, {"fixed16": 256, "ceil_copy": 256, "ceil_copynt": 256})
    assert v == {"fixed16": {"FETCH_SIZE": [10.0]}, "ceil_copy": {"FETCH_SIZE": [5.0]},
                 "ceil_copynt": {"FETCH_SIZE": [7.0]}}


def _fake_result(name, gbs, us=50.0, lanes=10_000_000, bpk=32.0):
    return {"value": 1e11, "value_min": 0.9e11, "value_max": 1.1e11, "repeats": 3, "ms_per_step": 0.05,
            "kernel_us": us, "achieved_gbs": gbs, "bytes_per_key": bpk, "lanes": lanes, "kernel": "k", "desc": name,
            "enqueue_us_per_step": 5.0}


def _args(**kw):
    a = bench.parse(["--no-cpu", "--traffic", "off"])
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_roofline_divides_by_the_ceiling_measured_in_the_run():
    results = {"fixed16": _fake_result("fixed16", 6000.0), "ceil_copy": _fake_result("ceil_copy", 6400.0),
               "ceil_copynt": _fake_result("ceil_copynt", 6300.0),
               "var": _fake_result("var", 5200.0, lanes=100_000_000, bpk=284.0)}
    pmc = {"fixed16": {"_lanes": 10_000_000, "FETCH_SIZE": 160e6 / 2 / 1024, "WRITE_SIZE": 160e6 / 1024},
           "ceil_copy": {"_lanes": 10_000_000, "FETCH_SIZE": 160e6 / 2 / 1024, "WRITE_SIZE": 160e6 / 1024}}
    cal = bench.pmc_calibration(pmc)
    assert cal["ceil_copy"] == {"fetch_factor": 2.0, "write_factor": 1.0}
    ro = bench.roofline_of("fixed16", results["fixed16"], results, pmc, cal, _args())
    assert ro["frac_of_copy_ceiling"] == round(6000.0 / 6400.0, 4)
    assert ro["copy_ceiling"]["workload"] == "ceil_copy"
    assert ro["frac"] == 0.75 and ro["traffic"] == 320e6 and ro["traffic_over_algorithmic"] == 1.0
    assert ro["fetch_factor_from"] == "ceil_copy"
    # no read-mostly ceiling in this run: no fraction (never a constant)
    rv = bench.roofline_of("var", results["var"], results, pmc, cal, _args())
    assert rv["frac_of_copy_ceiling"] is None and "not measured" in rv["copy_ceiling"]


def test_line_for_eight_ranks_carries_per_rank_fields():
    world = 8
    results = {"fixed16": _fake_result("fixed16", 6000.0), "ceil_copy": _fake_result("ceil_copy", 6300.0)}
    per_rank = [{"rank": r, "device": r, "device_name": "AMD Instinct MI355X", "shard": None,
                 "kernel_us": {"fixed16": 50.0 + r, "ceil_copy": 48.0}, "verified": {"fixed16": True}}
                for r in range(world)]
    verified = {"fixed16": {"ok": True, "samples_per_rank": 20002}}
    line = bench.build_line(_args(), world, world, False, results, verified, per_rank,
                            {"fixed16": "keys/s", "ceil_copy": "lanes/s"}, None, "not collected", None, None, None)
    assert line["n_gpus"] == 8 and line["ranks"] == 8 and "rehearsal" not in line
    assert [p["device"] for p in line["per_rank"]] == list(range(8))
    assert line["slowest_over_fastest_rank"]["fixed16"] == round(57.0 / 50.0, 4)
    assert line["slowest_over_fastest_rank"]["ceil_copy"] == 1.0
    assert line["barrier_backend"] == "gloo"
    assert line["verified"] is True and line["secondary"]["ceil_copy"]["unit"] == "lanes/s"
    json_line = bench.json.dumps(line)
    assert "all_visible_cpus_extrapolated" not in json_line and "HBM_COPY" not in json_line


def test_multi_kernel_workload_counters_sum_over_its_kernels():
    rows = []
    for k, grid, fetch in (("k_wo_rank", 625152, 100.0), ("k_wo_scan_rows", 65536, 10.0), ("k_wo_place", 625152, 5.0)):
        for rep in range(3):
            rows.append({"Kernel_Name": "void shfhb::(anonymous namespace)::%s(...)" % k, "Grid_Size": str(grid),
                         "Counter_Name": "FETCH_SIZE", "Counter_Value": str(fetch + rep)})
    rows.append({"Kernel_Name": "void shfhb::k_fixed16<0>(...)", "Grid_Size": "256", "Counter_Name": "FETCH_SIZE",
                 "Counter_Value": "7"})
    vals = bench.parse_pmc_rows(rows, {"winorder": bench.grid_threads("winorder", 10_000_000), "fixed16": 256})
    m = bench.pmc_medians(vals["winorder"])
    assert m["FETCH_SIZE"] == 101.0 + 11.0 + 6.0  # the three kernels' medians, summed
    assert bench.pmc_medians(vals["fixed16"]) == {"FETCH_SIZE": 7.0}


def _full_results():
    names = bench.HASH_WORKLOADS + bench.CEIL_WORKLOADS
    return {n: _fake_result(n, 6000.0 + i, us=50.0 + i) for i, n in enumerate(names)}


def _compact(world, cpu=None, host_inc=None):
    results = _full_results()
    verified = {n: {"ok": True, "samples_per_rank": 20002} for n in bench.HASH_WORKLOADS}
    per_rank = [{"rank": r, "device": r, "device_name": "AMD Instinct MI355X", "shard": [r * 125_000_000,
                                                                                        (r + 1) * 125_000_000],
                 "kernel_us": {n: 50.0 + r for n in results}, "verified": {n: True for n in verified}}
                for r in range(world)] if world > 1 else None
    units = {n: "lanes/s" if n.startswith("ceil_") else "keys/s" for n in results}
    full = bench.build_line(_args(), world, world, False, results, verified, per_rank, units, None, "not collected",
                            cpu, host_inc, [[0, 1]] * world)
    return full, bench.compact_line(full, "gpurun_out/bench_detail_n%d.json" % world)


def test_stdout_line_fits_the_driver_tail_at_one_and_eight_ranks():
    """BENCH_r03's 28.8-KB line overflowed the driver's ~10.7-KB tail and went
    unparsed: the stdout line is capped at 4 KB, the rest goes to the detail file."""
    cpu = {"value": 1.476e8, "unit": "keys/s", "cores": 1, "kind": "reference", "sample": "x" * 400,
           "host_cpus": {"visible": 256}, "threads16": {"value": 2.1e9, "unit": "keys/s", "cores": 16, "sample": "y"}}
    hi = {"unit": "keys/s", "note": "n" * 500, "verified": True,
          "ceilings_gbs": {"h2d": 55.71, "d2h": 56.12, "both_h2d": 40.17, "both_d2h": 40.33, "both": 80.44,
                           "h2d_pageable": 51.32, "bytes_per_copy": 160000000}}
    for k in ("fixed16_pageable", "fixed16_pinned", "fixed16_pinned_staged", "var_pageable", "var_pinned",
              "fixed16_pageable_x16", "uid16_pageable", "uid16_pinned", "uid16_pinned_staged", "hashwin16_pageable",
              "uidwin16_pageable"):
        hi[k] = {"value": 2.5e9, "value_min": 2.4123e9, "value_max": 2.6123e9, "repeats": 5, "wire_bytes": 32.0,
                 "pcie_bound": 2.51375e9, "frac_of_pcie": 0.995}
    for world in (1, 8):
        full, line = _compact(world, cpu if world == 1 else None, hi if world == 1 else None)
        s = bench.json.dumps(line)
        assert len(s) <= bench.LINE_MAX_BYTES, (world, len(s))
        back = bench.json.loads(s)
        for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
                  "roofline", "cpu_baseline", "higher_is_better", "scaling", "vs_baseline"):
            assert k in back, k
        for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
            assert k in back["roofline"], k
        assert back["n_gpus"] == world and back["detail"].endswith("n%d.json" % world)
        # every hashing line of the run keeps a short record
        assert set(back["secondary"]) == set(bench.HASH_WORKLOADS) - {"fixed16"}
        assert all(set(e) >= {"value", "frac", "frac_of_ceiling", "verified"} for e in back["secondary"].values())
        assert len(bench.json.dumps(full)) > len(s)  # the detail record keeps what the line drops
    _, line1 = _compact(1, cpu, hi)
    assert line1["cpu_baseline"]["kind"] == "reference" and line1["cpu_baseline"]["multi"]["cores"] == 16
    assert line1["host_inclusive"]["fixed16_pinned"] == [2.5, 0.995]  # [G keys/s, frac_of_pcie]
    assert line1["host_inclusive"]["uid16_pageable"] == [2.5, 0.995] and line1["host_inclusive"]["unit"] == "G keys/s"
    assert line1["host_inclusive"]["pcie_gbs"] == {"h2d": 55.71, "d2h": 56.12, "both": 80.44, "h2d_pageable": 51.32}
    _, line8 = _compact(8)
    assert "per_rank" not in line8 and line8["slowest_over_fastest_rank"]["fixed16"] == round(57.0 / 50.0, 4)


def test_pcie_bound_takes_the_tightest_ceiling():
    """A host line's PCIe bound (bench.pcie_bound): no faster than its host ->
    device bytes at the H2D ceiling, its device -> host bytes at the D2H
    ceiling, or both at the two directions' aggregate."""
    c = {"h2d": 50.0, "d2h": 40.0, "both": 60.0}
    assert abs(bench.pcie_bound(c, 16, 16) - 60e9 / 32) < 1  # symmetric: the aggregate
    assert abs(bench.pcie_bound(c, 16, 0) - 50e9 / 16) < 1  # one way: that direction
    assert abs(bench.pcie_bound(c, 4, 16) - 40e9 / 16) < 1  # mostly back: D2H
    assert abs(bench.pcie_bound(c, 16, 8) - 60e9 / 24) < 1  # UID parts: 16 in, 8 out
    # a kernel over PCIe (zero copy) moving both directions at once: the better mechanism wins
    z = dict(c, zc_h2d=52.0, zc_d2h=45.0, zc_both=84.0)
    assert abs(bench.pcie_bound(z, 16, 16) - 84e9 / 32) < 1
    assert abs(bench.pcie_bound(z, 16, 0) - 52e9 / 16) < 1
    assert abs(bench.pcie_bound(z, 4, 16) - 45e9 / 16) < 1


def test_compact_line_trims_to_the_cap_whatever_the_detail():
    full, _ = _compact(1)
    for i in range(200):  # far more secondary lines than any run has
        full["secondary"]["extra%03d" % i] = dict(full["secondary"]["var"])
    line = bench.compact_line(full, "d.json")
    assert len(bench.json.dumps(line)) <= bench.LINE_MAX_BYTES
    assert line["roofline"]["frac"] == full["roofline"]["frac"]


def test_shared_order_kernels_go_to_the_workload_that_ran_them():
    """winorder and hashwin16 share the scan and scatter kernels (same grids):
    each row goes to the workload whose own first kernel was dispatched last."""
    rows, d = [], 0
    for first, scan_val in (("k_wo_rank", 1.0), ("k_fixed16_win", 7.0)):
        for rep in range(2):
            for k, v in ((first, 100.0), ("k_wo_scan_rows", scan_val), ("k_wo_place", scan_val * 10)):
                d += 1
                rows.append({"Kernel_Name": "void shfhb::(anonymous namespace)::%s(...)" % k, "Grid_Size": "625152",
                             "Counter_Name": "FETCH_SIZE", "Counter_Value": str(v), "Dispatch_Id": str(d)})
    rows.reverse()  # file order does not matter: rows are taken in dispatch order
    g = bench.grid_threads("winorder", 10_000_000)
    vals = bench.parse_pmc_rows(rows, {"winorder": g, "hashwin16": g})
    assert bench.pmc_medians(vals["winorder"])["FETCH_SIZE"] == 100.0 + 1.0 + 10.0
    assert bench.pmc_medians(vals["hashwin16"])["FETCH_SIZE"] == 100.0 + 7.0 + 70.0


def test_a_real_run_record_leaves_room_under_the_cap():
    """The full record of a real N = 1 run on the box (round 6, with the host
    lines' PCIe fields): its stdout line keeps every block and at least 200 B
    under the 4-KB cap, so digits that differ by run cannot push a block out."""
    import os

    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r6", "bench_r6f",
                     "bench_detail_n1.json")
    if not os.path.exists(p):  # profiles/ does not travel to the GPU box
        pytest.skip("profiles/r6/bench_r6f absent")
    full = bench.json.load(open(p))
    line = bench.compact_line(full, "gpurun_out/bench_detail_n1.json")
    s = bench.json.dumps(line)
    assert len(s) <= bench.LINE_MAX_BYTES - 200, len(s)
    for k in ("host_inclusive", "secondary", "ceilings_gbs", "cpu_baseline", "roofline"):
        assert k in line, k
    assert set(line["secondary"]) == set(full["secondary"]) - {k for k in full["secondary"] if k.startswith("ceil_")}
    assert line["host_inclusive"]["uid16_pageable"][1] == full["host_inclusive"]["uid16_pageable"]["frac_of_pcie"]
