"""bench.py host logic (no GPU): the defaults the driver relies on, the workload / config
naming, the PMC-traffic lookup and the CPU-core accounting of the baseline."""
import csv
import json
import statistics
import sys

import pytest

import bench


def _args(monkeypatch, *argv):
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
    return bench.parse()


def test_defaults_are_the_driver_contract(monkeypatch):
    a = _args(monkeypatch)
    assert (a.gpus, a.steps, a.warmup) == (1, 50, 5)
    assert a.n is None and a.k is None          # -> N = 65536, k = 256 in main()
    assert a.workload == "rbf" and a.storage == "auto"
    assert a.configs3_n == 131072               # the configs[3] leg rides along on every N
    a = _args(monkeypatch, "--gpus", "8", "--steps", "20", "--warmup", "5")
    assert (a.gpus, a.steps, a.warmup) == (8, 20, 5)
    assert a.n is None                          # value stays the configs[2] problem at N > 1


def test_metric_matches_baseline():
    base = json.loads((bench.REPO / "BASELINE.json").read_text())
    assert bench.METRIC == base["metric"]


def test_reference_step_times_are_baseline_md():
    # 0.105 s (N = 15540), 2.073 s (~157k), 6.600 s (~505k)
    assert bench.REF_STEP_S == {15540: 0.105, 156510: 2.073, 505050: 6.600}


def test_pmc_traffic_is_refused_when_stale(tmp_path, monkeypatch):
    """bench.py reports PMC traffic only for entries collected on the current sources
    (scripts/pmc_head.py stamps csrc_sha); anything else is null with the reason."""
    key = "rbf_n65536_nystrom256/sym/gpus1"
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_traffic.json").write_text(json.dumps({
        key: {"hbm_bytes_per_launch": 1.7e10, "csrc_sha": bench.csrc_hash()},
        "old/sym/gpus1": {"hbm_bytes_per_launch": 1.0, "csrc_sha": "0123456789abcdef"},
        "unstamped/sym/gpus1": {"hbm_bytes_per_launch": 1.0}}))
    real = bench.REPO
    monkeypatch.setattr(bench, "library_hash", lambda: bench.csrc_hash())
    monkeypatch.setattr(bench, "REPO", tmp_path)
    (tmp_path / "mlff-preconditioner_amd").symlink_to(real / "mlff-preconditioner_amd")
    (tmp_path / "include").symlink_to(real / "include")
    assert bench.pmc_traffic(key) == (1.7e10, None)
    for k in ("old/sym/gpus1", "unstamped/sym/gpus1"):
        v, why = bench.pmc_traffic(k)
        assert v is None and why.startswith("stale")
    v, why = bench.pmc_traffic("no_such/sym/gpus1")
    assert v is None and "no PMC entry" in why
    # a binary built from other sources: refused whatever the entry says
    monkeypatch.setattr(bench, "library_hash", lambda: "feedfacefeedface")
    v, why = bench.pmc_traffic(key)
    assert v is None and why.startswith("binary/source mismatch")


def test_usable_cores_is_consistent():
    c = bench.usable_cores()
    assert c["cores"] >= 1
    assert c["cores"] <= c["affinity_cpus"]
    if c["cgroup_quota_cpus"] is not None:
        assert c["cores"] <= max(1, int(c["cgroup_quota_cpus"]))


def test_timing_every_brackets_some_steps():
    """The timed region brackets every timing_every(steps)-th iteration: at least 4 (or all)
    of any run of `steps` consecutive iterations are bracketed, so the per-kernel averages
    of the line always exist (a 5-step run once divided by zero bracketed iterations)."""
    for steps in (1, 2, 3, 5, 10, 20, 50, 200):
        e = bench.timing_every(steps)
        assert 1 <= e <= bench.TIMING_EVERY
        for first in range(1, 3 * e + 2):
            hits = sum(1 for it in range(first, first + steps) if it % e == 0)
            assert hits >= min(4, steps), (steps, e, first, hits)


def test_pmc_head_medians_optional_kernels(tmp_path):
    """scripts/pmc_head.py folds the last STEPS dispatches of every kernel of a group; a kernel
    marked '?' (k_mf_z: launched only where Zt is stored) may be absent."""
    sys.path.insert(0, str(bench.REPO / "scripts"))
    import pmc_head

    d = tmp_path / "pass"
    d.mkdir()
    names = ["void mlff::(anonymous namespace)::k_rec_g<1, false, 8, 4, 16, true>(RecArgs)",
             "void mlff::(anonymous namespace)::k_rec_fin<true>(double const*, int)"]
    with open(d / "x_counter_collection.csv", "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Value"])
        for i in range(10):
            w.writerow([2 * i, names[0], 100 + i])
            w.writerow([2 * i + 1, names[1], 10 + i])
    m = pmc_head.medians(d, pmc_head.GROUPS["matfree"])
    assert set(m) == {"k_rec_g", "k_rec_fin"}              # k_mf_z? absent: skipped
    steps = pmc_head.STEPS
    assert m["k_rec_g"] == (statistics.median(range(110 - steps, 110)), steps)
    with pytest.raises(SystemExit):
        pmc_head.medians(d, ["k_symv_dyn"])                 # a required kernel must be there


def test_iteration_bytes_use_the_apply_form_that_ran():
    """iter_gbs_algorithmic counts the low-rank apply's bytes as the library reports them for
    the form that ran (one pass: T read once), not the two-pass 16 k N: the round-3 nanotube
    line (k = 2701, one-pass apply 397.6 MB, operator 32.8 MB) is 431.3 MB per iteration, not
    the 7.59 TB/s-worth two-pass figure."""
    n, k = 15540, 2701
    one_pass = 8.0 * k * n + 16.0 * 256 * n + 24.0 * n
    b = bench.iteration_bytes(32.8e6, one_pass, n)
    assert b == pytest.approx(32.8e6 + one_pass + 56.0 * n)
    assert b < 32.8e6 + 16.0 * k * n                   # below the two-pass count
    assert bench.iteration_bytes(1e9, 0.0, n) == 1e9 + 56.0 * n   # no preconditioner


def test_many_point_workload_arguments(monkeypatch):
    """The ethanol legs at the reference's published sizes: matrix-free
    storage with a chosen operator form, and the reference step times they are quoted against."""
    a = _args(monkeypatch, "--workload", "ethanol", "--m", "5833", "--storage", "matfree",
              "--mf-form", "pt")
    assert (a.workload, a.m, a.storage, a.mf_form) == ("ethanol", 5833, "matfree", "pt")
    assert 27 * 583 in bench.REF_STEP_S_ETHANOL and 27 * 2777 in bench.REF_STEP_S_ETHANOL
    assert bench.REF_STEP_S_ETHANOL[27 * 5833] == 0.550
    assert _args(monkeypatch).mf_form is None          # the library's default form


def test_self_launch_plan(monkeypatch):
    """Plain `bench.py --gpus N` (no WORLD_SIZE): N rank processes of the same script and
    arguments, rank r on device r, the torchrun variables set, rendezvous on 127.0.0.1."""
    argv = ["--gpus", "4", "--steps", "3", "--warmup", "1"]
    plans = bench.spawn_plan(argv, 4, 29511, {"KEEP": "1", "WORLD_SIZE": "9"})
    assert len(plans) == 4
    for r, (cmd, env) in enumerate(plans):
        assert cmd[0] == sys.executable and cmd[-len(argv):] == argv
        assert cmd[-len(argv) - 1].endswith("bench.py")
        assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"]) == (str(r), str(r), "4")
        assert env["LOCAL_WORLD_SIZE"] == "4" and env["KEEP"] == "1"
        assert (env["MASTER_ADDR"], env["MASTER_PORT"]) == ("127.0.0.1", "29511")
    assert 0 < bench.free_port() < 65536


def test_main_self_launches_without_world_size(monkeypatch):
    """main() hands `--gpus N > 1` without WORLD_SIZE to launch_ranks before it imports the
    library, and exits with its status; under torchrun (WORLD_SIZE set) it does not."""
    seen = {}

    def fake_launch(plans, timeout):
        seen["n"], seen["timeout"] = len(plans), timeout
        return 7

    monkeypatch.setattr(bench, "launch_ranks", fake_launch)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "2"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7 and seen == {"n": 8, "timeout": 1800.0}


def _plan(codes_sleep):
    """Fake ranks: rank r sleeps s_r seconds, then exits with c_r."""
    plans = []
    for r, (c, s) in enumerate(codes_sleep):
        plans.append(([sys.executable, "-c", f"import time, sys; time.sleep({s}); sys.exit({c})"],
                      {"RANK": str(r), "PATH": "/usr/bin:/bin"}))
    return plans


def test_launch_ranks_propagates_exit_status():
    import time

    assert bench.launch_ranks(_plan([(0, 0), (0, 0.2), (0, 0)]), timeout=60) == 0
    # rank 1 fails while rank 0 would run for a minute: rank 0 is stopped, its status returned
    t0 = time.monotonic()
    assert bench.launch_ranks(_plan([(0, 60), (3, 0.1)]), timeout=120) == 3
    assert time.monotonic() - t0 < 30
    # ranks past the timeout are stopped: 124
    t0 = time.monotonic()
    assert bench.launch_ranks(_plan([(0, 60), (0, 60)]), timeout=1) == 124
    assert time.monotonic() - t0 < 30


def test_exact_anchor_fixture_is_consistent():
    """tests/golden/rbf_dd_n65536.json (make_dd_anchor.py, GPU): the anchor the bench's
    solve_to_1e-6 holds the configs[2] count to; its oracle fractions restate the committed
    long-double and six-order band files."""
    a = bench.exact_anchor()
    assert a is not None and a["n"] == 65536 and a["k"] == 256 and a["info"] == 0
    g = bench.REPO / "tests" / "golden"
    for n in (8192, 16384):
        ld = json.loads((g / f"rbf_ld_n{n}.json").read_text())["iters"]
        bd = json.loads((g / f"rbf_band_n{n}.json").read_text())
        assert a["anchors"][str(n)]["oracle_long_double"] == ld
        frac = max(abs(v["iters"] - ld) for v in bd["variants"].values()) / ld
        assert a["fp64_distance_fraction"][f"oracle_fp64_n{n}"] == pytest.approx(frac)
    assert a["oracle_fp64_iters"]["rbf_solve_n65536.npz"] == 8528
