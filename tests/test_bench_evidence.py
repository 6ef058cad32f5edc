"""The bench line's counter evidence is tied to committed PMC files of the kernels that run:
the roofline's `traffic` and the `counters` object come from profiles/pmc_<workload>.json only when that file
measured the same kernel instantiation at the same batch size and grid (another launch's counters are
never reported as this one's). Checked on a synthetic summary in the format tools/pmc_kernels.py writes."""
import json

import bench


def _summary(tmp_path, workload="config4", batch=65536):
    ens = bench.ensemble_symbol(0, True)
    doc = {"batch": batch, "kernels": {
        ens: {"hbm_bytes_per_launch": 29_700_000, "l2_hit_rate": 0.92, "dispatches": 40},
        "fd::anon::feat_slot_kernel [grid 65536]": {"hbm_bytes_per_launch": 18_400_000, "l2_hit_rate": 0.69,
                                                    "dispatches": 40},
        "fd::anon::feat_slot_kernel [grid 1048576]": {"hbm_bytes_per_launch": 300_000_000, "l2_hit_rate": 0.5,
                                                      "dispatches": 400},
        "fd::anon::feat_bucket_lean_kernel<1> [grid 65536]": {"hbm_bytes_per_launch": 53_200_000,
                                                              "l2_hit_rate": 0.81, "dispatches": 40},
        "fd::anon::feat_bucket_kernel<1> [grid 1048576]": {"hbm_bytes_per_launch": 500_000_000, "dispatches": 400},
        bench.LSTM4_SYMBOL: {"hbm_bytes_per_launch": 3_100_000, "mfma_busy": 0.5, "dispatches": 40}}}
    (tmp_path / f"pmc_{workload}.json").write_text(json.dumps(doc))
    return ens


def test_pmc_traffic_matches_the_running_instantiation(tmp_path):
    ens = _summary(tmp_path)
    assert bench.pmc_traffic("config4", 65536, ens, root=tmp_path) == 29_700_000
    assert bench.pmc_traffic("config4", 1024, ens, root=tmp_path) is None  # another batch size
    assert bench.pmc_traffic("config4", 65536, bench.ensemble_symbol(0, False), root=tmp_path) is None
    assert bench.pmc_traffic("config4", 65536, bench.ensemble_symbol(1, False), root=tmp_path) is None
    assert bench.pmc_traffic("config9", 65536, ens, root=tmp_path) is None  # no file


def test_pmc_counters_join_live_durations_at_the_run_grid_only(tmp_path):
    ens = _summary(tmp_path)
    groups = {"features": (["fd::anon::feat_slot_kernel", "fd::anon::feat_bucket_lean_kernel<1>"], "features"),
              "ensemble": ([ens], "ens"),
              # measured only at another grid (the history's large launches): omitted, not substituted
              "full_bucket": (["fd::anon::feat_bucket_kernel<1>"], "features")}
    c = bench.pmc_counters("config4", 65536, groups, {"features": 70.0, "ens": 90.0}, root=tmp_path)
    f, e = c["features"], c["ensemble"]
    assert f["hbm_bytes_per_launch"] == 18_400_000 + 53_200_000
    assert f["pmc_entries"] == ["fd::anon::feat_slot_kernel [grid 65536]",
                                "fd::anon::feat_bucket_lean_kernel<1> [grid 65536]"]
    assert abs(e["achieved_GBs"] - 29_700_000 / 90e-6 / 1e9) < 0.01
    assert "full_bucket" not in c
    c5 = bench.pmc_counters("config4", 65536, {"lstm": ([bench.LSTM4_SYMBOL], "lstm_head")}, {"lstm_head": 22.0},
                            root=tmp_path)
    assert c5["lstm"]["mfma_busy"][bench.LSTM4_SYMBOL] == 0.5
    assert bench.pmc_counters("config4", 4096, groups, {}, root=tmp_path) is None


def test_committed_summaries_parse():
    """the committed profiles/pmc_*.json are in the format the lookup reads"""
    for p in sorted((bench.REPO / "profiles").glob("pmc_*.json")):
        d = json.loads(p.read_text())
        assert int(d["batch"]) > 0 and isinstance(d["kernels"], dict), p


def test_secondary_workloads_only_for_the_config4_line(monkeypatch):
    """The default line (config 4, N = 1) runs the other BASELINE configurations as child processes after its own
    measurements; N > 1, other workloads, the children themselves ('none') and FD_BENCH_SECONDARY=0 run none."""
    class A:
        secondary = None
    monkeypatch.delenv("FD_BENCH_SECONDARY", raising=False)
    assert bench._secondary_list(A, 1, "config4") == list(bench.SECONDARY_DEFAULT)
    assert bench._secondary_list(A, 2, "config4") == []
    assert bench._secondary_list(A, 1, "config5") == []
    A.secondary = "none"
    assert bench._secondary_list(A, 1, "config4") == []
    A.secondary = "config5, ingest,bogus,config4"
    assert bench._secondary_list(A, 1, "config4") == ["config5", "ingest"]
    A.secondary = None
    monkeypatch.setenv("FD_BENCH_SECONDARY", "0")
    assert bench._secondary_list(A, 1, "config4") == []
