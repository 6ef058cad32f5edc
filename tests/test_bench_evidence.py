"""The bench line's counter evidence is tied to committed PMC files of the kernels that run:
the roofline's `traffic` and the `counters` object come from profiles/pmc_<workload>.json only when that file
measured the same kernel instantiation at the same batch size."""
import bench


def test_pmc_traffic_matches_the_running_instantiation():
    sym = bench.ensemble_symbol(0, True)  # N = 1: column outputs, wide chunk layout
    t = bench.pmc_traffic("config4", 65536, sym)
    assert t is not None and t > 18_000_000  # at least the algorithmic 18.6 MB per launch
    assert bench.pmc_traffic("config4", 1024, sym) is None  # another batch size
    assert bench.pmc_traffic("config4", 65536, bench.ensemble_symbol(1, False)) is None  # not measured (N > 1 form)
    assert bench.pmc_traffic("config9", 65536, sym) is None  # no file


def test_pmc_counters_join_live_durations():
    groups = {"features": (["fd::anon::feat_slot_kernel", "fd::anon::feat_bucket_lean_kernel<1>"], "features"),
              "ensemble": ([bench.ensemble_symbol(0, True)], "ens")}
    c = bench.pmc_counters("config4", 65536, groups, {"features": 70.0, "ens": 90.0})
    f, e = c["features"], c["ensemble"]
    # the 64 k step launch of the slot kernel, not the warm-history setup's large ones
    assert 1e6 < f["hbm_bytes_per_launch"] < 2e8 and set(f["l2_hit_rate"]) == set(groups["features"][0])
    assert abs(e["achieved_GBs"] - e["hbm_bytes_per_launch"] / 90e-6 / 1e9) < 0.01
    c5 = bench.pmc_counters("config5", 1024, {"lstm": ([bench.LSTM4_SYMBOL], "lstm_head")}, {"lstm_head": 22.0})
    assert 0.0 < c5["lstm"]["mfma_busy"][bench.LSTM4_SYMBOL] <= 1.0
    assert bench.pmc_counters("config4", 4096, groups, {}) is None
