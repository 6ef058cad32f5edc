"""Register budgets of the hot kernels, from the compiler's resource remarks the build records
(realtime-fraud-detection_amd/lib/kernel_resources.json, fdengine/build.py).

The pipelined stream's step depends on a residency arithmetic, not only on each kernel's speed: the fused ensemble
kernel runs four waves per SIMD (one 1024-thread workgroup per CU) and the next micro-batch's lean bucket kernel
must fit ONE more wave beside them, or the feature chain waits for ensemble workgroups to leave and the step
becomes the sum of the two (round 4: the compact prologue took the ensemble kernel from 54 to 94 VGPRs; config 4
went from 0.089 to 0.116 ms per step until it was brought back to 62)."""
import json

import pytest

from fdengine.build import RESOURCES

VGPRS_PER_SIMD_LANE = 512  # gfx950: VGPR file per SIMD lane (wave64), allocated in granules of 8


def _granule(v):
    return (v + 7) // 8 * 8


@pytest.fixture(scope="module")
def res():
    if not RESOURCES.exists():
        pytest.skip("no kernel_resources.json: build the library first (__graft_entry__.build())")
    return json.loads(RESOURCES.read_text())


def _find(res, *parts):
    hits = {k: v for k, v in res.items() if all(p in k for p in parts)}
    assert hits, f"no kernel matching {parts}"
    return hits


def test_ensemble_and_lean_bucket_share_a_simd(res):
    ens = _find(res, "ensemble_kernelILi8E")
    lean = _find(res, "feat_bucket_lean_kernelILi1E")
    worst_ens = max(v["vgpr"] for v in ens.values())
    worst_lean = max(v["vgpr"] for v in lean.values())
    assert 4 * _granule(worst_ens) + _granule(worst_lean) <= VGPRS_PER_SIMD_LANE, (worst_ens, worst_lean)


@pytest.mark.parametrize("parts", [("ensemble_kernelILi8E",), ("feat_slot_kernel",), ("feat_bucket_lean_kernel",),
                                   ("split_walk_pair_kernel",), ("split_sum_pair_blend_kernel",),
                                   ("lstm_kernel4",), ("feat_bucket_gather_kernel",)])
def test_hot_kernels_do_not_spill(res, parts):
    for name, v in _find(res, *parts).items():
        assert v["scratch"] == 0, f"{name} spills {v['scratch']} B/lane"


def test_ingest_keeps_four_waves_per_simd(res):
    for name, v in _find(res, "ingest_json_kernel").items():
        assert v["vgpr"] <= 128 and v["occupancy"] >= 4, (name, v)
