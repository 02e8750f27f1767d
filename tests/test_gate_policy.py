"""N7 counter-gate policy (native/include/gate_policy.h) through the
validator's ``--check-gate`` mode: the same code the validator runs on the
counters of its counted GEMM, here fed counter tuples on the CPU.

Healthy tuple: the MI355X values of profiles/r2_gate/aql_v2.json (4096^3,
256 CUs, 8 GRBM instances)."""

import json
import pathlib
import re
import subprocess

import pytest

from amdgpu_operator import native

VALIDATOR = str(native.binary("amdgpu-validator"))
_HDR = (pathlib.Path(__file__).resolve().parents[1] / "native" / "include" / "gemm_default.h").read_text()
WPT = int(re.search(r"kGemmWavesPerTile = (\d+);", _HDR).group(1))  # waves per 256x256 tile of the default GEMM
N = 4096
MOPS = 2 * N ** 3 // 512          # 268,435,456
WAVES = (N // 256) ** 2 * WPT     # 1,024 (4 waves a tile)
BUSY = MOPS // 2                  # 134,217,728 (measured: exactly MOPS/2)
GUI = 2134600                     # 8 XCDs summed (~267 k cycles each)


def verdict(m=N, n=N, k=N, cus=256, mops=MOPS, busy=BUSY, waves=WAVES, gui=GUI, samples=8, min_util=0.2):
    spec = ",".join(str(x) for x in (m, n, k, cus, mops, busy, waves, gui, samples))
    p = subprocess.run([VALIDATOR, "--check-gate", spec, "--min-mfma-util", str(min_util)],
                       capture_output=True, text=True, timeout=30)
    out = json.loads(p.stdout)
    assert (p.returncode == 0) == out["ok"]
    return out


def test_healthy_mi355x_counters_pass():
    v = verdict()
    assert v["ok"] and v["reason"] == ""
    assert v["expected_mops"] == MOPS and v["expected_waves"] == WAVES
    assert v["mfma_util"] == pytest.approx(0.4912, abs=1e-3)


@pytest.mark.parametrize("field,delta,why", [
    ("waves", -1, "SQ_WAVES"), ("waves", +1, "SQ_WAVES"), ("waves", -WPT, "SQ_WAVES"),
    ("mops", -1, "MFMA_MOPS"), ("mops", +1, "MFMA_MOPS"), ("mops", -32, "MFMA_MOPS")])
def test_off_by_one_counts_fail_closed(field, delta, why):
    kw = {"mops": MOPS, "waves": WAVES}
    kw[field] += delta
    v = verdict(**kw)
    assert not v["ok"] and why in v["reason"]


def test_below_busy_ratio_fails_closed():
    # the same work spread over 3x the elapsed cycles: a starved matrix pipe
    v = verdict(gui=GUI * 3)
    assert not v["ok"] and "below floor" in v["reason"]
    assert v["mfma_util"] < 0.2 <= v["mfma_util_floor"] + 1e-9


def test_inconsistent_or_missing_counters_fail_closed():
    assert "not counted" in verdict(busy=0)["reason"]
    assert "not counted" in verdict(gui=0)["reason"]
    assert "not counted" in verdict(samples=0)["reason"]
    assert "> 1" in verdict(gui=GUI // 4)["reason"]  # busier than every SIMD every cycle
    assert "CU count" in verdict(cus=0)["reason"]
    assert "multiple" in verdict(m=4000, n=4000, k=4000)["reason"]


def test_floor_scales_with_occupancy():
    # 1024^3 plugin-pod GEMM: 16 tiles on 256 CUs -> 1/16 of the floor
    n = 1024
    mops, waves = 2 * n ** 3 // 512, (n // 256) ** 2 * WPT
    v = verdict(m=n, n=n, k=n, mops=mops, busy=mops // 2, waves=waves, gui=8 * 40000)
    assert v["mfma_util_floor"] == pytest.approx(0.2 / 16)
    assert v["ok"], v
    # a CPX partition (32 CUs) runs 4096^3 at full occupancy: full floor
    v = verdict(cus=32, gui=GUI // 8 * 8, samples=1)
    assert v["mfma_util_floor"] == pytest.approx(0.2)


@pytest.mark.parametrize("kw,kind", [
    ({"waves": WAVES + 262}, "preempted"),                         # a queue remap restored our waves
    ({"gui": GUI * 4}, "preempted"),                               # our dispatch waited, the GPU stayed busy
    ({"mops": MOPS + 4096, "waves": WAVES + 64}, "foreign_mfma"),  # another process's MFMA kernel in the window
    ({"mops": MOPS // 2 + 8192, "waves": WAVES + 64}, ""),         # short of 2MNK even with foreign work: final
    ({"mops": MOPS * 2 + 22176832}, "foreign_mfma"),               # a resident co-tenant GEMM: our waves exact
    ({"mops": MOPS - 512}, ""),                                    # dropped work: final
    ({"waves": WAVES - 4}, ""),                                    # missing waves: final
])
def test_retry_only_on_other_parties_signatures(kw, kind):
    """Which failed windows aql_gate counts again (gate_policy.h
    gate_retry_kind): only those another process's work explains.  None of
    them passes - a pass needs the exact equalities on one attempt."""
    v = verdict(**kw)
    assert not v["ok"]
    assert v["retry"] == kind


def test_floor_zero_reports_only_but_equalities_still_hold():
    assert verdict(gui=GUI * 50, min_util=0)["ok"]
    assert not verdict(waves=WAVES - 1, min_util=0)["ok"]
