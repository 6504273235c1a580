"""bench.py's host-side checks, on the CPU: the RCCL rank check the N>1 line depends on
 and the PMC fields the roofline copies from the committed summaries."""
import os

import pytest


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


def test_comm_rank_check_passes_and_fails_loudly(bench):
    assert bench.check_comm_ranks((1, 0), 1, 0) == 1
    assert bench.check_comm_ranks((8, 5), 8, 5) == 8
    with pytest.raises(SystemExit, match=r"RCCL communicator has 1 ranks \(this is rank 0\), but WORLD_SIZE=2 RANK=1"):
        bench.check_comm_ranks((1, 0), 2, 1)
    with pytest.raises(SystemExit, match="WORLD_SIZE=8 RANK=3"):
        bench.check_comm_ranks((8, 2), 8, 3)


@pytest.mark.parametrize("cfg", ["C1", "C2", "C3"])
def test_pmc_fields_from_committed_summaries(bench, cfg):
    if not os.path.exists(bench.PMC_SUMMARY.format(cfg)):
        pytest.skip(f"no committed PMC summary for {cfg}")
    f = bench.pmc_fields(cfg)
    assert 0.0 < f["valu_lane_utilisation"] <= 1.0 and 0.0 <= f["wait_any_frac"] <= 1.0
    assert f["per_kernel"] and abs(sum(k["wave_cycle_share"] for k in f["per_kernel"].values()) - 1.0) < 1e-3
    assert bench.pmc_fields("C9") is None
