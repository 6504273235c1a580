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


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("cfg,ranks,steps", [("C1", 2, 2), ("C4", 2, 2), ("C3", 3, 1)])
def test_bench_multi_rank_harness_on_cpu(cfg, ranks, steps):
    """bench.py's N>1 control flow as the driver launches it (torch.distributed.run, one process per
    rank, gloo control plane), with RCCL replaced by a host transport (--host-rehearsal): the
    unique-id broadcast, check_comm_ranks on the group's real (size, rank), the weak/strong spp
    split, the shard capacities, the timed region's barriers and max over ranks, and the gather to
    rank 0 placed by om_shard_assemble_host (bench.py asserts every pixel's sample count and place).
    What stays unmeasured: RCCL itself with nranks > 1."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(ranks), "--host-rehearsal", "--config", cfg, "--steps", str(steps), "--warmup", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout                                  # rank 0 only
    d = lines[0]
    import bench as b
    W, H = b.CONFIGS[cfg].get("size", (1920, 1080))
    assert d["host_rehearsal"] and d["n_ranks"] == ranks and d["nranks_seen"] == ranks
    assert (d["W"], d["H"]) == (W, H)
    # C4 renders the fixed frame (strong scaling); the others render spp x N on 1/N of the tiles
    assert d["spp_step"] == b.SPP_PER_STEP * (1 if cfg == "C4" else ranks)
    assert d["spp_total"] == d["spp_step"] * steps
    tiles = ((W + 7) // 8) * ((H + 7) // 8)
    assert d["shard_capacity"] == -(-tiles // ranks) * 64 and d["shard_pixels"] <= d["shard_capacity"]
