"""bench.py's process setup without a GPU: the RCCL ("nccl") branch binds each rank to device
LOCAL_RANK and hands that device to init_process_group (the communicator's device), --one-device puts
every rank on device 0, gloo keeps scalars on the host, and a single process initialises no group.
torch.cuda.set_device / dist.init_process_group are recorded, not called."""
import argparse
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


@pytest.fixture
def recorded(monkeypatch):
    calls = {"set_device": [], "init": []}
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: calls["set_device"].append(d))
    monkeypatch.setattr(dist, "init_process_group", lambda *a, **k: calls["init"].append((a, k)))
    return calls


def _args(backend="nccl", one_device=False):
    return argparse.Namespace(backend=backend, one_device=one_device)


def test_nccl_rank_binds_its_local_device(recorded):
    env = {"WORLD_SIZE": "8", "RANK": "13", "LOCAL_RANK": "5"}
    rank, world, dev, sdev = bench.init_rank(_args(), env)
    assert (rank, world) == (13, 8) and dev == torch.device("cuda", 5) and sdev == dev
    assert recorded["set_device"] == [5]
    assert recorded["init"] == [(("nccl",), {"device_id": torch.device("cuda", 5)})]
    assert env["MASTER_ADDR"] == "127.0.0.1"


def test_one_device_and_gloo(recorded):
    rank, world, dev, sdev = bench.init_rank(_args("gloo", True), {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"})
    assert dev == torch.device("cuda", 0) and sdev == torch.device("cpu")
    assert recorded["set_device"] == [0] and recorded["init"] == [(("gloo",), {})]


def test_single_process_initialises_no_group(recorded):
    rank, world, dev, sdev = bench.init_rank(_args(), {})
    assert (rank, world) == (0, 1) and dev == torch.device("cuda", 0)
    assert recorded["init"] == []


def test_strong_scaling_configs_share_the_cloud():
    """--strong-configs only accepts frames of the 512^3 cloud (the grid is built once)."""
    with pytest.raises(ValueError, match="c4"):
        bench.strong_scaling(["c4"], None, 0, 2, torch.device("cuda", 0), torch.device("cpu"), 1, 0, None)
    with pytest.raises(ValueError, match="unknown mode"):
        bench.strong_scaling(["c3:fast"], None, 0, 2, torch.device("cuda", 0), torch.device("cpu"), 1, 0, None)


def test_request_roofline_uses_the_configs_own_counter_pass():
    """Counter passes of other workloads (tools/kernel_counters.sh ... --grid-n N: bench_args set) never
    feed the bench line's request_frac."""
    import json
    from pathlib import Path

    import bench

    r = bench.request_roofline("c3", 5.3e8, 0.35, 256)
    src = r["request_sources"][0]
    assert not json.loads((Path(bench.ROOT) / src).read_text()).get("bench_args"), src


def test_pipe_roofline_two_request_classes():
    """pipe_frac: stencil pieces at the pool-size gather ceiling plus the other requests at the L2 ceiling,
    from the committed counter / ceiling files; log-log interpolation between measured pool sizes."""
    pts = [(200.0, 4.0e8), (800.0, 2.0e8)]
    assert bench.interp_loglog(pts, 400.0) == pytest.approx(2.0e8 * 2 ** 0.5)
    assert bench.interp_loglog(pts, 100.0) == 4.0e8 and bench.interp_loglog(pts, 1600.0) == 2.0e8
    r = bench.pipe_roofline("c3", 5.95e6, 11.857, 797.2)
    assert r["pipe_frac"] is not None and 0.3 < r["pipe_frac"] < 1.2, r
    assert r["pipe_frac"] == pytest.approx(r["pipe_stencil_share"] + r["pipe_other_share"], abs=2e-4)
    assert all(src and src.startswith("profiles/") for src in r["pipe_sources"])
    assert bench.pipe_roofline("no-such-config", 5.95e6, 11.857, 797.2) == {"pipe_frac": None}
