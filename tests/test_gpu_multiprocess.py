"""The multi-GPU path with the HIP integrator in every rank: 2 processes on the box's one
GPU, torch.distributed over gloo, each rendering its share of the job space with
distributed.render_rank and summing the films with distributed.reduce_film (RCCL over xGMI on a node;
gloo through a host copy here).  The reduced film must equal the one-process HIP film and the oracle's
(sample counts exactly, XYZ to fp32 atomic-order rounding).  Also: bench.py --gpus 2 really runs two
ranks and reports n_gpus 2."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle_lib as O
from conftest import assert_hip_untouched
from volume_path_tracer_amd import distributed as D
from volume_path_tracer_amd.scenes import SynthGrid, workload

ROOT = Path(__file__).resolve().parents[1]
pytestmark = [pytest.mark.gpu, pytest.mark.spawns]

W, H, GRID = 64, 40, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, spp, out_dir):
    sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
    import torch
    import torch.distributed as dist

    from volume_path_tracer_amd import distributed as D
    from volume_path_tracer_amd.render import Integrator
    from volume_path_tracer_amd.scenes import SynthGrid, workload

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wl = workload("c3", width=W, height=H, spp=spp, grid_n=GRID)
    it = Integrator(wl.cfg, SynthGrid(1, GRID).grid(), None, device=0)
    D.render_rank(it, rank, world, spp, mode)
    D.reduce_film(it.film)
    torch.cuda.synchronize()
    if rank == 0:
        np.save(Path(out_dir) / "reduced.npy", it.film.cpu().numpy())
        it.film.zero_()
        it.render_jobs(0, it.jobs_per_wave * D.total_samples_per_pixel(world, spp, mode))
        np.save(Path(out_dir) / "single.npy", it.film_host())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["weak", "strong"])
def test_hip_integrator_world2_gloo(mode, tmp_path):
    import torch.multiprocessing as mp

    assert_hip_untouched()
    spp, world = 4, 2
    mp.start_processes(_worker, args=(world, _free_port(), mode, spp, str(tmp_path)), nprocs=world,
                       start_method="spawn")
    got, single = np.load(tmp_path / "reduced.npy"), np.load(tmp_path / "single.npy")
    total = D.total_samples_per_pixel(world, spp, mode)
    wl = workload("c3", width=W, height=H, spp=total, grid_n=GRID)
    ref, _, _ = O.render_jobs(wl.cfg, O.OracleGrid(SynthGrid(1, GRID).grid()), None, 0, wl.cfg.jobs_per_wave() * total)
    for f in (got, single):
        np.testing.assert_array_equal(f[..., 3], float(total))
        np.testing.assert_allclose(f[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)
    # one process, one launch: the ordered film is the oracle's bit for bit (the reduced film sums two ranks'
    # partial films, a different fp32 association)
    assert single.tobytes() == ref.tobytes()


def _rccl_worker(rank, world, port, out_dir):
    sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
    import torch
    import torch.distributed as dist

    from volume_path_tracer_amd import distributed as D
    from volume_path_tracer_amd.render import Integrator
    from volume_path_tracer_amd.scenes import SynthGrid, workload

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)  # as bench.init_rank does
    wl = workload("c3", width=W, height=H, spp=3, grid_n=GRID)
    it = Integrator(wl.cfg, SynthGrid(1, GRID).grid(), None, device=0)
    D.render_rank(it, rank, world, 3, "weak")
    torch.cuda.synchronize()
    before = it.film.clone()
    # the collectives the multi-GPU path issues: the film's device-pointer all-reduce (reduce_film's call) and the
    # bench's scalar MAX / SUM reductions on the device
    dist.all_reduce(it.film, op=dist.ReduceOp.SUM)
    t = torch.tensor([2.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n = torch.tensor([7.0], dtype=torch.float64, device=dev)
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    torch.cuda.synchronize()
    info = {"backend": dist.get_backend(), "film_unchanged": bool(torch.equal(before, it.film)),
            "max": float(t.item()), "sum": float(n.item()),
            "rccl_version": ".".join(str(x) for x in torch.cuda.nccl.version())}
    (Path(out_dir) / "rccl.json").write_text(json.dumps(info))
    np.save(Path(out_dir) / "film.npy", it.film.cpu().numpy())
    dist.destroy_process_group()


def test_rccl_one_rank_film_all_reduce(tmp_path):
    """RCCL itself on the MI355X: a one-rank "nccl" process group bound to device 0 -- the
    library load, communicator init and the device-pointer all-reduce of an Integrator's film that
    distributed.reduce_film issues on a node (RCCL refuses two ranks on one GPU, so world 1 is what one box can
    run).  The film comes back unchanged, the counts exact and the film the oracle's bit for bit."""
    import torch.multiprocessing as mp

    assert_hip_untouched()
    mp.start_processes(_rccl_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, start_method="spawn")
    info = json.loads((tmp_path / "rccl.json").read_text())
    print("rccl:", info)
    assert info["backend"] == "nccl" and info["film_unchanged"] and info["max"] == 2.5 and info["sum"] == 7.0
    film = np.load(tmp_path / "film.npy")
    wl = workload("c3", width=W, height=H, spp=3, grid_n=GRID)
    ref, _, _ = O.render_jobs(wl.cfg, O.OracleGrid(SynthGrid(1, GRID).grid()), None, 0, wl.cfg.jobs_per_wave() * 3)
    np.testing.assert_array_equal(film[..., 3], 3.0)
    assert film.tobytes() == ref.tobytes()


def test_bench_gpus2_spawns_two_ranks(tmp_path):
    """bench.py --gpus 2 without torchrun's environment starts 2 ranks itself (before touching the
    GPU); here both share the box's one GPU over gloo (--backend gloo --one-device)."""
    assert_hip_untouched()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--spp", "2", "--no-cpu-baseline", "--backend", "gloo", "--one-device", "--strong-configs", "c3,c3:pixel"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["value"] > 0
    # and the strong-scaling record: the whole C3 frame dealt over the 2 ranks, timed the same way
    s = line["scaling_strong"]["c3"]
    assert s["value"] > 0 and s["ms_per_step"] > 0 and "1920x1080, 256 spp" in s["workload"]
    # ... with its own 1-GPU time of the same frame (rank 0 alone) and the speedup / efficiency from it
    assert s["one_gpu_ms_per_step"] > 0
    assert s["speedup_vs_1gpu"] == pytest.approx(s["one_gpu_ms_per_step"] / s["ms_per_step"], rel=2e-3)
    assert s["efficiency"] == pytest.approx(s["speedup_vs_1gpu"] / 2, rel=2e-3)
    p = line["scaling_strong"]["c3:pixel"]  # the same frame in the throughput mode, labelled as such
    assert p["value"] > 0 and "throughput mode" in p["workload"]
    # WORLD_SIZE that disagrees with --gpus is an error
    env2 = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r2 = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"], cwd=ROOT, env=env2,
                        capture_output=True, text=True, timeout=120)
    assert r2.returncode != 0 and "WORLD_SIZE" in r2.stderr
