"""The N > 1 path on CPU: wave sharding + film all-reduce over gloo (world size 2) reproduces the
single-process render.  The per-rank renderer here is the CPU oracle (test infrastructure); on
GPUs it is the HIP integrator with the same job ranges (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from volume_path_tracer_amd import distributed as D


def test_partitions_cover_job_space():
    for world in (1, 2, 3, 8):
        for spp in (1, 4, 7, 64):
            strong = sorted(w for r in range(world) for a, n in D.rank_wave_ranges(r, world, spp, "strong")
                            for w in range(a, a + n))
            assert strong == list(range(1, spp + 1))
            weak = sorted(w for r in range(world) for a, n in D.rank_wave_ranges(r, world, spp, "weak")
                          for w in range(a, a + n))
            assert weak == list(range(1, world * spp + 1))
    assert D.rank_job_ranges(1, 2, 4, 100, "weak") == [(400, 400)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, spp, out_path):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests")]
    import torch
    import torch.distributed as dist
    import oracle_lib as O
    from volume_path_tracer_amd import distributed as D
    from volume_path_tracer_amd.scenes import SynthGrid, workload

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wl = workload("c3", width=40, height=24, spp=spp, grid_n=64)
    dens = SynthGrid(1, 64).grid()
    od = O.OracleGrid(dens)
    T = wl.cfg.jobs_per_wave()
    film = np.zeros((wl.cfg.height, wl.cfg.width, 4), np.float32)
    for b, n in D.rank_job_ranges(rank, world, spp, T, mode):
        f, _, _ = O.render_jobs(wl.cfg, od, None, b, n)
        film += f
    t = torch.from_numpy(film)
    D.reduce_film(t)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["weak", "strong"])
def test_gloo_world2_matches_single(mode, tmp_path):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    import oracle_lib as O
    from volume_path_tracer_amd.scenes import SynthGrid, workload

    spp, world = 4, 2
    out = tmp_path / "film.npy"
    mp.start_processes(_worker, args=(world, _free_port(), mode, spp, str(out)), nprocs=world, start_method="spawn")
    got = np.load(out)
    wl = workload("c3", width=40, height=24, spp=spp, grid_n=64)
    od = O.OracleGrid(SynthGrid(1, 64).grid())
    total = D.total_samples_per_pixel(world, spp, mode)
    ref, _, _ = O.render_jobs(wl.cfg, od, None, 0, wl.cfg.jobs_per_wave() * total)
    np.testing.assert_array_equal(got[..., 3], float(total))
    np.testing.assert_allclose(got[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)
