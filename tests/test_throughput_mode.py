"""Throughput mode: one RNG stream per pixel, hash(seed, jid * tile_area + pixel).
It is not the reference's sample sequence: it must agree with it in expectation only, and the GPU
must reproduce the oracle's restatement of the mode bit for bit."""
import numpy as np
import pytest

import oracle_lib as O
from volume_path_tracer_amd import capi
from volume_path_tracer_amd.scenes import SynthGrid, workload


def _setup(name="c3", w=32, h=24, spp=16, n=64):
    wl = workload(name, width=w, height=h, spp=spp, grid_n=n)
    dens = SynthGrid(wl.density_kind, wl.grid_n).grid()
    return wl, dens, O.OracleGrid(dens, fix_majorants=True)


def test_pixel_mode_matches_reference_in_expectation():
    wl, dens, od = _setup()
    jobs = wl.cfg.jobs_per_wave() * wl.spp
    f_ref, _ = O.render_jobs_mode(wl.cfg, od, None, 0, jobs, capi.VPT_RNG_REFERENCE, records=False)
    f_pix, r_pix = O.render_jobs_mode(wl.cfg, od, None, 0, jobs, capi.VPT_RNG_PIXEL, records=True)
    assert (f_ref[..., 3] == f_pix[..., 3]).all()
    m_ref, m_pix = f_ref[..., :3].sum((0, 1)), f_pix[..., :3].sum((0, 1))
    # the per-sample radiance spread gives the standard error of the image mean
    r = r_pix[~np.isnan(r_pix[:, 0])]
    se = r.std(axis=0) * np.sqrt(len(r)) * wl.cfg.camera_parameters.imaging_ratio
    assert (np.abs(m_ref - m_pix) < 5 * se * np.sqrt(2)).all(), (m_ref, m_pix, se)
    # and it is a different sample sequence
    assert not np.array_equal(f_ref, f_pix)


def test_device_state_machine_pixel_mode_on_host():
    """The kernel's state machine (hostsim) in throughput mode: same samples, film and counts."""
    import hostsim_lib as HS

    wl = workload("c4", width=37, height=29, spp=2, grid_n=64)
    dens, temp = SynthGrid(1, 64).grid(), SynthGrid(2, 64).grid()
    od, ot = O.OracleGrid(dens, fix_majorants=True), O.OracleGrid(temp, fix_majorants=False)
    jobs = wl.cfg.jobs_per_wave() * 2
    f_o, r_o = O.render_jobs_mode(wl.cfg, od, ot, 0, jobs, capi.VPT_RNG_PIXEL)
    f_h, r_h, c_h = HS.render_jobs(wl.cfg, dens, temp, 0, jobs, records=True, rng_mode=capi.VPT_RNG_PIXEL)
    assert r_h.tobytes() == r_o.tobytes()
    assert c_h["samples"] == 37 * 29 * 2
    np.testing.assert_array_equal(f_h[..., 3], f_o[..., 3])
    np.testing.assert_allclose(f_h[..., :3], f_o[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("chunk", [2, 16, 64])
def test_pixel_chunks_keep_every_pixels_stream_on_host(chunk):
    """Work items of `chunk` pixels (vpt_gpu_set_pixel_chunk) trace the same samples as one pixel per item:
    each pixel seeds its own stream when it starts; clipped tiles end their chunks early."""
    import ctypes as C

    import hostsim_lib as HS

    wl = workload("c3", width=37, height=29, spp=2, grid_n=64)
    dens = SynthGrid(wl.density_kind, wl.grid_n).grid()
    jobs = wl.cfg.jobs_per_wave() * 2
    _, r_1, c_1 = HS.render_jobs(wl.cfg, dens, None, 0, jobs, records=True, rng_mode=capi.VPT_RNG_PIXEL)
    L = HS.lib()
    L.vpths_set_pixel_chunk.argtypes = [C.c_int]
    L.vpths_set_pixel_chunk(chunk)
    try:
        _, r_k, c_k = HS.render_jobs(wl.cfg, dens, None, 0, jobs, records=True, rng_mode=capi.VPT_RNG_PIXEL)
    finally:
        L.vpths_set_pixel_chunk(1)
    assert r_k.tobytes() == r_1.tobytes()
    assert c_k == c_1


@pytest.mark.gpu
@pytest.mark.parametrize("name,n,chunk", [("c3", 64, 0), ("c4", 64, 0), ("c3", 64, 8), ("c4", 64, 64)])
def test_gpu_pixel_mode_bit_exact(name, n, chunk):
    import torch

    from volume_path_tracer_amd.render import Integrator

    wl = workload(name, width=37, height=29, spp=2, grid_n=n)
    dens = SynthGrid(wl.density_kind, wl.grid_n).grid()
    temp = SynthGrid(2, wl.grid_n).grid() if wl.temperature else None
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.set_rng_mode(capi.VPT_RNG_PIXEL)
    it.set_pixel_chunk(chunk)
    jobs = wl.cfg.jobs_per_wave() * 2
    area = int(wl.cfg.tile_size[0] * wl.cfg.tile_size[1])
    rec = torch.full((jobs * area, 3), float("nan"), dtype=torch.float32, device=it.dev)
    film = torch.zeros_like(it.film)
    it.render_jobs(0, jobs, film=film, records=rec)
    torch.cuda.synchronize()
    od = O.OracleGrid(dens, fix_majorants=True)
    ot = O.OracleGrid(temp, fix_majorants=False) if temp is not None else None
    f_o, r_o = O.render_jobs_mode(wl.cfg, od, ot, 0, jobs, capi.VPT_RNG_PIXEL)
    r_g = rec.cpu().numpy()
    assert it.counters()["samples"] == 37 * 29 * 2
    assert r_g.tobytes() == r_o.tobytes()
    np.testing.assert_array_equal(film.cpu().numpy()[..., 3], f_o[..., 3])
    # and back to the reference streams
    it.set_rng_mode(capi.VPT_RNG_REFERENCE)
    f_ref, r_ref, _ = O.render_jobs(wl.cfg, od, ot, 0, jobs, records=True)
    rec.fill_(float("nan"))
    it.render_jobs(0, jobs, film=torch.zeros_like(it.film), records=rec)
    torch.cuda.synchronize()
    assert rec.cpu().numpy().tobytes() == r_ref.tobytes()
