"""Oracle-independent anchors for the sparse NanoVDB levels and the camera.

1. Camera: the reference's raster -> world direction (src/camera.cpp:45-57, include/vpt/camera.hpp:14-23)
   recomputed in float64 (tests/analytic_anchor.py, no oracle matrix): the oracle's and the GPU's fp32
   camera rays (the Logger's new_ray events, worker.cpp:124-125) agree within a few ulp, without
   jitter on every pixel and with jitter on each job's first pixel (its jitter = the first two draws
   of pcg32_fast seeded with hash(seed, jid), recomputed in Python and checked against the SURVEY KATs).
2. Transport through every tree level: an absorption-only scene (sigma_s = 0, distant light off, no
   jitter) over the anchor grid -- leaves, active AND inactive lower-node tiles, empty upper-node slots
   (HDDA dim 128), an active upper-node tile, empty root space (dim 4096) and an active root tile --
   whose per-pixel survival probability exp(-sigma_a * integral of rho [m > 0]) is integrated exactly in
   float64 from the grid description (analytic_anchor.optical_depth).  Bar as in test_analytic.py:
   each pixel's surviving count inside its exact binomial tails (Bonferroni), and the mean z-score
   within 4 / sqrt(pixels).  A wrong tile value, a level's majorant (volume.cpp:18-36), the inactive
   tiles' zero majorant, the clip to indexBBox, or the camera shifts it.
"""
import numpy as np
import pytest

import analytic_anchor as A
import oracle_lib as O
from volume_path_tracer_amd.scenes import SynthGrid, workload

SIGMA_A = 0.01
ULP = 2.0 ** -24


# ---- RNG and camera -------------------------------------------------------------------------------
def test_python_rng_matches_survey_kats():
    kat = {(10, 0): (0x2B3709D35ACDD2E9, [1846738701, 1516240651, 2895873600, 2052828018]),
           (10, 32400): (0x049AE8A3554EDD3B, [1805829371, 4083204118, 3994801159, 3711332802]),
           (500, 32399): (0x0BAD42B31B1A3CED, [3037361848, 1263350600, 2513201965, 2450829360])}
    for (seed, jid), (h, u) in kat.items():
        assert A.murmur_seed(seed, jid) == h
        g = A.Pcg32Fast(h)
        assert [g.u32() for _ in range(4)] == u
    g = A.Pcg32Fast(A.murmur_seed(10, 1))
    assert [float(g.uniform()) for _ in range(2)] == [np.float32(0.0850023404), np.float32(0.876347423)]


def camera_config(jitter: bool):
    """A non-square frame and a camera pose with a non-unit, non-orthogonal up vector."""
    wl = workload("c3", width=40, height=24, spp=1, grid_n=64)
    cp = wl.cfg.camera_parameters
    cp.position[:] = [3.5, -2.25, -310.0]
    cp.look[:] = [10.0, 5.0, 4.0]
    cp.up[:] = [0.1, 2.0, 0.2]
    cp.vfov_deg = 37.5
    wl.cfg.worker_parameters.use_jitter = 1 if jitter else 0
    return wl


def new_ray_directions(events, cfg, jitter: bool):
    """(measured fp32 directions, float64 expectations) of the new_ray events: every pixel without
    jitter; each job's first pixel with jitter (its first two draws, worker.cpp:121-122)."""
    T = cfg.jobs_per_wave()
    tw, th = int(cfg.tile_size[0]), int(cfg.tile_size[1])
    ntx = -(-cfg.width // tw)
    ev = events[events["type"] == 0]
    got, px, py = [], [], []
    for e in ev:
        tile = int(e["jid"]) % T
        x0, y0 = (tile % ntx) * tw, (tile // ntx) * th
        rw = min(cfg.width - x0, tw)
        pix = int(e["pixel"])
        jx = jy = np.float32(0)
        if jitter:
            if pix != 0:
                continue
            g = A.Pcg32Fast(A.murmur_seed(cfg.seed, int(e["jid"])))
            jx, jy = g.uniform() * np.float32(0.5), g.uniform() * np.float32(0.5)
        # raster point in float32, as generate_ray forms it (pt + 0.5 + jitter)
        px.append(np.float32(np.float32(x0 + pix % rw) + np.float32(0.5)) + jx)
        py.append(np.float32(np.float32(y0 + pix // rw) + np.float32(0.5)) + jy)
        got.append(e["v"][3:6])
    return np.array(got, np.float64), A.camera_dirs(cfg, np.array(px), np.array(py))


def check_camera(events, cfg, jitter):
    got, want = new_ray_directions(events, cfg, jitter)
    assert len(got) == (cfg.jobs_per_wave() if jitter else cfg.width * cfg.height)
    err = np.abs(got - want).max()
    # fp32 products and one normalisation: a few ulp of a unit vector; a wrong composition order,
    # aspect ratio, half-pixel offset or jitter scale is >= 1e-4
    assert err < 8 * ULP, err / ULP
    return err


@pytest.mark.parametrize("jitter", [False, True])
def test_oracle_camera_rays_match_float64_camera(jitter):
    wl = camera_config(jitter)
    od = O.OracleGrid(SynthGrid(1, 64).grid(), fix_majorants=True)
    ev, _ = O.render_jobs_events(wl.cfg, od, None, 0, wl.cfg.jobs_per_wave())
    check_camera(ev, wl.cfg, jitter)


@pytest.mark.gpu
@pytest.mark.parametrize("jitter", [False, True])
def test_gpu_camera_rays_match_float64_camera(jitter):
    from volume_path_tracer_amd.render import Integrator

    wl = camera_config(jitter)
    it = Integrator(wl.cfg, SynthGrid(1, 64).grid(), None, device=0)
    ev = it.trace_jobs(0, wl.cfg.jobs_per_wave())
    check_camera(ev, wl.cfg, jitter)


# ---- transport through every tree level -----------------------------------------------------------
def sparse_config(w, h, spp):
    wl = workload("c3", width=w, height=h, spp=spp, grid_n=64)
    cfg = wl.cfg
    cp = cfg.camera_parameters
    cp.position[:] = [0.0, 0.0, -50000.0]  # world; index = world - MAP_VEC
    cp.look[:] = [0.0, 0.0, 0.0]
    cp.up[:] = [0.0, 1.0, 0.0]
    cp.vfov_deg = float(2.0 * np.degrees(np.arctan(72.0 / 50000.0)))  # the L0 column plus a margin
    v = cfg.volume_parameters
    v.sigma_s, v.sigma_a = 0.0, SIGMA_A
    wp = cfg.worker_parameters
    wp.distant_light_multiplier = 0.0  # Li == 0: no NEE (worker.cpp:57-58)
    wp.use_jitter = 0                  # one ray per pixel: the expectation needs no jitter integral
    return wl


def expected_survival(cfg, eps=1e-3):
    """Per pixel exp(-tau) along its float64 camera ray, and the largest change under +-eps pixel
    offsets (pixels whose ray grazes a majorant discontinuity are excluded by the caller)."""
    W, H = cfg.width, cfg.height
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float64)
    o = np.array(cfg.camera_parameters.position[:], np.float64) - np.array(A.MAP_VEC)
    out = []
    for dx, dy in ((0, 0), (eps, 0), (-eps, 0), (0, eps), (0, -eps)):
        d = A.camera_dirs(cfg, (xs + 0.5 + dx).reshape(-1), (ys + 0.5 + dy).reshape(-1))
        out.append(np.exp(-SIGMA_A * A.optical_depth(o, d)).reshape(H, W))
    t = out[0]
    return t, np.max([np.abs(x - t) for x in out[1:]], axis=0)


def check_sparse_film(cfg, film, spp):
    from scipy.stats import binom

    le = np.asarray(cfg.worker_parameters.infinite_light_xyz, np.float64) * cfg.worker_parameters.infinite_light_multiplier
    r = cfg.camera_parameters.imaging_ratio
    np.testing.assert_array_equal(film[..., 3], spp)
    est = film[..., 1].astype(np.float64) / film[..., 3] / (r * le[1])
    t, spread = expected_survival(cfg)
    miss = t == 1.0  # rays that pass beside the index bbox
    np.testing.assert_allclose(est[miss], 1.0, rtol=2e-5)
    use = (spread < 1e-3) & ~miss
    assert use.sum() >= 0.7 * use.size, use.sum()
    assert t[use].min() < 0.5 and (t[use] < 0.8).mean() > 0.5, (t[use].min(), t[use].max())  # every level weighs in
    k = np.rint(est[use] * spp)
    assert np.abs(est[use] * spp - k).max() < 0.05
    ti = t[use]
    p_two = 2 * np.minimum(binom.cdf(k, spp, ti), binom.sf(k - 1, spp, ti))
    assert p_two.min() > 1e-3 / use.sum(), (p_two.min(), int(k[p_two.argmin()]), ti[p_two.argmin()])
    z = (est[use] - ti) / np.sqrt(ti * (1 - ti) / spp)
    assert abs(z.mean()) < 4.0 / np.sqrt(z.size), (z.mean(), z.size)
    return z


def test_anchor_integral_self_check():
    """The exact piecewise integral against brute-force midpoint sums on a few rays (every region)."""
    rng = np.random.default_rng(1)
    o = np.array([64.0, 64.0, -50000.0])
    d = np.stack([rng.uniform(-0.0012, 0.0014, 6), rng.uniform(-0.0012, 0.0014, 6), np.ones(6)], 1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tau = A.optical_depth(o, d)
    zs = np.concatenate([np.linspace(0, 130, 260001), np.linspace(130, A.Z_END, 1000001)[1:]])
    for r in range(6):
        ts = (zs - o[2]) / d[r, 2]
        mid, dt = 0.5 * (ts[1:] + ts[:-1]), np.diff(ts)
        p = o + mid[:, None] * d[r]
        f = A.trilinear(p) * A.majorant_positive(*(np.floor(p[:, q]).astype(np.int64) for q in range(3)))
        assert abs((f * dt).sum() - tau[r]) < 3e-4 * tau[r], (r, (f * dt).sum(), tau[r])


def test_anchor_grid_levels():
    """The anchor grid answers getValue / getDim / majorant per level as analytic_anchor models it
    (through the product's flattened tables, host side)."""
    import hostsim_lib as HS

    g = A.anchor_grid()
    pts = np.array([[3, 5, 7], [64, 64, 70], [72, 64, 70], [5, 5, 125], [5, 5, 200], [5, 5, 4000],
                    [200, 5, 4000], [5, 5, 5000], [5, 5, 9000], [1000, 2000, 12000]], np.int32)
    val, dim, maj = HS.probe(g, pts)
    np.testing.assert_array_equal(val, A.voxel_value(*pts.T).astype(np.float32))
    np.testing.assert_array_equal(dim, [8, 8, 8, 8, 128, 128, 128, 4096, 4096, 4096])
    np.testing.assert_array_equal(maj > 0, A.majorant_positive(*pts.T))


def test_oracle_sparse_levels_absorption_matches_analytic():
    """The CPU oracle against the float64 expectation: 24x24 pixels, 512 spp."""
    wl = sparse_config(24, 24, 512)
    od = O.OracleGrid(A.anchor_grid(), fix_majorants=True)
    film, _, c = O.render_jobs(wl.cfg, od, None, 0, wl.cfg.jobs_per_wave() * 512)
    check_sparse_film(wl.cfg, film, 512)


@pytest.mark.gpu
@pytest.mark.parametrize("runs", [0, 1])
def test_gpu_sparse_levels_absorption_matches_analytic(runs):
    """The production HIP kernel (plain and run-skipping variants) against the float64 expectation:
    96x96 pixels at 1024 spp."""
    from volume_path_tracer_amd.render import Integrator

    wl = sparse_config(96, 96, 1024)
    it = Integrator(wl.cfg, A.anchor_grid(), None, device=0)
    it.set_run_skipping(runs)
    it.render_waves(1, 1024)
    check_sparse_film(wl.cfg, it.film_host(), 1024)
