"""Analytic anchor for the SCATTERING half of the transport, independent of the oracle.

The absorption anchors (test_analytic.py, test_analytic_sparse.py) run with sigma_s = 0 and the
distant light off, so the reference's scattering quirks were checked only against the oracle, which
restates the same reading of worker.cpp.  Two expectations computed here from first principles pin them:

1. **Single scatter with NEE** on C2's constant cube: sigma_a = 0, sigma_s = 0.01, g = 0.4,
   the distant light on, `max_depth = 2`, no jitter.  The depth counter is incremented twice per scatter
   (worker.cpp:130 and :169), so a path scatters at most once: the scatter's `depth++` takes depth to 1,
   the `for` increment to 2 and the loop ends -- with `terminated` false, so the environment light is
   added (worker.cpp:198-200) on that depth-bound exit as on an escape.  With sigma_a = 0 no path is
   absorbed, so every sample is

       L = Le_inf + [first real collision at x] * Li * HG_ref(w . wi, g) * T_shadow(x)

   and  E[L] = Le_inf + Li * HG_ref(w . wi, g) * I,  I = the chord integral of
   sigma_s rho(t) exp(-sigma_s tau(t0, t)) exp(-sigma_s tau_shadow(x(t))) (analytic_anchor.single_scatter).
   Delta tracking's first real collision has density sigma_s rho exp(-sigma_s tau); ratio tracking with
   Russian roulette (worker.cpp:68-85) is unbiased for exp(-sigma_s tau_shadow); HG_ref is the reference's
   NEE phase, den = 1 + g^2 + 2 g (w . wi) with the FORWARD ray direction w (utils.hpp:61-66,
   worker.cpp:88).  The light direction is chosen so w . wi ~ -0.8: the mirrored and pbrt signs then differ
   9x.
2. **HG sampling distribution** from the Logger event log (worker.cpp:16-48): for every scatter, cos of the
   angle between the incoming and the sampled direction follows the forward-peaked HG law of
   sample_henyey_greenstein (random.hpp:56-84, local z = w, no minus sign: mean cos = +g), and the azimuth
   about w is uniform.

Bars: per pixel, the t statistic of the mean over K independent batches (jobs of distinct waves) inside
its two-sided t-distribution tail (p > 1e-3 / pixels); the pooled z-score of all pixels' deviations within
4; Kolmogorov-Smirnov p > 1e-3 for the sampling laws.  `test_anchor_rejects_mutants` shows the bar has the
power to see the quirks: the oracle rebuilt with each mutation (oracle/vpt_oracle.cpp VPTO_MUTANT: the NEE
phase with pbrt's sign, the sampling sign flipped, one depth increment per scatter, the environment light
only on escape) fails it.
"""
from __future__ import annotations

import numpy as np
import pytest

import analytic_anchor as A
import oracle_lib as O
from volume_path_tracer_amd.scenes import SynthGrid, workload

SIGMA_S = 0.01
G = 0.4
WI = (0.3, 0.5, -0.8)          # distant light inv_direction (toward the light): w . wi ~ -0.8
INDEX_OF_WORLD = 64.0          # the cube's map: world = index - 64


def scatter_config(w, h, spp):
    wl = workload("c2", width=w, height=h, spp=spp)
    v = wl.cfg.volume_parameters
    v.sigma_s, v.sigma_a, v.henyey_greenstein_g = SIGMA_S, 0.0, G
    p = wl.cfg.worker_parameters
    p.max_depth = 2
    p.use_jitter = 0
    p.distant_light_inv_direction[:] = WI
    return wl


_EXPECTED: dict = {}


def expected_nee(cfg):
    """Per pixel [H, W]: (HG_ref(w . wi) * I, tau) in float64; the camera rays through pixel centres
    (jitter drawn but scaled by 0, worker.cpp:121-122) from the float64 camera of analytic_anchor."""
    W, H = cfg.width, cfg.height
    key = (W, H, tuple(cfg.camera_parameters.position[:]), tuple(cfg.worker_parameters.distant_light_inv_direction[:]),
           cfg.volume_parameters.henyey_greenstein_g, cfg.volume_parameters.sigma_s)
    if key not in _EXPECTED:
        _EXPECTED[key] = _expected_nee(cfg)
    return _EXPECTED[key]


def _expected_nee(cfg):
    W, H = cfg.width, cfg.height
    ys, xs = np.mgrid[0:H, 0:W]
    d = A.camera_dirs(cfg, xs.ravel() + 0.5, ys.ravel() + 0.5)
    o = np.asarray(cfg.camera_parameters.position[:], np.float64) + INDEX_OF_WORLD
    wi = np.asarray(cfg.worker_parameters.distant_light_inv_direction[:], np.float64)
    wi /= np.linalg.norm(wi)
    g = float(cfg.volume_parameters.henyey_greenstein_g)
    s = float(cfg.volume_parameters.sigma_s)
    I, tau = np.zeros(d.shape[0]), np.zeros(d.shape[0])
    for c in range(0, d.shape[0], 128):
        I[c:c + 128], tau[c:c + 128] = A.single_scatter(o, d[c:c + 128], wi, s)
    hg = A.hg_reference(d @ wi, g)
    return (hg * I).reshape(H, W), tau.reshape(H, W)


def scatter_report(cfg, films):
    """films: [K, H, W, 4] from K batches of equal spp.  Returns a dict with `ok` and the statistics."""
    from scipy.stats import t as student_t

    K = films.shape[0]
    spp_b = films[0, 0, 0, 3]
    assert (films[..., 3] == spp_b).all()
    wp = cfg.worker_parameters
    le = np.asarray(wp.infinite_light_xyz[:], np.float64) * wp.infinite_light_multiplier
    li = np.asarray(wp.distant_light_xyz[:], np.float64) * wp.distant_light_multiplier
    r = cfg.camera_parameters.imaging_ratio
    est = films[..., :3].astype(np.float64) / spp_b / r                      # [K, H, W, 3] batch means of L
    nee, tau = expected_nee(cfg)
    rep = {"K": K, "spp": int(spp_b) * K}
    # Every sample is Le + c * Li (c >= 0): the channels of the NEE part stay in Li's ratios.
    m = est.mean(axis=0)
    rep["channel_dev"] = float(np.abs((m[..., 0] - le[0]) * li[1] - (m[..., 1] - le[1]) * li[0]).max())
    ok_channels = rep["channel_dev"] < 1e-4 * li[0] * (1.0 + m[..., 1].max())
    miss = tau == 0.0
    ok_miss = bool(np.allclose(m[miss][..., 1], le[1], rtol=2e-5)) if miss.any() else True
    sel = (1.0 - np.exp(-SIGMA_S * tau)) >= 0.1                              # enough scatters per batch
    y = est[..., 1]
    mean = y.mean(axis=0)[sel]
    se = y.std(axis=0, ddof=1)[sel] / np.sqrt(K)
    expect = le[1] + li[1] * nee[sel]
    assert (se > 0).all()
    tstat = (mean - expect) / se
    p = 2.0 * student_t.sf(np.abs(tstat), K - 1)
    z = float((mean - expect).sum() / np.sqrt((se ** 2).sum()))
    rep.update(pixels=int(sel.sum()), p_min=float(p.min()), z=z, rel_dev=float((mean - expect).sum() / expect.sum()),
               miss_pixels=int(miss.sum()), ok_channels=bool(ok_channels), ok_miss=ok_miss)
    rep["ok"] = bool(ok_channels and ok_miss and p.min() > 1e-3 / sel.sum() and abs(z) < 4.0)
    return rep


def scatter_pairs(ev):
    """(incoming, outgoing) directions of every scatter in an event log sorted by (jid, seq): the
    incoming one is the direction of the same pixel's previous new_ray / scatter event."""
    from volume_path_tracer_amd.capi import EVENT_NAMES

    nr, sc = EVENT_NAMES.index("new_ray"), EVENT_NAMES.index("scatter")
    rays = ev[(ev["type"] == nr) | (ev["type"] == sc)]
    prev, cur = rays[:-1], rays[1:]
    m = (cur["type"] == sc) & (cur["jid"] == prev["jid"]) & (cur["pixel"] == prev["pixel"])
    return prev["v"][m, 3:6].astype(np.float64), cur["v"][m, 3:6].astype(np.float64)


def sampling_report(ev, g):
    from scipy.stats import kstest

    w, o = scatter_pairs(ev)
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    o /= np.linalg.norm(o, axis=1, keepdims=True)
    mu = (w * o).sum(axis=1)
    # azimuth about w in any right-handed frame (a uniform law stays uniform under a rotation)
    a = np.where(np.abs(w[:, :1]) < 0.9, [[1.0, 0.0, 0.0]], [[0.0, 1.0, 0.0]])
    e1 = np.cross(w, a)
    e1 /= np.linalg.norm(e1, axis=1, keepdims=True)
    e2 = np.cross(w, e1)
    phi = np.arctan2((o * e2).sum(axis=1), (o * e1).sum(axis=1))
    p_mu = kstest(np.clip(mu, -1.0, 1.0), lambda x: A.hg_cos_cdf(x, g)).pvalue
    p_phi = kstest(phi, "uniform", args=(-np.pi, 2.0 * np.pi)).pvalue
    return {"scatters": int(mu.size), "mean_cos": float(mu.mean()), "p_cos": float(p_mu), "p_phi": float(p_phi),
            "ok": bool(mu.size >= 5000 and p_mu > 1e-3 and p_phi > 1e-3)}


def sampling_config(w=16, h=16, spp=4):
    """C2's cube as BASELINE runs it (sigma_s 0.15, g 0.4, max_depth 100): tens of scatters per path."""
    wl = workload("c2", width=w, height=h, spp=spp)
    return wl


# ---- expectation self-checks ---------------------------------------------------------------------------
def test_cube_optical_depth_matches_brute_force():
    rng = np.random.default_rng(1)
    o = rng.uniform(-20, 150, size=(8, 3))
    d = rng.normal(size=(8, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tau = A.cube_od(o, d, np.zeros(8), np.full(8, np.inf))
    t = np.linspace(0, 400, 800001)[:-1] + 0.00025
    for i in range(8):
        p = o[i] + t[:, None] * d[i]
        inb = np.all((p >= 0) & (p <= 128), axis=1)
        assert abs((A.cube_density(p) * inb).sum() * 0.0005 - tau[i]) < 1e-3  # the entry face is a step


def test_single_scatter_integral_matches_brute_force():
    """The composite quadrature of single_scatter against a fine midpoint rule on a few rays."""
    o = np.array([64.0, 64.0, -236.0])
    d = np.array([[0.0, 0.0, 1.0], [0.21, -0.13, 1.0], [-0.26, 0.25, 1.0]])
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    wi = np.asarray(WI) / np.linalg.norm(WI)
    I, _ = A.single_scatter(o, d, wi, SIGMA_S)
    for i in range(3):
        t0, t1 = A.cube_chord(o[None], d[i:i + 1])
        n = 20000
        t = t0[0] + (np.arange(n) + 0.5) * (t1[0] - t0[0]) / n
        x = o + t[:, None] * d[i]
        tc = A.cube_od(np.broadcast_to(o, (n, 3)), np.broadcast_to(d[i], (n, 3)), np.full(n, t0[0]), t)
        ts = A.cube_od(x, np.broadcast_to(wi, (n, 3)), np.full(n, 1e-5), np.full(n, np.inf))
        ref = (SIGMA_S * A.cube_density(x) * np.exp(-SIGMA_S * (tc + ts))).sum() * (t1[0] - t0[0]) / n
        assert abs(I[i] - ref) < 1e-6 * max(1.0, ref), (i, I[i], ref)


def test_hg_cdf_is_the_sampler_law():
    """hg_cos_cdf inverts the reference's cos(theta) formula: F(cos(u)) = 1 - u."""
    u = np.linspace(0.0, 1.0, 101)
    cos = (1 + G * G - ((1 - G * G) / (1 + G - 2 * G * u)) ** 2) / (2 * G)
    np.testing.assert_allclose(A.hg_cos_cdf(cos, G), 1.0 - u, atol=1e-12)


# ---- the oracle --------------------------------------------------------------------------------------
ORACLE_SHAPE = (24, 24, 16, 32)      # width, height, batches K, spp per batch


def oracle_batches(mutant=0):
    w, h, K, spp_b = ORACLE_SHAPE
    wl = scatter_config(w, h, K * spp_b)
    od = O.OracleGrid(SynthGrid(0, 128).grid(), fix_majorants=True, L=O.lib(mutant))
    T = wl.cfg.jobs_per_wave()
    films = np.stack([O.render_jobs(wl.cfg, od, None, k * spp_b * T, spp_b * T)[0] for k in range(K)])
    return wl.cfg, films


def oracle_events(mutant=0):
    wl = sampling_config()
    od = O.OracleGrid(SynthGrid(0, 128).grid(), fix_majorants=True, L=O.lib(mutant))
    ev, _ = O.render_jobs_events(wl.cfg, od, None, 0, wl.cfg.jobs_per_wave() * wl.spp, capacity=1 << 21)
    return ev


def test_oracle_single_scatter_matches_analytic():
    cfg, films = oracle_batches()
    rep = scatter_report(cfg, films)
    assert rep["ok"], rep
    assert rep["pixels"] >= 300


def test_oracle_hg_sampling_law():
    rep = sampling_report(oracle_events(), G)
    assert rep["ok"], rep
    assert abs(rep["mean_cos"] - G) < 0.02


@pytest.mark.parametrize("mutant,kind", [(1, "nee"), (2, "sampling"), (3, "nee"), (4, "nee")])
def test_anchor_rejects_mutants(mutant, kind):
    """Each mutation of the oracle fails the anchor that targets it (the bar has the power)."""
    if kind == "nee":
        cfg, films = oracle_batches(mutant)
        rep = scatter_report(cfg, films)
    else:
        rep = sampling_report(oracle_events(mutant), G)
    assert not rep["ok"], rep


# ---- the production HIP kernels ----------------------------------------------------------------------
GPU_SHAPE = (64, 64, 16, 64)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["plain", "runs", "temperature"])
def test_gpu_single_scatter_matches_analytic(variant):
    """Production kernels (density-only with and without run skipping, and the temperature kernel with a
    constant temperature grid: sigma_a = 0 makes its emission 0), 64x64 pixels, 16 batches of 64 waves."""
    import torch

    from volume_path_tracer_amd.render import Integrator

    w, h, K, spp_b = GPU_SHAPE
    wl = scatter_config(w, h, K * spp_b)
    temp = SynthGrid(0, 128).grid() if variant == "temperature" else None
    it = Integrator(wl.cfg, SynthGrid(0, 128).grid(), temp, device=0)
    if variant != "temperature":
        it.set_run_skipping(1 if variant == "runs" else 0)
    assert it.kernel_variant()["has_temperature"] == (variant == "temperature")
    films = torch.zeros((K, h, w, 4), dtype=torch.float32, device="cuda:0")
    for k in range(K):
        it.render_waves(1 + k * spp_b, spp_b, film=films[k])
    torch.cuda.synchronize()
    rep = scatter_report(wl.cfg, films.cpu().numpy())
    print(variant, rep)
    assert rep["ok"], rep
    assert rep["pixels"] >= 2000


@pytest.mark.gpu
def test_gpu_hg_sampling_law():
    """Scatter directions of the HIP integrator's event log (the Logger variant of the kernel, which runs
    the production kernel's device code with the event sink on)."""
    from volume_path_tracer_amd.render import Integrator

    wl = sampling_config(32, 32, 4)
    it = Integrator(wl.cfg, SynthGrid(0, 128).grid(), None, device=0)
    ev = it.trace_jobs(0, wl.cfg.jobs_per_wave() * wl.spp, capacity=1 << 23)
    rep = sampling_report(ev, G)
    print(rep)
    assert rep["ok"], rep
    assert rep["scatters"] >= 20000
    assert abs(rep["mean_cos"] - G) < 0.01
