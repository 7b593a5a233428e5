"""Job order never changes samples (every job keeps its jid and RNG stream): films rendered under the
built-in cost order, caller-supplied tile costs (vpt_gpu_set_tile_costs) and an explicit job
permutation (vpt_gpu_set_job_permutation) agree to fp32 atomic-order rounding, with exact sample
counts (added per launch by the count kernel), and equal the oracle's film."""
import numpy as np
import pytest

import oracle_lib as O
from volume_path_tracer_amd import capi
from volume_path_tracer_amd.render import Integrator
from volume_path_tracer_amd.scenes import SynthGrid, workload

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

WAVES = 3


@pytest.fixture(scope="module")
def setup():
    wl = workload("c3", width=96, height=64, spp=WAVES, grid_n=64)
    dens = SynthGrid(wl.density_kind, wl.grid_n).grid()
    it = Integrator(wl.cfg, dens, None, device=0)
    od = O.OracleGrid(dens, fix_majorants=True)
    film_o, _, _ = O.render_jobs(wl.cfg, od, None, 0, it.jobs_per_wave * WAVES)
    return wl, it, film_o


def _frame(it):
    it.film.zero_()
    it.render_waves(1, WAVES)
    return it.film_host().copy()


def _check(f, film_o):
    np.testing.assert_array_equal(f[..., 3], WAVES)
    np.testing.assert_allclose(f[..., :3], film_o[..., :3], rtol=1e-5, atol=1e-6)


def test_orders_render_the_same_film(setup):
    wl, it, film_o = setup
    T = it.jobs_per_wave
    base = _frame(it)
    _check(base, film_o)
    for mode in (capi.VPT_ORDER_JID, capi.VPT_ORDER_COST_WAVE_MAJOR, capi.VPT_ORDER_COST_TILE_MAJOR,
                 capi.VPT_ORDER_COST_TAIL, capi.VPT_ORDER_COST_SAME_TILE):
        it.set_job_order(mode)
        _check(_frame(it), film_o)
    # caller-supplied costs: the reverse of the estimates
    est, _ = it.tile_costs()
    it.set_tile_costs(-est)
    _check(_frame(it), film_o)
    # an explicit permutation of the frame's jobs
    perm = np.random.default_rng(7).permutation(T * WAVES).astype(np.uint32)
    it.set_job_permutation(perm)
    _check(_frame(it), film_o)
    it.set_job_permutation(None)
    _check(_frame(it), film_o)


def test_job_permutation_rejects_non_permutations(setup):
    _, it, _ = setup
    with pytest.raises(RuntimeError):
        it.set_job_permutation(np.array([0, 0, 1], np.uint32))
    with pytest.raises(RuntimeError):
        it.set_job_permutation(np.array([0, 3, 1], np.uint32))


def test_tile_costs_reject_non_finite(setup):
    """NaN / inf costs would make the ranking's comparator no strict weak ordering."""
    _, it, _ = setup
    est, rank = it.tile_costs()
    for bad in (np.nan, np.inf):
        c = est.copy()
        c[len(c) // 2] = bad
        with pytest.raises(RuntimeError):
            it.set_tile_costs(c)
    np.testing.assert_array_equal(it.tile_costs()[1], rank)  # the ranking is unchanged


def test_sample_counts_for_partial_job_ranges(setup):
    """The count kernel's per-pixel job count for ranges that start and end inside waves."""
    wl, it, _ = setup
    T = it.jobs_per_wave
    W, H = wl.cfg.width, wl.cfg.height
    tw, th = int(wl.cfg.tile_size[0]), int(wl.cfg.tile_size[1])
    ntx = -(-W // tw)
    for b, n in ((5, 7), (T - 3, T + 9), (2 * T + 1, 1), (0, 2 * T + 5)):
        it.film.zero_()
        it.render_jobs(b, n)
        f = it.film_host()
        want = np.zeros((H, W), np.float32)
        for jid in range(b, b + n):
            t = jid % T
            x0, y0 = (t % ntx) * tw, (t // ntx) * th
            want[y0:y0 + th, x0:x0 + tw] += 1
        np.testing.assert_array_equal(f[..., 3], want)
