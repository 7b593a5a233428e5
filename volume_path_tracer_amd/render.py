"""Host driver: the reference's work-distribution API over the HIP integrator.

``TileProvider`` restates include/vpt/tile_provider.hpp / src/tile_provider.cpp (job id -> (tile,
wave), wave bookkeeping, stop_at_next_wave, progress/ETA).  ``run`` is the drop-in for
``vpt::run`` (src/worker.cpp:92-208): instead of tracing one token at a time on a CPU thread, it
drains the provider in contiguous job-id batches and launches each batch on the GPU.  Job ids key
the RNG streams (hash(seed, jid)), so the batching does not change any sample.

Device memory (film, per-sample records) is plain torch CUDA tensors — torch is plumbing here; the
integrator itself is the HIP kernel in libvpt_amd.so.
"""
from __future__ import annotations

import ctypes as C
import threading
import time
from typing import Optional

import numpy as np

from . import capi


def ceildiv(a: int, b: int) -> int:
    return a // b + (a % b != 0)


class TileProvider:
    """tile_provider.cpp:14-111 — job index -> (tile, wave); waves start when first touched."""

    def __init__(self, img_size, waves: int, tile_size):
        self.img_w, self.img_h = int(img_size[0]), int(img_size[1])
        self.tile_w, self.tile_h = int(tile_size[0]), int(tile_size[1])
        self.ntx, self.nty = ceildiv(self.img_w, self.tile_w), ceildiv(self.img_h, self.tile_h)
        self.num_tiles = self.ntx * self.nty
        self.requested_waves = int(waves)
        self.max_wave_idx = 0
        self._job_idx = 0
        self._force_stop = False
        self._lock = threading.Lock()
        self._start = time.monotonic()

    # token next() without per-tile wave gating: on the GPU the film adds are atomics, so two
    # waves of a tile may be in flight together (the reference serialises them, tile_provider.cpp:40-60).
    def next_batch(self, max_jobs: int):
        """Reserve up to max_jobs consecutive job ids: (jid_begin, count), count 0 when done."""
        with self._lock:
            if self._force_stop:
                return self._job_idx, 0
            end = self.requested_waves * self.num_tiles
            begin = self._job_idx
            count = max(0, min(max_jobs, end - begin))
            self._job_idx += count
            if count:
                self.max_wave_idx = max(self.max_wave_idx, 1 + (begin + count - 1) // self.num_tiles)
            return begin, count

    def job(self, jid: int):
        """(tile, wave) of a job id (tile_provider.cpp:30-31)."""
        return jid % self.num_tiles, 1 + jid // self.num_tiles

    def compute_tile_rect(self, tile: int):
        """tile_provider.cpp:95-105 -> (x0, y0, w, h)."""
        x0 = (tile % self.ntx) * self.tile_w
        y0 = (tile // self.ntx) * self.tile_h
        return x0, y0, min(self.img_w - x0, self.tile_w), min(self.img_h - y0, self.tile_h)

    def stop_at_next_wave(self):
        """tile_provider.cpp:107-110: requested_waves = the highest wave already started."""
        with self._lock:
            self.requested_waves = self.max_wave_idx

    def stop_now(self):
        self._force_stop = True

    def reset_eta(self):
        self._start = time.monotonic()

    def progress_ratio(self) -> float:
        total = self.requested_waves * self.num_tiles
        return self._job_idx / total if total else 1.0

    def progress(self) -> int:
        return int(self.progress_ratio() * 100.0)

    def eta(self) -> float:
        p = self.progress_ratio()
        el = time.monotonic() - self._start
        return (1 - p) / (p / el) if p > 0 and el > 0 else float("inf")


class Integrator:
    """One HIP context on one device: the flattened grids, scene constants and a film."""

    def __init__(self, cfg: capi.Configuration, density, temperature=None, device: int = 0, blackbody=None):
        import torch

        self.torch = torch
        self.cfg = cfg.copy()
        self.device = int(device)
        self.dev = torch.device("cuda", self.device)
        L = capi.lib()
        h = C.c_void_p()
        dens_desc = density.desc if hasattr(density, "desc") else density
        temp_desc = None if temperature is None else (temperature.desc if hasattr(temperature, "desc") else temperature)
        bb = None
        if blackbody is not None:
            bb = np.ascontiguousarray(blackbody, np.float32)
        capi.check(L.vpt_gpu_create(C.byref(self.cfg), C.byref(dens_desc),
                                    C.byref(temp_desc) if temp_desc is not None else None,
                                    bb.ctypes.data_as(C.POINTER(C.c_float)) if bb is not None else None,
                                    self.device, C.byref(h)), "vpt_gpu_create")
        self._attach(h)

    def _attach(self, h) -> None:
        self.h = h
        jpw, tot = C.c_uint64(), C.c_uint64()
        capi.check(capi.lib().vpt_gpu_job_space(h, C.byref(jpw), C.byref(tot)), "vpt_gpu_job_space")
        self.jobs_per_wave, self.total_jobs = int(jpw.value), int(tot.value)
        self.film = self.torch.zeros((self.cfg.height, self.cfg.width, 4), dtype=self.torch.float32, device=self.dev)

    @classmethod
    def create_many(cls, cfg: capi.Configuration, density, temperature=None, devices=(0,)) -> list:
        """One Integrator per device with the grids flattened once (vpt_gpu_create_many, what the multi-GPU drop-in
        uses); devices may repeat (several contexts on one GPU)."""
        import torch

        L = capi.lib()
        dens_desc = density.desc if hasattr(density, "desc") else density
        temp_desc = None if temperature is None else (temperature.desc if hasattr(temperature, "desc") else temperature)
        n = len(devices)
        devs = (C.c_int * n)(*[int(d) for d in devices])
        hs = (C.c_void_p * n)()
        cfg_c = cfg.copy()
        capi.check(L.vpt_gpu_create_many(C.byref(cfg_c), C.byref(dens_desc),
                                         C.byref(temp_desc) if temp_desc is not None else None, None, devs, n, hs),
                   "vpt_gpu_create_many")
        out = []
        for d, h in zip(devices, hs):
            it = cls.__new__(cls)
            it.torch, it.cfg, it.device = torch, cfg.copy(), int(d)
            it.dev = torch.device("cuda", it.device)
            it._attach(C.c_void_p(h))
            out.append(it)
        return out

    def setup_timings(self) -> dict:
        """vpt_gpu_setup_timings (ms): flatten + majorant fix, upload, the rest, tile costs, device bind."""
        ms = (C.c_double * 5)()
        capi.check(capi.lib().vpt_gpu_setup_timings(self.h, ms, 5), "vpt_gpu_setup_timings")
        return dict(zip(("flatten_fix", "upload", "rest", "tile_costs", "bind"), (float(x) for x in ms)))

    def __del__(self):
        try:
            if getattr(self, "h", None):
                capi.lib().vpt_gpu_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def stream_handle(self, stream=None) -> int:
        s = stream if stream is not None else self.torch.cuda.current_stream(self.dev)
        return int(s.cuda_stream)

    def render_jobs(self, jid_begin: int, jid_count: int, film=None, records=None, stream=None):
        """Asynchronously render jobs [jid_begin, jid_begin + jid_count) into `film` (default: own)."""
        film = self.film if film is None else film
        assert film.is_cuda and film.dtype == self.torch.float32 and film.is_contiguous()
        assert film.numel() == self.cfg.height * self.cfg.width * 4
        L = capi.lib()
        s = C.c_void_p(self.stream_handle(stream))
        if records is None:
            capi.check(L.vpt_gpu_render_jobs(self.h, jid_begin, jid_count, C.c_void_p(film.data_ptr()), s),
                       "vpt_gpu_render_jobs")
        else:
            area = int(self.cfg.tile_size[0] * self.cfg.tile_size[1])
            assert records.numel() >= jid_count * area * 3 and records.dtype == self.torch.float32
            capi.check(L.vpt_gpu_render_jobs_records(self.h, jid_begin, jid_count, C.c_void_p(film.data_ptr()),
                                                     C.c_void_p(records.data_ptr()), s),
                       "vpt_gpu_render_jobs_records")

    def render_waves(self, first_wave: int, num_waves: int, film=None, stream=None):
        """Waves are 1-based (tile_provider.cpp:30): wave w covers jids [(w-1)*T, w*T)."""
        self.render_jobs((first_wave - 1) * self.jobs_per_wave, num_waves * self.jobs_per_wave, film, None, stream)

    def trace_jobs(self, jid_begin: int, jid_count: int, capacity: int = 1 << 20, film=None, stream=None):
        """Render jobs and return their Logger events (worker.cpp:16-48) as a numpy array of
        capi.EVENT_DTYPE sorted by (jid, seq).  Raises if more than `capacity` events occur."""
        torch = self.torch
        film = self.film if film is None else film
        buf = torch.empty((max(1, capacity), capi.EVENT_DTYPE.itemsize), dtype=torch.uint8, device=self.dev)
        n = C.c_uint64()
        capi.check(capi.lib().vpt_gpu_trace_jobs(self.h, jid_begin, jid_count, C.c_void_p(film.data_ptr()),
                                                 C.c_void_p(buf.data_ptr()), capacity, C.byref(n),
                                                 C.c_void_p(self.stream_handle(stream))), "vpt_gpu_trace_jobs")
        if n.value > capacity:
            raise RuntimeError(f"trace_jobs: {n.value} events exceed capacity {capacity}")
        ev = buf[: n.value].cpu().numpy().view(capi.EVENT_DTYPE).reshape(-1)
        return np.sort(ev, order=["jid", "seq"])

    def majorant_trace(self, origin, direction, max_rows: int = 1 << 16) -> np.ndarray:
        """Volume::log_majorant_trace (volume.cpp:176-192) rows [n][9] for one world ray."""
        o = np.ascontiguousarray(origin, np.float32).reshape(3)
        d = np.ascontiguousarray(direction, np.float32).reshape(3)
        rows = np.zeros((max_rows, 9), np.float32)
        n = C.c_int()
        fp = C.POINTER(C.c_float)
        capi.check(capi.lib().vpt_gpu_majorant_trace(self.h, o.ctypes.data_as(fp), d.ctypes.data_as(fp),
                                                     rows.ctypes.data_as(fp), max_rows, C.byref(n)),
                   "vpt_gpu_majorant_trace")
        if n.value > max_rows:
            raise RuntimeError(f"majorant_trace: {n.value} segments exceed max_rows {max_rows}")
        return rows[: n.value].copy()

    def set_rng_mode(self, mode: int) -> None:
        """capi.VPT_RNG_REFERENCE (default, the reference's samples) or capi.VPT_RNG_PIXEL
        (throughput mode: one stream per pixel; matches the reference only in expectation)."""
        capi.check(capi.lib().vpt_gpu_set_rng_mode(self.h, int(mode)), "vpt_gpu_set_rng_mode")

    def set_pixel_chunk(self, chunk: int) -> None:
        """Throughput mode: pixels per work item (0 = auto; else a power of two dividing the tile area).
        Samples never depend on it."""
        capi.check(capi.lib().vpt_gpu_set_pixel_chunk(self.h, int(chunk)), "vpt_gpu_set_pixel_chunk")

    def set_run_skipping(self, mode: int) -> None:
        """-1: the creation-time choice; 0 / 1: force the run-skipping kernel variant off / on."""
        capi.check(capi.lib().vpt_gpu_set_run_skipping(self.h, int(mode)), "vpt_gpu_set_run_skipping")

    def set_latency_kernel(self, mode: int, ungated: int = -1) -> None:
        """The latency kernel (lane cold state in VGPRs, 4-5 waves per SIMD): -1 auto (latency-bound launches,
        C1, and partly filled ones, C2 and small shares), 0 never, 1 always; `ungated` 1 / 0: partly filled
        launches on it use the latency gates / the context's (-1 keeps; default 0).  Samples never depend on it."""
        capi.check(capi.lib().vpt_gpu_set_latency_kernel(self.h, int(mode), int(ungated)), "vpt_gpu_set_latency_kernel")

    def set_compaction(self, every: int) -> None:
        """Live-path compaction on partly filled latency launches every `every` outer iterations (0: off);
        see include/vpt_gpu.h vpt_gpu_set_compaction.  Samples never depend on it."""
        capi.check(capi.lib().vpt_gpu_set_compaction(self.h, int(every)), "vpt_gpu_set_compaction")

    def latency_kernel_info(self) -> dict:
        m, b = C.c_int(), C.c_int()
        capi.check(capi.lib().vpt_gpu_latency_kernel_info(self.h, C.byref(m), C.byref(b)), "vpt_gpu_latency_kernel_info")
        return {"mode": int(m.value), "resident_blocks_per_cu": int(b.value)}

    def kernel_variant(self) -> dict:
        """The production kernel this context launches."""
        t, r = C.c_int(), C.c_int()
        capi.check(capi.lib().vpt_gpu_kernel_variant(self.h, C.byref(t), C.byref(r)), "vpt_gpu_kernel_variant")
        return {"has_temperature": bool(t.value), "run_skipping": bool(r.value)}

    def set_film_order(self, mode: int, max_bytes: int = 0) -> None:
        """capi.VPT_FILM_ORDERED (default: every pixel's samples added in wave order, the reference's film bit
        for bit; `max_bytes` caps the sample buffer, 0 = auto) or capi.VPT_FILM_ATOMIC (fp32 atomics in
        completion order).  See include/vpt_gpu.h vpt_gpu_set_film_order."""
        capi.check(capi.lib().vpt_gpu_set_film_order(self.h, int(mode), int(max_bytes)), "vpt_gpu_set_film_order")

    def film_order_info(self) -> dict:
        m, b, o, a = C.c_int(), C.c_uint64(), C.c_uint64(), C.c_uint64()
        capi.check(capi.lib().vpt_gpu_film_order_info(self.h, C.byref(m), C.byref(b), C.byref(o), C.byref(a)),
                   "vpt_gpu_film_order_info")
        return {"mode": int(m.value), "buffer_bytes": int(b.value), "ordered_launches": int(o.value),
                "atomic_launches": int(a.value)}

    def set_job_order(self, mode: int) -> None:
        """Scheduling order of whole-wave launches: capi.VPT_ORDER_JID (TileProvider order),
        VPT_ORDER_COST_WAVE_MAJOR, VPT_ORDER_COST_TILE_MAJOR, VPT_ORDER_COST_TAIL or VPT_ORDER_COST_SAME_TILE
        (default; launches that add with film atomics take VPT_ORDER_COST_TAIL).
        Samples never depend on it."""
        capi.check(capi.lib().vpt_gpu_set_job_order(self.h, int(mode)), "vpt_gpu_set_job_order")

    def set_job_order_tail(self, waves: int) -> None:
        """VPT_ORDER_COST_TAIL's tile-major wave count (0 = auto)."""
        capi.check(capi.lib().vpt_gpu_set_job_order_tail(self.h, int(waves)), "vpt_gpu_set_job_order_tail")

    def tile_costs(self):
        """(cost float32[T], tile ranks by descending cost uint32[T]) of the job-order pass."""
        T = self.cfg.jobs_per_wave()
        cost, rank = np.zeros(T, np.float32), np.zeros(T, np.uint32)
        capi.check(capi.lib().vpt_gpu_tile_costs(self.h, cost.ctypes.data_as(C.POINTER(C.c_float)),
                                                  rank.ctypes.data_as(C.POINTER(C.c_uint32))), "vpt_gpu_tile_costs")
        return cost, rank

    def set_tile_costs(self, cost) -> None:
        """Replace the job-order cost estimates with per-tile costs (float32[T], e.g. measured)."""
        c = np.ascontiguousarray(cost, np.float32)
        assert c.shape == (self.cfg.jobs_per_wave(),)
        capi.check(capi.lib().vpt_gpu_set_tile_costs(self.h, c.ctypes.data_as(C.POINTER(C.c_float))),
                   "vpt_gpu_set_tile_costs")

    def set_job_permutation(self, perm) -> None:
        """Explicit order of launches with len(perm) jobs: item k renders job jid_begin + perm[k]
        (None or empty clears it).  Samples never depend on it."""
        p = np.ascontiguousarray(perm if perm is not None else [], np.uint32)
        capi.check(capi.lib().vpt_gpu_set_job_permutation(self.h, p.ctypes.data_as(C.POINTER(C.c_uint32)), p.size),
                   "vpt_gpu_set_job_permutation")

    def counters(self, reset: bool = False) -> dict:
        c = capi.Counters()
        capi.check(capi.lib().vpt_gpu_counters(self.h, C.byref(c), 1 if reset else 0), "vpt_gpu_counters")
        return c.as_dict()

    def set_tuning(self, gate_min: int = 0, gate_idle: int = -1, grid_blocks: int = 0, gate_eval: int = 0,
                   gate_walk: int = -1):
        capi.check(capi.lib().vpt_gpu_set_tuning(self.h, gate_min, gate_idle, grid_blocks, gate_eval, gate_walk),
                   "vpt_gpu_set_tuning")

    def set_latency_tuning(self, wave_lanes: int = -1, gate_min: int = 0, gate_idle: int = -1, gate_eval: int = 0,
                           gate_walk: int = -1):
        """Knobs of latency-bound launches (fewer items than grid lanes): lanes per wavefront that take
        jobs (0 = auto) and their gates; see include/vpt_gpu.h."""
        capi.check(capi.lib().vpt_gpu_set_latency_tuning(self.h, wave_lanes, gate_min, gate_idle, gate_eval, gate_walk),
                   "vpt_gpu_set_latency_tuning")

    PROFILE_BLOCKS = ["iter", "fetch", "pixel", "ray", "sample", "need_seg", "step", "draw", "trilinear",
                      "event", "shadow_hit", "none", "nee_done", "finish",
                      "w_walk", "w_eval", "w_nee", "w_finish", "w_ray", "w_pixel", "w_done"]

    PROFILE_SECTIONS = ["fetch", "pixel", "ray", "walk", "eval", "nee", "finish", "seg", "step", "draw"]

    def profile(self, reset: bool = False) -> dict:
        """SIMT profile of a -DVPT_PROFILE build: {block: (wave executions, mean active lanes)} and
        {"cycles": {section: share of wave time}}."""
        buf = (C.c_uint64 * 128)()
        capi.check(capi.lib().vpt_gpu_profile(self.h, buf, 128, 1 if reset else 0), "vpt_gpu_profile")
        out = {}
        for i, name in enumerate(self.PROFILE_BLOCKS):
            ex, lanes = int(buf[2 * i]), int(buf[2 * i + 1])
            out[name] = (ex, round(lanes / ex, 2) if ex else 0.0)
        base = 2 * len(self.PROFILE_BLOCKS)
        cyc = [int(buf[base + i]) for i in range(len(self.PROFILE_SECTIONS))]
        tot = sum(cyc) or 1
        out["cycles"] = {n: round(c / tot, 4) for n, c in zip(self.PROFILE_SECTIONS, cyc)}
        out["cycles_total"] = tot
        return out

    def launch_info(self):
        g, b = C.c_int(), C.c_int()
        capi.check(capi.lib().vpt_gpu_launch_info(self.h, C.byref(g), C.byref(b)), "vpt_gpu_launch_info")
        return int(g.value), int(b.value)

    def film_host(self) -> np.ndarray:
        self.torch.cuda.synchronize(self.dev)
        return self.film.cpu().numpy()


class Feed:
    """A running launch that renders job ids as they are pushed (vpt_gpu_feed_*, include/vpt_gpu.h) into
    `film` (a zeroed device tensor of the context's film shape) on `stream` (a torch stream of the device).  A
    staged feed counts its completed jobs per tile: snapshot() adds what it has rendered so far into a host
    film (also while it runs: the copy engines read the device film beside the launch), collect() the rest
    once it has ended (then it clears `film`)."""

    def __init__(self, integrator: "Integrator", film, stream, window: int = 1 << 19, staged: bool = False):
        self.it, self.film, self.stream = integrator, film, stream
        h = C.c_void_p()
        fn = "vpt_gpu_feed_open_staged" if staged else "vpt_gpu_feed_open"
        capi.check(getattr(capi.lib(), fn)(integrator.h, C.c_void_p(film.data_ptr()),
                                           C.c_void_p(int(stream.cuda_stream)), int(window), C.byref(h)), fn)
        self.h = h

    def push(self, jids) -> None:
        j = np.ascontiguousarray(jids, np.uint64)
        capi.check(capi.lib().vpt_gpu_feed_push(self.h, j.ctypes.data_as(C.POINTER(C.c_uint64)), j.size),
                   "vpt_gpu_feed_push")

    def close(self) -> None:
        capi.check(capi.lib().vpt_gpu_feed_close(self.h), "vpt_gpu_feed_close")

    def done(self) -> bool:
        d = C.c_int()
        capi.check(capi.lib().vpt_gpu_feed_query(self.h, C.byref(d), None), "vpt_gpu_feed_query")
        return bool(d.value)

    def backlog(self) -> int:
        b = C.c_uint64()
        capi.check(capi.lib().vpt_gpu_feed_backlog(self.h, C.byref(b)), "vpt_gpu_feed_backlog")
        return int(b.value)

    def destroy(self) -> None:
        if self.h:
            h, self.h = self.h, None
            capi.check(capi.lib().vpt_gpu_feed_destroy(h), "vpt_gpu_feed_destroy")

    def snapshot(self, film_host: np.ndarray) -> None:
        """Adds what a staged feed has rendered since the previous snapshot into film_host (float32,
        C-contiguous [H][W][4])."""
        assert film_host.dtype == np.float32 and film_host.flags.c_contiguous
        capi.check(capi.lib().vpt_gpu_feed_snapshot(self.h, film_host.ctypes.data_as(C.POINTER(C.c_float))),
                   "vpt_gpu_feed_snapshot")

    def collect(self, film_host: np.ndarray) -> None:
        """Waits for a staged feed and adds the rest of its film into film_host (float32, C-contiguous); frees it."""
        assert film_host.dtype == np.float32 and film_host.flags.c_contiguous
        h, self.h = self.h, None
        capi.check(capi.lib().vpt_gpu_feed_collect(h, film_host.ctypes.data_as(C.POINTER(C.c_float))),
                   "vpt_gpu_feed_collect")


def run(cfg: capi.Configuration, integrator: Integrator, tp: TileProvider, film: Optional[np.ndarray] = None,
        batch_jobs: int = 4096, flush_seconds: float = 0.2, window: int = 1 << 19) -> np.ndarray:
    """Drop-in for vpt::run (worker.cpp:92-208): drain `tp` on the GPU into `film` (host float32 [H][W][4],
    the reference's Image<float,4> layout), as include/vpt_run.hpp's drain does it (without its threads): the
    job ids go to one running launch through a staged feed (no launch drain between batches), every
    flush_seconds what it has completed is added into `film` (vpt_gpu_feed_snapshot) -- which therefore fills
    in during the run (main.cpp:101-132 shows it at 5 FPS) -- and the collect adds the rest."""
    torch = integrator.torch
    out = film if film is not None else np.zeros((integrator.cfg.height, integrator.cfg.width, 4), np.float32)
    if out.dtype != np.float32 or not out.flags.c_contiguous or out.size != integrator.film.numel():
        raise ValueError("run: film must be a C-contiguous float32 [H][W][4] array")
    dev_film = torch.zeros_like(integrator.film)
    torch.cuda.synchronize(integrator.dev)  # zeroed before the feed's launch (on its own stream) reads it
    stream = torch.cuda.Stream(device=integrator.dev)
    feed = Feed(integrator, dev_film, stream, window, staged=True)
    last = time.monotonic()
    try:
        while True:
            begin, count = tp.next_batch(batch_jobs)
            if count == 0:
                break
            feed.push(np.arange(begin, begin + count, dtype=np.uint64))
            if time.monotonic() - last >= flush_seconds:
                feed.snapshot(out)
                last = time.monotonic()
        feed.collect(out)
    finally:
        feed.destroy()
    return out


def film_to_xyz(film: np.ndarray) -> np.ndarray:
    """XYZ / W per pixel (main.cpp:15)."""
    return film[..., :3] / film[..., 3:4]
