"""Multi-GPU partition of the job space and the film reduce.

Jobs are (tile, wave) pairs keyed by job id; every wave covers the whole image, so sharding by
wave balances perfectly and keeps every RNG stream identical to the 1-GPU / CPU runs.

* ``weak``:  rank r renders its own block of ``spp`` waves, r*spp+1 .. (r+1)*spp — the per-GPU
             work is fixed as N grows and the reduced film holds N*spp samples per pixel.
* ``strong``: the ``spp`` waves of one image are split into N contiguous, balanced blocks (the
             round-robin deal of SURVEY §8e balances the same way; contiguous blocks keep it to one
             persistent-kernel launch per rank), so N GPUs share one fixed image.

After rendering, the H*W*4 fp32 films are summed over the ranks with one all-reduce
(RCCL over xGMI for the "nccl" backend; gloo in the CPU tests) — the only exchange the path has.
"""
from __future__ import annotations

from typing import List, Tuple


def rank_wave_ranges(rank: int, world: int, spp: int, mode: str = "weak") -> List[Tuple[int, int]]:
    """Contiguous (first_wave, num_waves) runs this rank renders (waves are 1-based)."""
    if not (0 <= rank < world) or spp <= 0:
        raise ValueError("bad rank/world/spp")
    if mode == "weak":
        return [(1 + rank * spp, spp)]
    if mode == "strong":
        base, extra = divmod(spp, world)
        first = 1 + rank * base + min(rank, extra)
        n = base + (1 if rank < extra else 0)
        return [(first, n)] if n else []
    raise ValueError(f"unknown mode {mode!r}")


def rank_job_ranges(rank: int, world: int, spp: int, jobs_per_wave: int, mode: str = "weak"):
    """The same partition as job-id ranges (jid_begin, jid_count)."""
    return [((w - 1) * jobs_per_wave, n * jobs_per_wave) for w, n in rank_wave_ranges(rank, world, spp, mode)]


def total_samples_per_pixel(world: int, spp: int, mode: str = "weak") -> int:
    return spp * world if mode == "weak" else spp


def render_rank(integrator, rank: int, world: int, spp: int, mode: str = "weak", film=None, stream=None):
    """Launch this rank's share of the job space on its integrator (asynchronously, on `stream`) into
    `film` (default: the integrator's own).  Returns the (jid_begin, count) ranges launched."""
    ranges = rank_job_ranges(rank, world, spp, integrator.jobs_per_wave, mode)
    for b, n in ranges:
        integrator.render_jobs(b, n, film=film, stream=stream)
    return ranges


def reduce_film(film, group=None):
    """Sum the per-rank films in place (every rank ends with the whole image): RCCL over xGMI for a
    device film with the "nccl" backend; with gloo (CPU tests, several ranks sharing one GPU) a
    device film is summed through a host copy."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if film.is_cuda and dist.get_backend(group) == "gloo":
            host = film.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            film.copy_(host)
        else:
            dist.all_reduce(film, op=dist.ReduceOp.SUM, group=group)
    return film
