"""Headless renderer: ``python -m volume_path_tracer_amd config_path output_path``.

The reference's main (src/main.cpp:26-146) without the raylib window: read the scene, load the
volume (relative to the scene file), render every wave on the GPU through the drop-in integrator,
convert the film to 8-bit sRGB (film_to_image) and save a PNG.

``--synthetic cloud|constant|fire[:N]`` replaces the volume file by a generated stand-in (the
reference's volumes are not shipped).  ``--spp`` overrides num_waves; ``--size WxH`` overrides
output_size.  Exits 1 on a fatal error, like vptFATAL.
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path


def _parse_synth(spec: str):
    kind, _, n = spec.partition(":")
    kinds = {"constant": (0, False), "cloud": (1, False), "fire": (1, True)}
    if kind not in kinds:
        raise ValueError(f"--synthetic wants constant|cloud|fire[:N], got {spec!r}")
    return kinds[kind][0], int(n or (128 if kind == "constant" else 512)), kinds[kind][1]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m volume_path_tracer_amd", description=__doc__.splitlines()[0])
    ap.add_argument("config_path")
    ap.add_argument("output_path")
    ap.add_argument("--synthetic", default=None, help="constant|cloud|fire[:N] stand-in volume")
    ap.add_argument("--spp", type=int, default=None, help="override num_waves")
    ap.add_argument("--size", default=None, help="override output_size, WxH")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--batch-jobs", type=int, default=4096, help="tokens taken per push into the running launch")
    ap.add_argument("--film-out", default=None, help="also save the raw XYZW film (.npy)")
    ap.add_argument("--event-log", default=None,
                    help="write the Logger event log (log.csv format) of the first --event-jobs jobs")
    ap.add_argument("--event-jobs", type=int, default=1)
    args = ap.parse_args(argv)

    from . import image, traces, volumes
    from .render import Integrator, TileProvider, run
    from .scenes import SynthGrid, read_configuration

    try:
        config_path = Path(args.config_path).resolve(strict=True)
        cfg = read_configuration(config_path)
        if args.spp is not None:
            cfg.num_waves = int(args.spp)
        if args.size:
            w, h = (int(v) for v in args.size.lower().split("x"))
            cfg.output_size[0], cfg.output_size[1] = w, h
        keep = []
        if args.synthetic:
            kind, n, with_temp = _parse_synth(args.synthetic)
            sd = SynthGrid(kind, n)
            st = SynthGrid(2, n) if with_temp else None
            keep += [sd, st]
            dens, temp = sd.grid(copy=False), (st.grid(copy=False) if st else None)
        else:
            vol = config_path.parent / cfg.volume_path.decode()
            dens, temp = volumes.read_grids(vol)
        if temp is not None and temp.leaf_count:
            print(f"TempMin: {float(temp.leaf_values.min())}, TempMax: {float(temp.leaf_values.max())}")

        it = Integrator(cfg, dens, temp, device=args.device)
        tp = TileProvider(cfg.output_size, cfg.num_waves, cfg.tile_size)
        tp.reset_eta()
        t0 = time.perf_counter()
        film = run(cfg, it, tp, batch_jobs=args.batch_jobs)
        ms = (time.perf_counter() - t0) * 1e3
        print(f"[vpt] Rendering complete in {ms:.0f} ms ({cfg.width}x{cfg.height}, {cfg.num_waves} spp)",
              file=sys.stderr)
        if args.event_log:
            scratch = it.torch.zeros_like(it.film)  # the traced jobs are not part of the image
            traces.write_event_log(it.trace_jobs(0, args.event_jobs, film=scratch), args.event_log)
        if args.film_out:
            import numpy as np

            np.save(args.film_out, film)
        image.save_png(args.output_path, image.film_to_image(film))
    except Exception as e:  # vptFATAL: message and exit(1)
        print(f"[vpt] FATAL: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
