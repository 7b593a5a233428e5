"""tools/ubench/gather `pool` output -> profiles/<tag>_pool_ceiling.json: the rate of divergent 32-byte
per-lane gathers (one stencil piece per lane, two adjacent 16-B loads) from tables of the stencil pool's
size, best over chains per lane at 4 / 7 waves per SIMD.  bench.py's roofline.pipe_frac interpolates it
at the run's pool size (log-log between the measured sizes).
Usage: python tools/pool_ceiling.py <tag> <pool.txt>"""
import json
import sys
from pathlib import Path

tag, txt = sys.argv[1], Path(sys.argv[2])
best = {}
for line in txt.read_text().splitlines():
    p = line.split()
    if len(p) == 6 and p[0] == "width" and p[1] == "32":
        mib, rate = float(p[2]), float(p[5]) * 1e9
        best[mib] = max(best.get(mib, 0.0), rate)
out = {"kind": "pool_ceiling", "entry_bytes": 32,
       "points": [{"table_mib": m, "entries_per_s_per_cu": round(best[m], 1)} for m in sorted(best)],
       "source": f"tools/ubench/gather pool ({txt.name}): random 32-B entries, 256 iterations per lane, 1 or 2 "
                 "chains per lane, 4 or 7 waves per SIMD, best of the four"}
dst = Path(__file__).resolve().parents[1] / "profiles" / f"{tag}_pool_ceiling.json"
dst.write_text(json.dumps(out, indent=1) + "\n")
print(dst)
