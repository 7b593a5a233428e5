#!/usr/bin/env python3
"""Move earlier rounds' profiles/ files under profiles/archive/ (VERDICT r05 hygiene), keeping in profiles/ the
current round's files and every file bench.py still reads (the newest *_pmc.json / *_counters.json per config, the
gather / pool / mix ceilings), and point the repository's text references at the moved files.

    python tools/archive_profiles.py r06      # keep r06* in profiles/
"""
import json
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
P = ROOT / "profiles"
keep_prefix = sys.argv[1] if len(sys.argv) > 1 else "r06"


def newest(pattern, match):
    for pf in sorted(P.glob(pattern), reverse=True):
        try:
            j = json.loads(pf.read_text())
        except Exception:
            continue
        if match(j):
            return pf.name
    return None


keep = set()
for cfg in ("c1", "c2", "c3", "c4", "c5"):
    for pat in ("*_pmc.json", "*_counters.json", "*_mix_ceiling.json"):
        n = newest(pat, lambda j, c=cfg: j.get("config") == c and not j.get("bench_args"))
        if n:
            keep.add(n)
for pat in ("*_gather_ceiling.json", "*_pool_ceiling.json"):
    n = newest(pat, lambda j: True)
    if n:
        keep.add(n)
keep |= {k.replace(".json", ".txt") for k in keep}  # their text companions
moved = []
(P / "archive").mkdir(exist_ok=True)
for f in sorted(P.iterdir()):
    if f.is_file() and re.match(r"r0\d", f.name) and not f.name.startswith(keep_prefix) and f.name not in keep:
        subprocess.run(["git", "mv", "-k", str(f), str(P / "archive" / f.name)], cwd=ROOT, check=True)
        moved.append(f.name)
# text references "profiles/<name>" -> "profiles/archive/<name>"
names = set(moved)
pat = re.compile(r"profiles/(r0[0-9A-Za-z_.\-]+)")
for t in subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True).stdout.split():
    if (not t.endswith((".md", ".py", ".sh", ".h", ".hpp", ".hip", ".cpp", ".txt")) or t.startswith("profiles/")
            or t in ("VERDICT.md", "ADVICE.md", "SURVEY.md", "BASELINE.md")):  # (the judge's / survey's files stay as written)
        continue
    path = ROOT / t
    s = path.read_text(errors="replace")
    s2 = pat.sub(lambda m: "profiles/archive/" + m.group(1) if m.group(1).rstrip(".,;:)") in names else m.group(0), s)
    if s2 != s:
        path.write_text(s2)
print(f"kept {len(keep)} referenced files, moved {len(moved)} to profiles/archive/")
