"""Generate tests/golden/pcg32_fast_ref.json from oracle/_ref/pcg32_fast_kat, a tool compiled
directly against the reference's vendored pcg header (external/pcg-cpp/include/pcg/pcg_random.hpp).
The 64-bit seeds are hash(seed, jid) values from tests/golden/rng_kat.json plus a few raw seeds."""
import json, subprocess
from pathlib import Path
root = Path(__file__).resolve().parents[1]
tool = root / "oracle/_ref/pcg32_fast_kat"
kat = json.loads((root / "tests/golden/rng_kat.json").read_text())
seeds = [c["hash"] for c in kat["cases"]] + ["0x1234", "0x0", "0xffffffffffffffff", "0x8000000000000000"]
out = {"_source": "oracle/_ref/pcg32_fast_kat (reference's vendored pcg_random.hpp), tools/make_golden_pcg.py", "streams": []}
for s in seeds:
    vals = subprocess.run([str(tool), s[2:], "64"], check=True, capture_output=True, text=True).stdout.split()
    out["streams"].append({"seed64": s, "u32": [int(v) for v in vals]})
(root / "tests/golden/pcg32_fast_ref.json").write_text(json.dumps(out, indent=1) + "\n")
print("wrote", len(out["streams"]), "streams")
