"""Extract the CIE 1931 2-degree colour-matching functions (360-830 nm, 1 nm) used by the reference.

Dev-time tool: reads the tabulated data out of the reference's `src/spectral_data/xyz.hpp`
(which itself carries pbrt-v4's copy of the CIE 1931 standard-observer tables, Apache-2.0) and writes
them as a plain CSV data file that the framework ships (`volume_path_tracer_amd/data/cie1931_xyz.csv`).
Only numbers are carried over; the float text is kept verbatim so that parsing it with strtof gives the
same float32 values the reference compiles into its binary (xyz.hpp:17,116,215,314).
"""
import re
import sys
from pathlib import Path

src = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/spectral_data/xyz.hpp").read_text()
out = Path(sys.argv[2] if len(sys.argv) > 2 else Path(__file__).resolve().parents[1] / "volume_path_tracer_amd/data/cie1931_xyz.csv")

def block(name):
    m = re.search(r"data_t\s+%s\s*\{(.*?)\};" % name, src, re.S)
    body = re.sub(r"//[^\n]*", "", m.group(1))
    vals = [v for v in re.split(r"[\s,]+", body) if v]
    assert len(vals) == 471, (name, len(vals))
    return vals

X, Y, Z = block("X"), block("Y"), block("Z")
yint = re.search(r"Y_integral\s*=\s*([0-9.eE+-]+)", src).group(1)
lines = ["# CIE 1931 2-degree standard observer, 1 nm steps (pbrt-v4 tables as used by the reference)",
         "# Y_integral=%s" % yint, "lambda_nm,x_bar,y_bar,z_bar"]
for i in range(471):
    lines.append("%d,%s,%s,%s" % (360 + i, X[i], Y[i], Z[i]))
out.write_text("\n".join(lines) + "\n")
print("wrote", out)
