"""Per-kernel ISA summary of /tmp/isa/vpt.s (from tools/isa_stats.sh): instruction count, scratch
accesses with their line numbers, and the loop labels, for the production kernel by default.
    python tools/isa_blocks.py [Lb0ELb0E]"""
import re, sys
t = open("/tmp/isa/vpt.s").read()
tag = sys.argv[1] if len(sys.argv) > 1 else "Lb0ELb0ELb0E"
m = re.search(r"^_ZN3vpt20vpt_integrate_kernelI%sEEvPKNS_8DevScene\w*:" % tag, t, re.M)
seg = t[m.end():]
seg = seg[:seg.index(".Lfunc_end")]
lines = seg.split("\n")
ins = [l for l in lines if l.startswith("\t") and not l.strip().startswith((";", "."))]
print("instructions", len(ins))
for i, l in enumerate(lines):
    s = l.strip()
    if "scratch_" in s:
        print(i, s)
