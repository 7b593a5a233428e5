"""Per-kernel ISA summary of the integrator kernels: instructions, SGPR spill traffic (v_writelane / v_readlane)
and scratch accesses, for the whole kernel and per region between its s_setprio marks (the walk loop runs at
priority 3, so its region is the one after `s_setprio 3`).

    hipcc -xhip --offload-arch=gfx950 --cuda-device-only -S <build.py's flags> volume_path_tracer_amd/csrc/vpt_gpu.hip -o /tmp/vpt.s
    python tools/isa_blocks.py /tmp/vpt.s [flags ...]

flags: the kernel's template bools HasTemp, Debug, Runs, Lat, Compact, Feed as a digit string (default: every
kernel; e.g. 000000 = the density kernel C3 runs, 001000 = its run-skipping variant, 100000 = the temperature
kernel C4 runs)."""
import re
import sys

INS = re.compile(r"^\s+[a-z]+_[a-z0-9_]+")


def count(lines):
    return (sum(1 for l in lines if INS.match(l)), sum("v_readlane" in l for l in lines),
            sum("v_writelane" in l for l in lines), sum("scratch_" in l for l in lines))


def main():
    text = open(sys.argv[1]).read()
    want = set(sys.argv[2:])
    for m in re.finditer(r"^(_ZN3vpt20vpt_integrate_kernelI(\w+?)EEv\w*):", text, re.M):
        flags = "".join(re.findall(r"Lb(\d)", m.group(2)))
        if want and flags not in want:
            continue
        body = text[m.end():text.index(".Lfunc_end", m.end())].split("\n")
        print("%s  insts %d  readlane %d  writelane %d  scratch %d" % ((flags,) + count(body)))
        marks = [i for i, l in enumerate(body) if "s_setprio" in l]
        if want:
            for a, b in zip([0] + marks, marks + [len(body)]):
                label = body[a].strip() if a in marks else "entry"
                print("   from %-12s insts %5d  readlane %3d  writelane %3d  scratch %d" % ((label,) + count(body[a:b])))


if __name__ == "__main__":
    main()
