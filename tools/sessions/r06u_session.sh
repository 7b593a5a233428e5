#!/bin/bash
# r06u: where the ordered drop-in frame's time goes -- C3 drop-in frames (harness drain, as bench's dropin) with the
# ordered frame off / on, VPT_DRAIN_TRACE phases; and the first call (mode=run) traced.
set -u
export TMPDIR=/tmp
O=gpurun_out/${SESSION:-r06u}; mkdir -p $O; G=/tmp/r06u_grid; mkdir -p $G
python - <<'PY' || exit 1
from pathlib import Path
from volume_path_tracer_amd import nvdb
from volume_path_tracer_amd.scenes import SynthGrid
g = SynthGrid(1, 512)  # (the owner stays alive while its grid is read)
Path("/tmp/r06u_grid/density.grid").write_bytes(nvdb.buffer_from_grid(g.grid(copy=False), "density"))
PY
B="tests/native/build/run_gpu_harness config=volume_path_tracer_amd/scenes/wdas_cloud.json w=1920 h=1080 waves=256 grid_n=512 kind=1 dist=800 threads=1 batch=4096 temperature=0"
for ord in 0 1; do
  VPT_DRAIN_TRACE=1 timeout -k 10 120 $B out=$G/f.f32 frames=3 warmup=1 ordered=$ord > $O/drain_ord$ord.out 2> $O/drain_ord$ord.err || exit 1
  echo "ordered=$ord $(grep render_ms $O/drain_ord$ord.out | tr '\n' ' ')"
done
for ord in 1 0; do
  VPT_DROPIN_ORDERED=$ord VPT_DRAIN_TRACE=1 timeout -k 10 120 $B out=$G/g.f32 mode=run gridbuf=$G/density.grid > $O/run_ord$ord.out 2> $O/run_ord$ord.err || exit 1
  echo "run ordered=$ord $(grep phases $O/run_ord$ord.out)"
done
rm -rf $G
