#!/bin/bash
# r06x: the first run() with the frame's fresh memory touched at allocation (a memset on the context's stream), C3,
# ordered on / off, alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O; G=/tmp/r06x_grid; mkdir -p $G
python - <<'PY' || exit 1
from pathlib import Path
from volume_path_tracer_amd import nvdb
from volume_path_tracer_amd.scenes import SynthGrid
g = SynthGrid(1, 512)  # (the owner stays alive while its grid is read)
Path("/tmp/r06x_grid/density.grid").write_bytes(nvdb.buffer_from_grid(g.grid(copy=False), "density"))
PY
B="tests/native/build/run_gpu_harness config=volume_path_tracer_amd/scenes/wdas_cloud.json w=1920 h=1080 waves=256 grid_n=512 kind=1 dist=800 threads=12 batch=4096 temperature=0"
for ord in 1 0 1 0; do
  VPT_DROPIN_ORDERED=$ord VPT_DRAIN_TRACE=1 timeout -k 10 120 $B out=$G/g.f32 mode=run gridbuf=$G/density.grid > $O/run_ord$ord.out 2> $O/run_ord$ord.err || exit 1
  echo "run ordered=$ord $(grep phases $O/run_ord$ord.out)"
done
rm -rf $G
