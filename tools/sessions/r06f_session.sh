#!/bin/bash
# r06f: kernel A/Bs on the ordered film: ordered-film stores from the lane itself (not regrouped), and the ray-setup
# block with its own gate (12 / 20 lanes); production parity of each variant, then C3 / C4 frames alternating.
set -u
export TMPDIR=/tmp
for v in direct gray12 gray20; do
  echo "== $v"
  bash tools/ab_lib.sh r06f_$v volume_path_tracer_amd/lib/libvpt_$v.so c3,c4 2 || exit $?
done
