#!/bin/bash
# Builds the integrator library of an earlier commit (A/B baselines): volume_path_tracer_amd/lib/libvpt_<name>.so
# Usage: bash tools/build_rev_lib.sh <commit> <name>
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/vpt_rev_$2
rm -rf $W && git -C $R worktree add -f $W $1 > /dev/null 2>&1
(cd $W && python -m volume_path_tracer_amd.build > /dev/null)
cp $W/volume_path_tracer_amd/lib/libvpt_amd.so $R/volume_path_tracer_amd/lib/libvpt_$2.so
git -C $R worktree remove --force $W
echo "built volume_path_tracer_amd/lib/libvpt_$2.so from $1"
