#!/bin/bash
# r05u3: the one-launch frames with the urgent-fetch gate (new) vs the library before it (prev): C3 / C4, 256 spp,
# best of 3 per run, alternating, 2 rounds (tools/tune.py, the bench's default grid and gates).
set -u
O=gpurun_out/r05u3; mkdir -p $O
for r in 1 2; do
  for c in c3 c4; do
    VPT_LIB=$PWD/volume_path_tracer_amd/lib/ab_prev/libvpt_amd.so timeout -k 10 300 python tools/tune.py --config $c --spp 256 --gates 6:8:36:4 --reps 3 > $O/${c}_prev_$r.jsonl 2>&1 || exit 1
    timeout -k 10 300 python tools/tune.py --config $c --spp 256 --gates 6:8:36:4 --reps 3 > $O/${c}_new_$r.jsonl 2>&1 || exit 1
    echo "$c round $r prev $(grep -o '"ms": [0-9.]*' $O/${c}_prev_$r.jsonl) new $(grep -o '"ms": [0-9.]*' $O/${c}_new_$r.jsonl)"
  done
done
