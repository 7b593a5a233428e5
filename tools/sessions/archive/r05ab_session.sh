#!/bin/bash
# r05ab: C3 one-launch frames, 256 spp, best of 3 per run: the library before the urgent-fetch gate (prev), with
# the gate's ballot always run (cur), and with the ballot behind a uniform feed-mode branch (new); 3 rounds,
# rotating order (tools/tune.py, the bench's default grid and gates).
set -u
O=gpurun_out/r05ab; mkdir -p $O
L=$PWD/volume_path_tracer_amd/lib
run() {  # name lib round
  VPT_LIB=$2 timeout -k 10 300 python tools/tune.py --config c3 --spp 256 --gates 6:8:36:4 --reps 3 > $O/c3_$1_$3.jsonl 2>&1 || exit 1
  echo "round $3 $1 $(grep -o '"ms": [0-9.]*' $O/c3_$1_$3.jsonl)"
}
run prev $L/ab_prev/libvpt_amd.so 1 && run cur $L/ab_cur/libvpt_amd.so 1 && run new $L/libvpt_amd.so 1 &&
run cur $L/ab_cur/libvpt_amd.so 2 && run new $L/libvpt_amd.so 2 && run prev $L/ab_prev/libvpt_amd.so 2 &&
run new $L/libvpt_amd.so 3 && run prev $L/ab_prev/libvpt_amd.so 3 && run cur $L/ab_cur/libvpt_amd.so 3
