#!/bin/bash
# Latency-bound launches (vpt_gpu_set_latency_tuning): parity tests, then C1 / C2 timing over grid sizes
# and latency knobs, then an A/B of the C3 frame against the previous library (libvpt_amd_base.so).
# Usage: bash tools/latency_sweep.sh <tag>
set -u
export TMPDIR=/tmp; O=gpurun_out/${1:-lat}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; if [ $rc -ne 0 ]; then tail -30 $O/pytest.log; exit $rc; fi
LAT=${LAT:-64:6:8:36:4,0:6:8:36:4,0:1:65:1:1,0:1:65:1:0,0:1:65:8:2,0:2:16:8:2}
timeout -k 10 300 python tools/tune.py --config c1 --spp 4 --gates 6:8:36:4 --blocks 256,512,1024,1792 --lat $LAT --reps 3 > $O/c1.log 2>&1 || { tail -5 $O/c1.log; exit 1; }
grep Msps $O/c1.log | cut -c1-200
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_base.so timeout -k 10 300 python tools/tune.py --config c1 --spp 4 --gates 6:8:36:4 --blocks 256,1792 --reps 3 > $O/c1_base.log 2>&1 || exit 1
grep Msps $O/c1_base.log | cut -c1-200
timeout -k 10 300 python tools/tune.py --config c2 --spp 64 --gates 6:8:36:4 --blocks 768,1792 --lat 0:6:8:36:4,0:1:65:1:1,0:2:16:8:2 --reps 2 > $O/c2.log 2>&1 || { tail -5 $O/c2.log; exit 1; }
grep Msps $O/c2.log | cut -c1-200
LIBS="libvpt_amd_base libvpt_amd" ROUNDS="1 2" bash tools/ab_libs.sh ${1:-lat}/ab
