export TMPDIR=/tmp; O=gpurun_out/ab; mkdir -p $O
for L in ${LIBS}; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 300 python tools/tune.py --spp 256 --gates ${GATES:-8:12:24:4} --reps 2 > $O/$L.log 2>&1 || exit $?
  echo "$L $(grep Msps $O/$L.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms"], d["Msps"])')"
done
