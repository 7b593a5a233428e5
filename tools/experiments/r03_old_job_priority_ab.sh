set -o pipefail
O=gpurun_out/r03z; mkdir -p $O
bash tools/ab_lib.sh r03z volume_path_tracer_amd/lib/libvpt_oldprio.so c3,c4 2 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
for us in 20000 80000 10000; do
  for c in c3 c4; do
    VPT_OLD_JOB_US=$us VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_oldprio.so timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/v_${us}_$c.json 2> $O/v_${us}_$c.err || exit 1
    python -c "import json; d=json.loads(open('$O/v_${us}_$c.json').read().strip().splitlines()[-1]); print('variant us=$us $c', d['ms_per_step'], d['value'])" >> $O/ab.txt
  done
done
timeout -k 10 200 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/base_c3_end.json 2>&1 && python -c "import json; d=json.loads(open('$O/base_c3_end.json').read().strip().splitlines()[-1]); print('base end c3', d['ms_per_step'])" >> $O/ab.txt
cat $O/ab.txt
