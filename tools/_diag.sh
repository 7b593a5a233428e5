export TMPDIR=/tmp; O=gpurun_out/diag; mkdir -p $O
( while sleep 20; do echo "tick $(date +%s)"; done ) & HB=$!
for OR in 0 2; do
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_prof.so timeout -k 10 300 python tools/tune.py --spp 256 --gates 8:12:24:4 --reps 1 --profile --order $OR > $O/prof.o$OR.log 2>&1 || { kill $HB; exit 1; }
echo "order $OR"; grep profile $O/prof.o$OR.log | cut -c1-1500
done
for OR in 0 2; do
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_ptime.so timeout -k 10 300 python tools/tune.py --spp 512 --gates 8:12:24:4 --reps 1 --profile --order $OR > $O/ptime.o$OR.log 2>&1 || { kill $HB; exit 1; }
grep cycles $O/ptime.o$OR.log | python3 -c "import sys,json; [print(json.loads(l)['profile']['cycles'], json.loads(l)['profile']['cycles_total']) for l in sys.stdin if 'profile' in l]"
done
kill $HB
