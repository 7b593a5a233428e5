# r03zp: the NEE-completion / ray-setup blocks' own gates (VPT_GATE_NEE / VPT_GATE_RAY, 0 = gate_min), C3 frames
set -o pipefail
O=gpurun_out/r03zp; mkdir -p $O
for spec in "0 0" "12 0" "20 0" "0 12" "0 20" "12 12" "0 0" "16 16"; do
  set -- $spec
  VPT_GATE_NEE=$1 VPT_GATE_RAY=$2 timeout -k 10 200 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/g_$1_$2.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$O/g_$1_$2.json').read().strip().splitlines()[-1]); print('nee $1 ray $2', d['ms_per_step'])"
done
