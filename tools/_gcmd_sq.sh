export TMPDIR=/tmp; O=gpurun_out/r01i; mkdir -p $O
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH" "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32"; do
  N=$(echo $P | cut -d' ' -f1-2 | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$N -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --spp 64 > $O/pmc_$N.log 2>&1
  rc=$?; echo "$P rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
done
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_prof.so timeout -k 10 300 python tools/tune.py --spp 64 --gates 8:8:16 --reps 1 --profile > $O/prof.log 2>&1; grep profile $O/prof.log
