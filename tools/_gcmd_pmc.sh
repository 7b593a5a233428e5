export TMPDIR=/tmp; O=gpurun_out/r01c; mkdir -p $O
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
grep -oE "^\s*(SQ|TCC|TCP|TA|GRBM)_[A-Z0-9_]+" $O/counters_list.txt | sort -u > $O/counter_names.txt || true
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$N -o run -- python3 tools/tune.py --spp 8 --gates 8:8 --reps 1 > $O/pmc_$N.log 2>&1
  rc=$?; echo "$P rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
done
