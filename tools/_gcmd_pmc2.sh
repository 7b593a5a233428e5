export TMPDIR=/tmp; O=gpurun_out/r01h; mkdir -p $O
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$N -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_$N.log 2>&1
  rc=$?; echo "$P rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
done
python3 tools/pmc_traffic.py r01 c3 256 $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/pmc_TCC_EA0_RDREQ_DRAM_sum $O/pmc_TCC_HIT_sum
cp profiles/r01_pmc.json $O/
