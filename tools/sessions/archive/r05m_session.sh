#!/bin/bash
# r05m: where the drop-in's host threads run -- the box's CPUs / NUMA nodes, the GPU's node, then C4 drop-in
# frames pinned to each node's granted CPUs (taskset before the program starts), 3 runs each, alternating.
set -u
O=gpurun_out/r05m; mkdir -p $O
lscpu | grep -E "^CPU\(s\)|NUMA|Socket|Model name|Thread" ; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null
python3 - <<'PY'
import os, glob
print("affinity", sorted(os.sched_getaffinity(0))[:64], len(os.sched_getaffinity(0)))
for d in sorted(glob.glob("/sys/class/drm/card*/device/numa_node")):
    print(d, open(d).read().strip())
for n in sorted(glob.glob("/sys/devices/system/node/node*/cpulist")):
    print(n, open(n).read().strip())
PY
H=tests/native/build/run_gpu_harness
run() {
  local tag=$1 cpus=$2; shift 2
  VPT_FEED_TRACE=1 VPT_DRAIN_TRACE=1 timeout -k 10 60 taskset -c $cpus $H config=volume_path_tracer_amd/scenes/fire.json \
    out=$O/film.f32 w=1920 h=1080 waves=256 grid_n=512 threads=1 batch=4096 temperature=1 warmup=1 frames=3 "$@" > $O/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc render_ms $(grep render_ms $O/$tag.log | awk '{print $3}' | tr '\n' ' ') blocked $(grep taker_blocked $O/$tag.log | awk '{print $5}' | tr '\n' ' ')"
  rm -f $O/film.f32
  [ $rc -eq 0 ] || exit $rc
}
timeout -k 10 120 python3 -c "
import torch, glob
p = torch.cuda.get_device_properties(0)
bus = '%04x:%02x:%02x' % (getattr(p, 'pci_domain_id', 0), p.pci_bus_id, p.pci_device_id)
print('gpu pci', bus, [open(d).read().strip() for d in glob.glob('/sys/bus/pci/devices/' + bus + '*/numa_node')])" || true
A=$(cat /sys/devices/system/node/node0/cpulist); B=$(cat /sys/devices/system/node/node1/cpulist)
for r in 1 2 3; do
  run node0_$r $A
  run node1_$r $B
done
