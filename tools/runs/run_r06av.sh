#!/bin/bash
set -o pipefail
# Round 6, pass av: does the calling thread's CPU (near / far from the GPU's NUMA node) move the
# 8-byte Reduce_local? (r06au: 5.28 and 5.80 us in two runs on one box)
O=gpurun_out/r06av
mkdir -p $O
node=$(cat /sys/class/drm/card*/device/numa_node 2>/dev/null | head -1)
echo "gpu numa node: $node; cpus allowed: $(grep Cpus_allowed_list /proc/self/status)"
for n in /sys/devices/system/node/node[0-9]*; do echo "$(basename $n): $(cat $n/cpulist)"; done
near=$(cat /sys/devices/system/node/node${node:-0}/cpulist | cut -d, -f1 | cut -d- -f1)
for nn in /sys/devices/system/node/node[0-9]*; do id=${nn##*node}; if [ "$id" != "${node:-0}" ]; then far=$(cut -d, -f1 $nn/cpulist | cut -d- -f1); break; fi; done
echo "near cpu $near far cpu $far"
for k in 1 2 3; do
  for c in $near $far; do
    echo "cpu $c: $(timeout -k 10 60 taskset -c $c tools/diag/rl_lat lib 5000 | grep 'C loop' | cut -c1-120)"
  done
done
for k in 1 2 3; do echo "unbound: $(timeout -k 10 60 tools/diag/rl_lat lib 5000 | grep 'C loop' | cut -c1-120)"; done
