#!/bin/bash
# Host placement probe (round 6): the box's NUMA layout, this process's CPU
# set, the GPU's NUMA node, and the a14 C-ABI median (tools/txlog_bench) with
# the process pinned to the allowed CPUs of each NUMA node in turn.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-numa}
mkdir -p "$O"
{
  lscpu | grep -i "numa\|socket\|^CPU(s)"
  grep Cpus_allowed_list /proc/self/status
  for d in /sys/bus/pci/drivers/amdgpu/0000:*; do
    [ -e "$d/numa_node" ] && echo "gpu $(basename $d) numa_node $(cat $d/numa_node) local_cpulist $(cat $d/local_cpulist 2>/dev/null)"
  done
} | tee "$O/numa.txt"
allowed=$(grep Cpus_allowed_list /proc/self/status | awk '{print $2}')
python3 - "$allowed" > "$O/sets.txt" <<'PY'
import sys, glob, os
def parse(s):
    out = set()
    for part in s.split(','):
        if '-' in part:
            a, b = part.split('-'); out |= set(range(int(a), int(b) + 1))
        elif part:
            out.add(int(part))
    return out
allowed = parse(sys.argv[1])
for n in sorted(glob.glob('/sys/devices/system/node/node[0-9]*')):
    cpus = parse(open(n + '/cpulist').read().strip()) & allowed
    if cpus:
        print(os.path.basename(n), ','.join(str(c) for c in sorted(cpus)))
PY
cat "$O/sets.txt"
for r in 1 2; do
  while read node cpus; do
    line=$(timeout -k 10 120 taskset -c "$cpus" ./tools/txlog_bench 200 | tail -1) || exit 1
    echo "round $r $node cpus $cpus $line" | tee -a "$O/numa.txt"
  done < "$O/sets.txt"
  line=$(timeout -k 10 120 ./tools/txlog_bench 200 | tail -1) || exit 1
  echo "round $r unpinned $line" | tee -a "$O/numa.txt"
done
