#!/bin/bash
# Effective clock and stall split of the leaf kernel vs the register-only SHA
# microbenchmark: GRBM_GUI_ACTIVE / 8 / duration, SQ_ACTIVE_INST_VALU,
# SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_WAVE_CYCLES (each pass its own run).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmcclk"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"
i=0
for ctrs in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$OUT/b$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --inflight 1 --no-cpu-baseline > "$OUT/b$i.log" 2>&1 || { echo "bench pass $i failed"; tail -5 "$OUT/b$i.log"; exit 1; }
  if [ -x "$GRAFT_REPO_ROOT/tools/microbench_sha" ]; then
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$OUT/m$i" -o run -- "$GRAFT_REPO_ROOT/tools/microbench_sha" > "$OUT/m$i.log" 2>&1 || { echo "micro pass $i failed"; tail -5 "$OUT/m$i.log"; exit 1; }
  fi
done
find "$OUT" -name "*.csv" | head
