#!/bin/bash
# PMC passes over the ragged workload (k_entries_varlen): instructions, clock,
# stall split; each counter set its own rocprofv3 run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmcrag"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"
i=0
for ctrs in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$OUT/r$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench_workloads.py" --workload ragged --steps 3 --warmup 1 --no-check ${RAG_ARGS} > "$OUT/r$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/r$i.log"; exit 1; }
done
python3 "$GRAFT_REPO_ROOT/tools/pmc_table.py" k_entries_varlen $(find "$OUT" -name "*counter_collection.csv")
