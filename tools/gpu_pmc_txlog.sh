#!/bin/bash
# PMC passes over the fused a14 group kernel (bench_workloads --workload txlog):
# stall split, instruction mix, HBM bytes; each counter set its own run.
# PMC_PY overrides the profiled script + args (e.g. "tools/txlog_resident.py 65536 5").
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmctx${PMC_TAG:-}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
P5="${PMC_EXTRA:-}"
for ctrs in "$P1" "$P2" "$P3" "$P4" ${P5:+"$P5"}; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$OUT/b$i" -o run -- python3 "$GRAFT_REPO_ROOT/"${PMC_PY:-bench_workloads.py --workload txlog --steps 3 --warmup 1 --prewarm 0} > "$OUT/b$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/b$i.log"; exit 1; }
done
python3 "$GRAFT_REPO_ROOT/tools/pmc_table.py" "${PMC_MATCH:-k_txlog_wave}" $(find "$OUT" -name "*counter_collection.csv") > "$OUT/table.txt"
