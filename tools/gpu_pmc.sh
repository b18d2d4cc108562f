#!/bin/bash
# Counter passes for the dominant kernel (separate rocprofv3 runs, each with
# --kernel-trace only beside --pmc; never combined with sys/runtime traces).
# PMC_CMD overrides the profiled python command (script path + args).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="${PMC_CMD:-$GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --prewarm 0 --no-cpu-baseline ${BENCH_ARGS}}"
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
            "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$OUT/p$i" -o run -- python3 $B > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
# summaries on the box (the raw per-dispatch CSVs of five passes exceed what
# gpurun copies back): the PMC table and the HBM traffic per launch
python3 "$GRAFT_REPO_ROOT/tools/pmc_table.py" "${PMC_MATCH:-k_entries_fixed}" $(find "$OUT" -name "*counter_collection.csv") > "$OUT/table.txt"
python3 "$GRAFT_REPO_ROOT/tools/traffic_json.py" "$OUT" "${PMC_MATCH:-k_entries_fixed}" "${PMC_LABEL:-bench.py C2 leaf launch}" "${PMC_ALG:-1140850688}" > "$OUT/traffic.json"
cat "$OUT/traffic.json"
rm -rf "$OUT"/p[0-9]*
