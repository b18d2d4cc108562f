#!/bin/bash
# After a change of the leaf-kernel defaults: htree parity suites, then C2
# (default and the driver's 20-step command), single build and C4 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_concurrency.py tests/test_gpu_multi.py tests/test_gpu_sharded.py tests/test_gpu_c_client.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -2 gpurun_out/pt.log
timeout -k 10 200 python bench.py > gpurun_out/c2.json 2> gpurun_out/c2.err || exit 1
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c2_20.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/c4.json 2>/dev/null || exit 1
for f in c2 c2_20 c4; do python -c "
import json;d=json.load(open('gpurun_out/$f.json'));r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['sha']['frac'], r['sha']['step']['frac'], d['single_build'])"; done
