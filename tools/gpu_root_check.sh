mkdir -p gpurun_out && timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_concurrency.py tests/test_gpu_multi.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1; tail -3 gpurun_out/pt.log; timeout -k 10 200 python bench.py --steps 2000 --no-cpu-baseline > gpurun_out/b3.json && timeout -k 10 200 python bench.py --steps 1000 --inflight 1 --no-cpu-baseline > gpurun_out/b1.json && python -c "
import json
for f in ['gpurun_out/b3.json','gpurun_out/b1.json']:
    d=json.load(open(f)); print(f, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['reduce_ms_per_build'], d['single_build'])
"
