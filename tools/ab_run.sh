set -e
for r in 1 2; do
 for v in new old; do
  for inf in 1 3; do
   if [ $v = old ]; then export MH_LIB_PATH=$PWD/build/ab/libold.so; else unset MH_LIB_PATH; fi
   echo "variant=$v inflight=$inf" >> gpurun_out/ab1.log
   timeout -k 10 120 python bench.py --inflight $inf --no-cpu-baseline --steps 40 >> gpurun_out/ab1.log 2>&1
  done
 done
done
unset MH_LIB_PATH
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "random_widths or wg_levels or c2_full or concurrent or reduce_nodes" > gpurun_out/ab1_tests.log 2>&1
