set -e
for rep in 1 2; do
  for u in 4 104 102 8; do
    B2P_UNROLL=$u timeout -k 10 120 python3 tools/perf_matrix.py --steps 30 --only "int8 256ch" --npol-out 1 >> gpurun_out/abp.log 2>&1
    B2P_UNROLL=$u timeout -k 10 120 python3 tools/perf_matrix.py --steps 20 --only "BMF" --npol-out 1 >> gpurun_out/abp.log 2>&1
  done
done
