set -e
for rep in 1 2 3; do
  for il in 0 1; do
    for npo in 1 2; do
      timeout -k 10 120 python3 tools/perf_matrix.py --tuning "{\"interleave\": $il}" --steps 30 --only "int8 256ch" --npol-out $npo >> gpurun_out/ab.log 2>&1
      timeout -k 10 120 python3 tools/perf_matrix.py --tuning "{\"interleave\": $il}" --steps 10 --only "int8 1024ch" --npol-out $npo >> gpurun_out/ab.log 2>&1
    done
  done
done
