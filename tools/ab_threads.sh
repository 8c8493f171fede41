#!/bin/bash
# workgroup width A/B for the int8 headline layouts (3 reps, 30 integrations each)
set -e
for rep in 1 2 3; do
  for t in 512 256 384 1024 128; do
    timeout -k 10 120 python3 tools/perf_matrix.py --tuning "{\"max_threads\": $t}" --steps 30 --only "int8 256ch" --npol-out 1 >> gpurun_out/abt.log 2>&1
    timeout -k 10 120 python3 tools/perf_matrix.py --tuning "{\"max_threads\": $t}" --steps 10 --only "int8 1024ch" --npol-out 1 >> gpurun_out/abt.log 2>&1
  done
done
