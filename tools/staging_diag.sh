#!/bin/bash
# Diagnosis of host-span staging faults: every case in its own process, each
# under its own time limit; stops at the first case whose process dies by a
# signal or times out (a fault or hang ends the run there).
cd "$(dirname "$0")/.." || exit 2
OUT=gpurun_out/staging_diag.jsonl
: > "$OUT"
run() {
  timeout -k 5 60 python3 tests/staging_case.py "$@" >> "$OUT" 2>> gpurun_out/staging_diag.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "{\"case\": \"$*\", \"rc\": $rc}" >> "$OUT"; exit $rc; fi
}
#   nbit be nchunk ncc nsamp_df nframes stage_mib register cuts seed
for L in "8 0 1 1024 1" "16 0 1 512 1" "16 1 48 7 128" "8 0 3 100 1"; do
  for SM in 1 2; do
    for REG in 0 1; do
      set -- $L
      FB=$(( $3 * $5 * $4 * 4 * $1 / 8 ))
      NF=$(( (3 << 20) / FB )); [ $NF -lt 2 ] && NF=2
      run $L $NF $SM $REG - 7
      run $L $NF $SM $REG $(( NF / 3 )),$(( NF / 2 )) 7
    done
  done
done
echo '{"done": true}' >> "$OUT"
