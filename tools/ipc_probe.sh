#!/bin/bash
# tools/ipc_probe.sh N OUT -- N fresh processes per export variant of
# bin/ipc_probe, then N importer processes against one device ring of 6
# blocks (dada_db -g), one JSON line each into OUT, a count per variant on
# stdout.  Each process runs under its own time limit; a fault, abort or time
# limit (exit > 1) ends the script.  DESIGN.md 7b.
cd "$(dirname "$0")/.." || exit 2
N=${1:-300}
OUT=${2:-gpurun_out/ipc_probe.jsonl}
BIN=paf-baseband2power_amd/bin
: > "$OUT"
one() {
  timeout -k 5 30 "$@" >> "$OUT" 2>> "$OUT.err"
  local rc=$?
  if [ $rc -gt 1 ]; then echo "stopping: $* exit $rc"; exit $rc; fi
}
for v in first delay order nomemset; do
  for i in $(seq 1 "$N"); do
    one $BIN/ipc_probe export $v
    [ $((i % 50)) -eq 0 ] && echo "[$(date +%T)] $v $i"
  done
  python3 - "$OUT" "$v" <<'EOF'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{"variant": "%s"' % sys.argv[2])]
bad = {}
for r in rows:
    for e in r.get("exports", []):
        if e["rc"]:
            bad[e["alloc"]] = bad.get(e["alloc"], 0) + 1
print(json.dumps({"variant": sys.argv[2], "processes": len(rows), "refused": bad}), flush=True)
EOF
done
KEY=7e40
$BIN/dada_db -k $KEY -d > /dev/null 2>&1
timeout -k 5 60 $BIN/dada_db -k $KEY -b 1249952 -n 6 -g 0 || exit 3
for i in $(seq 1 "$N"); do
  timeout -k 5 30 $BIN/ipc_probe import $KEY >> "$OUT" 2>> "$OUT.err"
  rc=$?
  if [ $rc -gt 1 ]; then echo "stopping: import exit $rc"; $BIN/dada_db -k $KEY -d; exit $rc; fi
  [ $((i % 50)) -eq 0 ] && echo "[$(date +%T)] import $i"
done
# the stage and its writers open the same ring's handles at the same moment
# (the GPU tests start them together): three importers at once, N/2 times
for i in $(seq 1 $((N / 2))); do
  for j in 1 2 3; do
    timeout -k 5 30 $BIN/ipc_probe import $KEY >> "$OUT.par$j" 2>> "$OUT.err" &
  done
  wait
  [ $((i % 50)) -eq 0 ] && echo "[$(date +%T)] concurrent import $i"
done
cat "$OUT".par* >> "$OUT" && rm -f "$OUT".par*
$BIN/dada_db -k $KEY -d
python3 - "$OUT" <<'EOF'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{"import"')]
print(json.dumps({"imports": len(rows), "failed": sum(1 for r in rows if r["rc"]),
                  "why": sorted({r["why"] for r in rows if r["rc"]})}), flush=True)
EOF
