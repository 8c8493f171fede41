#!/bin/bash
# every 5 s, the state and kernel wait channel of this job's python, stage and
# DADA processes, appended to $1 (a diagnostic beside a GPU run that may hang)
while true; do
  { date +%T; ps -eo pid,ppid,stat,wchan:32,etime,args | awk 'NR==1 || /python|paf_|dada_db/' | grep -v awk || true; } >> "$1"
  sleep 5
done
