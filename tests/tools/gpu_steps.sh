#!/bin/bash
# Run the GPU steps listed in a file (one command per line); continue after
# ordinary failures (exit 1/2), stop at the first timeout / abort / kill /
# segfault (exit >= 124) so nothing else touches a GPU in a bad state.
# usage: gpu_steps.sh <seconds-per-step> <logfile> <stepsfile>
per=$1; log=$2; steps=$3
while IFS= read -r c; do
  [ -z "$c" ] && continue
  case "$c" in \#*) continue;; esac
  echo "=== $c" | tee -a "$log"
  timeout -k 10 "$per" bash -c "$c" >> "$log" 2>&1
  rc=$?
  echo "=== rc=$rc" | tee -a "$log"
  if [ $rc -ge 124 ]; then echo "STOP: fatal rc=$rc" | tee -a "$log"; exit $rc; fi
done < "$steps"
exit 0
