#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; stop at the first step that faults, aborts,
# times out or segfaults (exit codes other than 0 = pass and 1 = test failures).
# usage: tools/gpu_run.sh "<timeout_s> <name> <command...>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  t=$(echo "$spec" | awk '{print $1}'); name=$(echo "$spec" | awk '{print $2}'); cmd=$(echo "$spec" | cut -d' ' -f3-)
  echo "=== $name (timeout $t): $cmd"
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
done
