#!/bin/bash
# Run GPU steps in order: "name|seconds|command" arguments.  A step that exits 0 or 1
# (tests failed / benchmark error) lets the next one run; any other status (time
# limit 124/137, abort 134, segfault 139, GPU fault) ends the call there.
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "[steps] $name (limit ${secs}s): $cmd"
  # a line a minute while the step runs (the step's own time limit still bounds it)
  (while sleep 60; do echo "[steps] $name running $(date +%T)" >> gpurun_out/heartbeat.log; done) &
  hb=$!
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  kill $hb 2>/dev/null
  echo "[steps] $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[steps] stopping after $name (rc=$rc)"
    exit $rc
  fi
done
