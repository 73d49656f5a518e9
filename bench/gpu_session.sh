#!/bin/bash
# Run GPU steps in order; a test failure (exit 1) continues, anything else (fault, abort,
# timeout, signal) stops the session.  usage: bash bench/gpu_session.sh 'name|secs|cmd' ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "[session] $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[session] $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[session] stopping after $name (rc=$rc)"
    exit $rc
  fi
done
