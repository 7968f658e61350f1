#!/bin/bash
# Run a sequence of GPU steps on the gpurun box. Each step has its own time limit.
# A plain failure (exit 1, e.g. a failing assertion) is recorded and the next step
# runs; a fault, abort, kill or time-out (exit >= 124) ends the session at once.
# usage: tools/gpu_session.sh "<name>|<seconds>|<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
status=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] $(date +%T) limit ${secs}s: $cmd"
  # a progress line a minute while the step runs (a long parity test prints nothing until
  # it ends); the step's own time limit still bounds it
  ( while sleep 60; do echo "... [$name] $(date +%T) running" >> gpurun_out/heartbeat.log; done ) &
  hb=$!
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  kill "$hb" 2>/dev/null; wait "$hb" 2>/dev/null
  echo "=== [$name] rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then
    echo "=== stopping: step $name ended with $rc (fault/abort/timeout)"
    exit $rc
  fi
  [ $rc -ne 0 ] && status=1
done
exit $status
