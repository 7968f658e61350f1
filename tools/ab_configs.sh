#!/bin/bash
# A/B timings of the headline (shard 0 of 1/2/4/8) with an environment knob off and on:
#   tools/ab_configs.sh VAR OFF ON      e.g. tools/ab_configs.sh FR_TAIL_PRIO 0 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
var=${1:-FR_TAIL_PRIO}; off=${2:-0}; on=${3:-1}
T="timeout -k 10 120 python3 tools/time_config.py"
: > gpurun_out/ab.jsonl
for sh in 8 4 2 1; do
  for v in "$off" "$on" ${4:-}; do
    echo -n "$var=$v " >> gpurun_out/ab.jsonl
    env "$var=$v" $T scene_08 1920 1080 256 8 5 $sh >> gpurun_out/ab.jsonl || exit $?
  done
done
