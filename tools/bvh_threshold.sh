#!/bin/bash
# In-order loop vs forced BVH per scene (tools/time_config.py), for the kBvhMinCost choice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for cfg in "scene_01 1920 1080 64 8" "scene_04 1920 1080 64 8" "scene_05 1920 1080 64 8" \
           "gen:50:sphere 1920 1080 32 8" "gen:100:sphere 1920 1080 32 8" "gen:200:sphere 1920 1080 32 8" \
           "gen:50:cube 1920 1080 32 8" "gen:100:cube 1920 1080 32 8" "gen:200:cube 1920 1080 32 8" \
           "gen:400:cube 1920 1080 32 8"; do
  for bv in 0 1; do
    FR_BVH=$bv timeout -k 5 120 python tools/time_config.py $cfg 2 | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['scene'], 'FR_BVH=$bv', round(d['kernel_ms_median'],2), 'ms', round(d['segments']/d['samples'],2), 'seg/sample', flush=True)" || exit $?
  done
done
