#!/bin/bash
# camera compiled into the scene kernel (FR_JIT_CAM via FR_JIT_OPTS) against the default
export FR_JIT_CACHE=$PWD/gpurun_out/jc_cam
CAM="$(cat gpurun_out/camdef.txt)"
FR_JIT_OPTS="$CAM" timeout -k 10 120 python -u tools/jit_check.py scene_08 2>/dev/null || exit 1
for rep in 1 2 3; do
  echo -n "default "; timeout -k 10 120 python -u tools/shard_stream.py 1 30 2>/dev/null || exit 1
  echo -n "cam     "; FR_JIT_OPTS="$CAM" timeout -k 10 120 python -u tools/shard_stream.py 1 30 2>/dev/null || exit 1
done
