#!/bin/bash
# overlapping traces (small shards): reserve 1 vs 0; N = 4 serial vs overlapping
export FR_JIT_CACHE=$PWD/gpurun_out/jc
for rep in 1 2; do
  echo -n "N8 auto r1 "; timeout -k 10 120 python -u tools/shard_stream.py 8 40 2>/dev/null || exit 1
  echo -n "N8 auto r0 "; FR_FRAME_PIPE_RESERVE=0 timeout -k 10 120 python -u tools/shard_stream.py 8 40 2>/dev/null || exit 1
  echo -n "N4 auto r1 "; timeout -k 10 120 python -u tools/shard_stream.py 4 40 2>/dev/null || exit 1
  echo -n "N4 ovl  r1 "; FR_FRAME_PIPE=2 timeout -k 10 120 python -u tools/shard_stream.py 4 40 2>/dev/null || exit 1
  echo -n "N4 ovl  r0 "; FR_FRAME_PIPE=2 FR_FRAME_PIPE_RESERVE=0 timeout -k 10 120 python -u tools/shard_stream.py 4 40 2>/dev/null || exit 1
done
