#!/bin/bash
# FR_FRAME_PIPE A/B at shard 0 of N (bench.py's streamed loop, tools/shard_stream.py)
mkdir -p gpurun_out/pipe_ab
export FR_JIT_CACHE=$PWD/gpurun_out/pipe_ab/jitcache
for rep in 1 2; do
  for n in 1 2 4 8; do
    for pipe in 0 1 2; do
      FR_FRAME_PIPE=$pipe timeout -k 10 120 python -u tools/shard_stream.py $n 30 || exit 1
    done
  done
done
