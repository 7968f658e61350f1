#!/bin/bash
# serial vs overlapping traces at N = 1, 2, 4 (three frame slots)
export FR_JIT_CACHE=$PWD/gpurun_out/jc
for rep in 1 2; do
  for n in 1 2 4; do
    echo -n "N$n serial "; FR_FRAME_PIPE=1 timeout -k 10 120 python -u tools/shard_stream.py $n 30 2>/dev/null || exit 1
    echo -n "N$n overlap "; FR_FRAME_PIPE=2 timeout -k 10 120 python -u tools/shard_stream.py $n 30 2>/dev/null || exit 1
  done
done
