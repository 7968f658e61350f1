#!/bin/bash
# three frame slots: the trace grid's reserved CU slot (1) against none (0), streamed N = 1
export FR_JIT_CACHE=$PWD/gpurun_out/jc
for rep in 1 2 3; do
  for r in 1 0; do
    echo -n "reserve $r "; FR_FRAME_PIPE_RESERVE=$r timeout -k 10 120 python -u tools/shard_stream.py 1 30 2>/dev/null || exit 1
  done
done
