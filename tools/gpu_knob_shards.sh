#!/bin/bash
# a build variant against the default at shard 0 of 1 and of 8 (bench.py's streamed loop)
export FR_JIT_CACHE=$PWD/gpurun_out/jc_ab
for rep in 1 2 3; do
  for n in 1 8; do
    for lib in fo-rma_amd/libforma_rt.so "$@"; do
      echo -n "$(basename $lib) "
      FORMA_RT_LIB=$PWD/$lib timeout -k 10 120 python -u tools/shard_stream.py $n 30 2>/dev/null || exit 1
    done
  done
done
