#!/bin/bash
# sum_kernel priority A/B in the pipelined bench loop
mkdir -p gpurun_out/r03h
O=gpurun_out/r03h
export FR_JIT_CACHE=$PWD/$O/jitcache
for i in 1 2; do
  for lib in fo-rma_amd/libforma_rt.so fo-rma_amd/build/ab/libforma_rt_prio0.so; do
    for k in 5 20; do
      FORMA_RT_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --no-pmc --no-cpu-baseline --steps $k > $O/b.json 2>/dev/null || exit 1
      python -c "import json;d=json.load(open('$O/b.json'));print('$(basename $lib) K=$k', d['value'], d['ms_per_step'], d['trace_kernel_ms_per_launch'], d['trace_kernel_ms_min_max'])"
    done
  done
done
for n in 8 4; do
  for lib in fo-rma_amd/libforma_rt.so fo-rma_amd/build/ab/libforma_rt_prio0.so; do
    FORMA_RT_LIB=$PWD/$lib timeout -k 10 120 python -u tools/shard_stream.py $n 30 2>/dev/null || exit 1
  done
done
