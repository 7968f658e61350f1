#!/bin/bash
# three-slot frame pipeline: tests, shard A/B, bench
mkdir -p gpurun_out/r03g
O=gpurun_out/r03g
export FR_JIT_CACHE=$PWD/$O/jitcache
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_scene_jit.py -k "streamed_frames or pipelined or multi_context or launch_log or prepare or pass_pipeline or c4_shards" -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for n in 1 8 1 8; do
  for pipe in 0 ""; do
    FR_FRAME_PIPE=$pipe timeout -k 10 120 python -u tools/shard_stream.py $n 30 2>/dev/null || exit 1
  done
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-pmc --no-cpu-baseline > $O/bench_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$O/bench_$i.json'));print('bench K=5', d['value'], d['ms_per_step'], d['trace_kernel_ms_per_launch'], d['trace_kernel_ms_min_max'])"
  timeout -k 10 200 python -u bench.py --no-pmc --no-cpu-baseline --steps 20 > $O/bench20_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$O/bench20_$i.json'));print('bench K=20', d['value'], d['ms_per_step'], d['trace_kernel_ms_per_launch'], d['trace_kernel_ms_min_max'])"
done
