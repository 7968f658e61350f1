#!/bin/bash
# round-3 session-2 GPU check: scene-kernel and frame-pipeline tests, C2 A/B, bench A/B
set -o pipefail
mkdir -p gpurun_out/r03e
export FR_JIT_CACHE=$PWD/gpurun_out/r03e/jitcache
O=gpurun_out/r03e
timeout -k 10 420 python -u -m pytest tests/test_scene_jit.py tests/test_gpu_parity.py -k "jit or streamed_frames or pipelined" \
  -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 240 python -u tools/ab_bench.py fo-rma_amd/libforma_rt.so fo-rma_amd/libforma_rt.so@FR_SCENE_JIT=1 \
  --reps 3 --scene scene_01 --spp 64 > $O/ab_c2.log 2>&1 || exit 1
cat $O/ab_c2.log
for i in 1 2; do
  for pipe in 0 1; do
    FR_FRAME_PIPE=$pipe timeout -k 10 200 python -u bench.py --steps 15 --warmup 2 --no-pmc --no-cpu-baseline \
      > $O/bench_pipe${pipe}_$i.json 2> $O/bench_pipe${pipe}_$i.err || exit 1
    python -c "import json;d=json.load(open('$O/bench_pipe${pipe}_$i.json'));print('pipe=$pipe', d['value'], d['ms_per_step'], d['trace_kernel_ms'], d['occupancy_wg_per_cu'], d['scene_kernel'])"
  done
done
