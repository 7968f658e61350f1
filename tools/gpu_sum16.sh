#!/bin/bash
# sum_kernel 16-B table: record-format tests, then streamed A/B against the previous build
export FR_JIT_CACHE=$PWD/gpurun_out/jc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "record_formats or golden or streamed_frames or pipelined or c1_full" -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/sum16_tests.log 2>&1 || { tail -20 gpurun_out/sum16_tests.log; exit 1; }
tail -1 gpurun_out/sum16_tests.log
bash tools/gpu_knob_shards.sh fo-rma_amd/build/ab/libforma_rt_prev.so
