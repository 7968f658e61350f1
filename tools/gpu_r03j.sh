#!/bin/bash
# config timings (scene kernel on) after the reserve rule; C2 / C5 streamed A/B of the pipeline
export FR_JIT_CACHE=$PWD/gpurun_out/jc
FR_SCENE_JIT=1 bash tools/time_all_configs.sh && cp gpurun_out/configs.jsonl gpurun_out/r03j_configs_jit.jsonl || exit 1
