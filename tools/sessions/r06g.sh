#!/bin/bash
# round 6 measurements on the final kernels: FR_SECCNT entries and lanes (C3, C5), counter-free
# kernel traces (bench.py for C3, 22 C5 frames), C3 counters, every BASELINE config, and every
# shard of N = 1/2/4/8 streamed on one device (DESIGN.md §6's prediction)
P3="python3 tools/pmc_frame.py scene_08 1920 1080 256 8 3"
P5="python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 22"
L=fo-rma_amd/build/ab/libforma_rt_seccnt.so
tools/gpu_session.sh \
 "r06g_seccnt_c3|200|FORMA_RT_LIB=$L python3 tools/seccnt_run.py scene_08 1920 1080 256" \
 "r06g_seccnt_c5|200|FORMA_RT_LIB=$L python3 tools/seccnt_run.py gen:10000:sphere 1920 1080 512" \
 "r06g_c3kt|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r06g_c3kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc" \
 "r06g_c5kt|300|FR_SCENE_JIT=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r06g_c5kt -o kt --output-format csv -- $P5" \
 "r06g_c3sq|200|FR_SCENE_JIT=1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/r06g_c3sq -o p --output-format csv -- $P3" \
 "r06g_c3sq2|200|FR_SCENE_JIT=1 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/r06g_c3sq2 -o p --output-format csv -- $P3" \
 "r06g_c3w|200|FR_SCENE_JIT=1 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/r06g_c3w -o p --output-format csv -- $P3" \
 "r06g_c3f|200|FR_SCENE_JIT=1 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/r06g_c3f -o p --output-format csv -- $P3" \
 "r06g_configs|600|bash tools/time_all_configs.sh && cp gpurun_out/configs.jsonl gpurun_out/r06g_configs.jsonl" \
 "r06g_shards1|120|FR_SCENE_JIT=1 python3 tools/shard_stream.py 1 20 --warm 20" \
 "r06g_shards2|120|FR_SCENE_JIT=1 python3 tools/shard_stream.py 2 20 --warm 20" \
 "r06g_shards4|120|FR_SCENE_JIT=1 python3 tools/shard_stream.py 4 20 --warm 20" \
 "r06g_shards8|120|FR_SCENE_JIT=1 python3 tools/shard_stream.py 8 20 --warm 20"
