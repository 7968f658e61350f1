#!/bin/bash
# round 6 measurements on the final kernels (after the node-step tail and the zero planes):
# the lens pre-scale test, smoke, the bench line, counter-free kernel traces (bench.py for C3,
# 22 C5 frames), C3 and C5 counters, FR_SECCNT entries and lanes, every BASELINE config, every
# shard of N = 1/2/4/8 streamed on one device, N = 2 and 8 rehearsals (frame_matches_n1)
P3="python3 tools/pmc_frame.py scene_08 1920 1080 256 8 3"
P5="python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 3"
K5="python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 22"
L=fo-rma_amd/build/ab/libforma_rt_seccnt.so
R="python3 -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
tools/gpu_session.sh \
 "r06z_lens_test|300|python3 -u -m pytest tests/test_gpu_parity.py -x -q -k lens_radius --timeout 200 --timeout-method thread" \
 "r06z_smoke|200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "r06z_bench|300|python3 -u bench.py" \
 "r06z_c3kt|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r06z_c3kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc" \
 "r06z_c5kt|300|FR_SCENE_JIT=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r06z_c5kt -o kt --output-format csv -- $K5" \
 "r06z_c3sq|200|FR_SCENE_JIT=1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/r06z_c3sq -o p --output-format csv -- $P3" \
 "r06z_c3sq2|200|FR_SCENE_JIT=1 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/r06z_c3sq2 -o p --output-format csv -- $P3" \
 "r06z_c3w|200|FR_SCENE_JIT=1 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/r06z_c3w -o p --output-format csv -- $P3" \
 "r06z_c3f|200|FR_SCENE_JIT=1 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/r06z_c3f -o p --output-format csv -- $P3" \
 "r06z_c5sq|200|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/r06z_c5sq -o p --output-format csv -- $P5" \
 "r06z_c5sq2|200|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/r06z_c5sq2 -o p --output-format csv -- $P5" \
 "r06z_c5w|200|rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/r06z_c5w -o p --output-format csv -- $P5" \
 "r06z_c5f|200|rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/r06z_c5f -o p --output-format csv -- $P5" \
 "r06z_seccnt_c3|200|FORMA_RT_LIB=$L python3 tools/seccnt_run.py scene_08 1920 1080 256" \
 "r06z_seccnt_c5|200|FORMA_RT_LIB=$L python3 tools/seccnt_run.py gen:10000:sphere 1920 1080 512" \
 "r06z_configs|600|bash tools/time_all_configs.sh && cp gpurun_out/configs.jsonl gpurun_out/r06z_configs.jsonl" \
 "r06z_shards1|120|python3 tools/shard_stream.py 1 20 --warm 20" \
 "r06z_shards2|120|python3 tools/shard_stream.py 2 20 --warm 20" \
 "r06z_shards4|120|python3 tools/shard_stream.py 4 20 --warm 20" \
 "r06z_shards8|120|python3 tools/shard_stream.py 8 20 --warm 20" \
 "r06z_rehearse2|300|FR_BENCH_DEVICE=0 $R --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2" \
 "r06z_rehearse8|300|FR_BENCH_DEVICE=0 $R --nproc-per-node 8 --master-port 29512 bench.py --gpus 8 --steps 10 --warmup 2"
