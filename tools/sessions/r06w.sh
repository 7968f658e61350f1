#!/bin/bash
# round 6 measurements on the final kernels (after the jitter merge, the folded scales and the
# BVH stack sentinel): smoke, the bench line, counter-free kernel traces (bench.py for C3, 22
# C5 frames), C3 and C5 counters, FR_SECCNT entries and lanes
P3="python3 tools/pmc_frame.py scene_08 1920 1080 256 8 3"
P5="python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 3"
K5="python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 22"
L=fo-rma_amd/build/ab/libforma_rt_seccnt.so
tools/gpu_session.sh \
 "r06w_smoke|200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "r06w_bench|300|python3 -u bench.py" \
 "r06w_c3kt|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r06w_c3kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc" \
 "r06w_c5kt|300|FR_SCENE_JIT=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r06w_c5kt -o kt --output-format csv -- $K5" \
 "r06w_c3sq|200|FR_SCENE_JIT=1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/r06w_c3sq -o p --output-format csv -- $P3" \
 "r06w_c3sq2|200|FR_SCENE_JIT=1 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/r06w_c3sq2 -o p --output-format csv -- $P3" \
 "r06w_c3w|200|FR_SCENE_JIT=1 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/r06w_c3w -o p --output-format csv -- $P3" \
 "r06w_c3f|200|FR_SCENE_JIT=1 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/r06w_c3f -o p --output-format csv -- $P3" \
 "r06w_c5sq|200|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/r06w_c5sq -o p --output-format csv -- $P5" \
 "r06w_c5sq2|200|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/r06w_c5sq2 -o p --output-format csv -- $P5" \
 "r06w_c5w|200|rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/r06w_c5w -o p --output-format csv -- $P5" \
 "r06w_c5f|200|rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/r06w_c5f -o p --output-format csv -- $P5" \
 "r06w_seccnt_c3|200|FORMA_RT_LIB=$L python3 tools/seccnt_run.py scene_08 1920 1080 256" \
 "r06w_seccnt_c5|200|FORMA_RT_LIB=$L python3 tools/seccnt_run.py gen:10000:sphere 1920 1080 512"
