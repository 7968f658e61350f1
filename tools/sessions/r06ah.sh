#!/bin/bash
# round 6, final tree: C5's counter-free kernel trace, counters and FR_SECCNT on the final
# kernel (FR_KREJ_BVH 2, the leaf records' radius^2)
B=fo-rma_amd/build/ab
P5="python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 3"
K5="python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 22"
L=$B/libforma_rt_seccnt.so
tools/gpu_session.sh \
 "r06ah_c5kt|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r06ah_c5kt -o kt --output-format csv -- $K5" \
 "r06ah_c5sq|200|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/r06ah_c5sq -o p --output-format csv -- $P5" \
 "r06ah_c5sq2|200|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/r06ah_c5sq2 -o p --output-format csv -- $P5" \
 "r06ah_c5w|200|rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/r06ah_c5w -o p --output-format csv -- $P5" \
 "r06ah_c5f|200|rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/r06ah_c5f -o p --output-format csv -- $P5" \
 "r06ah_seccnt_c5|200|FORMA_RT_LIB=$L python3 tools/seccnt_run.py gen:10000:sphere 1920 1080 512"
