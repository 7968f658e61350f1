#!/bin/bash
# round 6: C5 with attenuation-class records after the unrolled-list fix: timing against the
# unwinding kernel (FR_DEFER=0), parity, FR_SECCNT entries, counters
P="python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 3"
T="python3 tools/time_config.py gen:10000:sphere 1920 1080 512 8 5"
tools/gpu_session.sh \
 "r06d_time_new|120|$T" "r06d_time_old|120|FR_DEFER=0 $T" "r06d_time_new2|120|$T" "r06d_time_old2|120|FR_DEFER=0 $T" \
 "r06d_seccnt_c5|200|FORMA_RT_LIB=fo-rma_amd/build/ab/libforma_rt_seccnt.so python3 tools/seccnt_run.py gen:10000:sphere 1920 1080 512" \
 "r06d_c5sq|200|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/r06d_c5sq -o p --output-format csv -- $P" \
 "r06d_c5sq2|200|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/r06d_c5sq2 -o p --output-format csv -- $P" \
 "r06d_c5w|200|rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/r06d_c5w -o p --output-format csv -- $P" \
 "r06d_parity|600|python3 -u -m pytest tests/test_gpu_parity.py -k 'bvh or record_formats or attenuation' -x -q --timeout 300 --timeout-method thread" \
 "r06d_parity_c5|700|python3 -u -m pytest tests/test_gpu_parity.py -k 'c5_generator' -x -q --timeout 650 --timeout-method thread"
