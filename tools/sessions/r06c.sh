#!/bin/bash
# round 6: BVH kernels with 8-B attenuation-class records (C5): parity, timing against the
# unwinding kernel (FR_DEFER=0), FR_SECCNT region entries for the phase model, counters
P="python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 3"
tools/gpu_session.sh \
 "r06c_parity|600|python3 -u -m pytest tests/test_gpu_parity.py -k 'bvh or c5 or record_formats or attenuation' -x -q --timeout 300 --timeout-method thread" \
 "r06c_time_c5_new|200|python3 tools/time_config.py gen:10000:sphere 1920 1080 512 8 5" \
 "r06c_time_c5_old|200|FR_DEFER=0 python3 tools/time_config.py gen:10000:sphere 1920 1080 512 8 5" \
 "r06c_time_c5_new2|200|python3 tools/time_config.py gen:10000:sphere 1920 1080 512 8 5" \
 "r06c_time_c5_old2|200|FR_DEFER=0 python3 tools/time_config.py gen:10000:sphere 1920 1080 512 8 5" \
 "r06c_seccnt_c5|200|FORMA_RT_LIB=fo-rma_amd/build/ab/libforma_rt_seccnt.so python3 tools/seccnt_run.py gen:10000:sphere 1920 1080 512" \
 "r06c_seccnt_c5old|200|FR_DEFER=0 FORMA_RT_LIB=fo-rma_amd/build/ab/libforma_rt_seccnt.so python3 tools/seccnt_run.py gen:10000:sphere 1920 1080 512" \
 "r06c_seccnt_c3|200|FORMA_RT_LIB=fo-rma_amd/build/ab/libforma_rt_seccnt.so python3 tools/seccnt_run.py scene_08 1920 1080 256" \
 "r06c_c5sq|200|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/r06c_c5sq -o p --output-format csv -- $P" \
 "r06c_c5sq2|200|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/r06c_c5sq2 -o p --output-format csv -- $P" \
 "r06c_c5w|200|rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/r06c_c5w -o p --output-format csv -- $P"
