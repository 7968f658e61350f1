#!/bin/bash
# round 6: C5 counters on the final kernel; N = 8 frame-pipeline knobs on the final kernel
# (slowest shard of 8, shard 5, and shard 0), each in its own process
P5="python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 3"
B=fo-rma_amd/build/ab
S="python3 tools/shard_stream.py 8 30 --warm 20 --shards 5,0"
tools/gpu_session.sh \
 "r06h_c5sq|200|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/r06h_c5sq -o p --output-format csv -- $P5" \
 "r06h_c5sq2|200|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/r06h_c5sq2 -o p --output-format csv -- $P5" \
 "r06h_c5w|200|rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/r06h_c5w -o p --output-format csv -- $P5" \
 "r06h_c5f|200|rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/r06h_c5f -o p --output-format csv -- $P5" \
 "r06h_n8_base|120|$S" \
 "r06h_n8_res1|120|FR_FRAME_PIPE_RESERVE=1 $S" \
 "r06h_n8_res3|120|FR_FRAME_PIPE_RESERVE=3 $S" \
 "r06h_n8_slots3|120|FR_FRAME_SLOTS=3 $S" \
 "r06h_n8_serial|120|FR_FRAME_PIPE=1 $S" \
 "r06h_n8_prio1|120|FORMA_RT_LIB=$B/libforma_rt_sumprio1.so $S" \
 "r06h_n8_prio3|120|FORMA_RT_LIB=$B/libforma_rt_sumprio3.so $S" \
 "r06h_n8_base2|120|$S" \
 "r06h_n1_prio1|120|FORMA_RT_LIB=$B/libforma_rt_sumprio1.so python3 tools/shard_stream.py 1 20 --warm 20" \
 "r06h_n1_base|120|python3 tools/shard_stream.py 1 20 --warm 20"
