#!/bin/bash
# round 6: re-tune the headline kernel's rejection exit threshold and claim batching after the
# fma box test (bench.py's streamed loop, interleaved)
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06p_ab_knobs|600|python3 tools/stream_ab.py --reps 3 base: krej7:FORMA_RT_LIB=$B/libforma_rt_krej7.so krej12:FORMA_RT_LIB=$B/libforma_rt_krej12.so claim2:FORMA_RT_LIB=$B/libforma_rt_claim2.so claim4:FORMA_RT_LIB=$B/libforma_rt_claim4.so"
