#!/bin/bash
# round 6, final tree: the whole GPU suite, then the headline kernel's rejection exit threshold
# and claim batching re-tuned after the sample-start changes (bench.py's streamed loop)
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06aa_gpu_suite|1000|python3 -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread" \
 "r06aa_ab_knobs|600|python3 tools/stream_ab.py --reps 3 base: krej7:FORMA_RT_LIB=$B/libforma_rt_krej7.so krej12:FORMA_RT_LIB=$B/libforma_rt_krej12.so claim2:FORMA_RT_LIB=$B/libforma_rt_claim2.so claim4:FORMA_RT_LIB=$B/libforma_rt_claim4.so"
