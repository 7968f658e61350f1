#!/bin/bash
# round 6: the jitter numerator's 2^23 added at the claim (fx = 2^24 x + 2^23), so a starting
# lane's numerator is fx + px: the GPU suite, then the headline's streamed loop against the
# previous commit's kernel
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06u_gpu_tests|1000|python3 -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread" \
 "r06u_stream_ab|450|python3 tools/stream_ab.py --reps 4 new: head:FORMA_RT_LIB=$B/libforma_rt_head.so"
