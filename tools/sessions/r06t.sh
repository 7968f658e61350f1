#!/bin/bash
# round 6: the lens sample's 2^-23 scale folded into a pre-scaled lens radius, the scatter's
# into one fma per coordinate: the GPU suite, then the headline's streamed loop and C5 against
# the previous commit's kernels
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06t_gpu_tests|1000|python3 -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread" \
 "r06t_stream_ab|450|python3 tools/stream_ab.py --reps 4 new: head:FORMA_RT_LIB=$B/libforma_rt_head.so" \
 "r06t_ab_c5|450|python3 tools/ab_bench.py fo-rma_amd/libforma_rt.so $B/libforma_rt_head.so --reps 3 --scene gen:10000:sphere --spp 512"
