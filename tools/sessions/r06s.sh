#!/bin/bash
# round 6: a sample's jitter draws merged into its first lens try (every lane draws three at
# full width; a camera lane draws the fourth in its branch): the GPU suite, then the headline's
# streamed loop and C5 against the previous commit's kernels
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06s_gpu_tests|1100|python3 -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread" \
 "r06s_stream_ab|600|python3 tools/stream_ab.py --reps 4 new: head:FORMA_RT_LIB=$B/libforma_rt_head.so" \
 "r06s_ab_c5|600|python3 tools/ab_bench.py fo-rma_amd/libforma_rt.so $B/libforma_rt_head.so --reps 3 --scene gen:10000:sphere --spp 512"
