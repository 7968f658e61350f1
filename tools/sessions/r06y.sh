#!/bin/bash
# round 6: the BVH node step's outcome applied after its scalar or vector path (no register
# copy at the loop latch), and a scene-kernel slab plane at 0 as -o inv: the GPU suite, then
# the headline's streamed loop and C5 against the previous commit's kernels
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06y_gpu_tests|1000|python3 -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread" \
 "r06y_stream_ab|450|python3 tools/stream_ab.py --reps 4 new: head:FORMA_RT_LIB=$B/libforma_rt_head.so" \
 "r06y_ab_c5|450|python3 tools/ab_bench.py fo-rma_amd/libforma_rt.so $B/libforma_rt_head.so --reps 3 --scene gen:10000:sphere --spp 512"
