#!/bin/bash
# round 6: the BVH traversal stack addressed by LDS byte address, with a sentinel row of
# kBvhEnd below level 0 (a pop needs no empty test): the GPU suite, then C5 against the
# previous commit's kernel
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06v_gpu_tests|1000|python3 -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread" \
 "r06v_ab_c5|450|python3 tools/ab_bench.py fo-rma_amd/libforma_rt.so $B/libforma_rt_head.so --reps 3 --scene gen:10000:sphere --spp 512"
