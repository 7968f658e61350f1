#!/bin/bash
# round 6: the BVH leaf records carry RN(radius^2) in place of a sphere's radius: the GPU
# suite, then C5 against the previous commit's kernel
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06ac_gpu_suite|1000|python3 -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread" \
 "r06ac_ab_c5|450|python3 tools/ab_bench.py fo-rma_amd/libforma_rt.so $B/libforma_rt_head.so --reps 3 --scene gen:10000:sphere --spp 512"
