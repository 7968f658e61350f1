#!/bin/bash
# round 6: the BVH walk's origin-reach test as one v_max3 with |.| source modifiers: the BVH
# parity tests, then C5 against the previous commit's kernel
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06ad_bvh_tests|900|python3 -u -m pytest tests -m gpu -x -q -k 'bvh or far or c5' --timeout 700 --timeout-method thread" \
 "r06ad_ab_c5|450|python3 tools/ab_bench.py fo-rma_amd/libforma_rt.so $B/libforma_rt_head.so --reps 3 --scene gen:10000:sphere --spp 512"
