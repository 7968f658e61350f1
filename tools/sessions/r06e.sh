#!/bin/bash
# round 6: A/B of (1) the box test as fma(lo, inv, -o inv) (FR_BOX_FMA, a different image:
# measurement only) against the product kernel, bench.py's streamed loop; (2) C5 BVH kernel
# knobs: rejection-loop exit threshold and claim batching for the attenuation-class kernel
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06e_ab_boxfma|400|python3 tools/stream_ab.py --reps 4 base: boxfma:FORMA_RT_LIB=$B/libforma_rt_boxfma.so --allow-diff boxfma" \
 "r06e_ab_c5|400|python3 tools/ab_bench.py fo-rma_amd/libforma_rt.so $B/libforma_rt_krejb9.so $B/libforma_rt_krejb6.so $B/libforma_rt_claimb3.so --reps 3 --scene gen:10000:sphere --spp 512"
