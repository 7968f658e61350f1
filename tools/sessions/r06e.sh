#!/bin/bash
# round 6: A/B of (1) the box test as fma(lo, inv, -o inv) (FR_BOX_FMA, a different image:
# measurement only) against the product kernel, bench.py's streamed loop; (2) C5 BVH kernel:
# near/far child by xor (against 9acf37d), rejection-loop exit threshold, claim batching,
# 8 waves per SIMD
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06e_ab_boxfma|400|python3 tools/stream_ab.py --reps 4 base: boxfma:FORMA_RT_LIB=$B/libforma_rt_boxfma.so --allow-diff boxfma" \
 "r06e_ab_c5|400|python3 tools/ab_bench.py fo-rma_amd/libforma_rt.so $B/libforma_rt_noxor.so $B/libforma_rt_krejb9.so $B/libforma_rt_claimb3.so $B/libforma_rt_bvhw8.so --reps 3 --scene gen:10000:sphere --spp 512"
