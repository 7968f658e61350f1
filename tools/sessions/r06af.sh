#!/bin/bash
# round 6: C5's rejection exit threshold (FR_KREJ_BVH) below the shared default of 4
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06af_ab_c5_krej|900|python3 tools/ab_bench.py fo-rma_amd/libforma_rt.so $B/libforma_rt_krejb0.so $B/libforma_rt_krejb1.so $B/libforma_rt_krejb2.so $B/libforma_rt_krejb3.so --reps 4 --scene gen:10000:sphere --spp 512"
