#!/bin/bash
# round 6: postponed leaves in the BVH walk (FR_BVH_POSTPONE, measured then removed): the GPU suite, then C5
# against the walk without them (a build of the same tree with FR_BVH_POSTPONE=0)
B=fo-rma_amd/build/ab
tools/gpu_session.sh \
 "r06r_gpu_tests|1100|python3 -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread" \
 "r06r_ab_c5_postpone|700|python3 tools/ab_bench.py fo-rma_amd/libforma_rt.so $B/libforma_rt_nopp.so fo-rma_amd/libforma_rt.so@FR_BVH_LEAF=2 --reps 3 --scene gen:10000:sphere --spp 512"
