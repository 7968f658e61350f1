#!/bin/bash
# round 6: C5 BVH leaf sizing by SAH termination (FR_BVH_SAH_CT: a node step's cost in leaf
# tests; FR_BVH_LEAF_CAP: largest SAH leaf) against the fixed 4-sphere leaves
L=fo-rma_amd/libforma_rt.so
tools/gpu_session.sh \
 "r06q_ab_c5_leaf|900|python3 tools/ab_bench.py $L $L@FR_BVH_SAH_CT=3 $L@FR_BVH_SAH_CT=4,FR_BVH_LEAF_CAP=8 $L@FR_BVH_SAH_CT=4 $L@FR_BVH_LEAF=8 --reps 3 --scene gen:10000:sphere --spp 512"
