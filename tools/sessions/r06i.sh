#!/bin/bash
# round 6: C5 octant-coherent node step (FR_BVH_OCTANT) A/B; the frame pipeline's reserve for
# overlapping shard traces at N = 4 and 8 (FR_FRAME_PIPE_RESERVE 2 default, 3, 4, 5)
B=fo-rma_amd/build/ab
S8="python3 tools/shard_stream.py 8 30 --warm 20 --shards 5,0"
S4="python3 tools/shard_stream.py 4 30 --warm 20 --shards 0,1"
tools/gpu_session.sh \
 "r06i_ab_oct|400|python3 tools/ab_bench.py fo-rma_amd/libforma_rt.so $B/libforma_rt_nooct.so --reps 4 --scene gen:10000:sphere --spp 512" \
 "r06i_n8_res2|120|$S8" "r06i_n8_res3|120|FR_FRAME_PIPE_RESERVE=3 $S8" "r06i_n8_res4|120|FR_FRAME_PIPE_RESERVE=4 $S8" \
 "r06i_n8_res5|120|FR_FRAME_PIPE_RESERVE=5 $S8" "r06i_n8_res2b|120|$S8" "r06i_n8_res3b|120|FR_FRAME_PIPE_RESERVE=3 $S8" \
 "r06i_n4_res2|120|$S4" "r06i_n4_res3|120|FR_FRAME_PIPE_RESERVE=3 $S4" "r06i_n4_res4|120|FR_FRAME_PIPE_RESERVE=4 $S4"
