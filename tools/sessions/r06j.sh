#!/bin/bash
# round 6: two frames' traces in flight at half the chip each (overlapping traces with four
# workgroup slots per CU reserved): N = 1 and 2 forced to overlap, N = 4 and 8 every shard
R4="FR_FRAME_PIPE_RESERVE=4"
tools/gpu_session.sh \
 "r06j_n1_base|120|python3 tools/shard_stream.py 1 30 --warm 20" \
 "r06j_n1_ov4|120|FR_FRAME_PIPE=2 $R4 python3 tools/shard_stream.py 1 30 --warm 20" \
 "r06j_n1_ov3|120|FR_FRAME_PIPE=2 FR_FRAME_PIPE_RESERVE=3 python3 tools/shard_stream.py 1 30 --warm 20" \
 "r06j_n1_ov2|120|FR_FRAME_PIPE=2 FR_FRAME_PIPE_RESERVE=2 python3 tools/shard_stream.py 1 30 --warm 20" \
 "r06j_n2_base|120|python3 tools/shard_stream.py 2 30 --warm 20" \
 "r06j_n2_ov4|120|FR_FRAME_PIPE=2 $R4 python3 tools/shard_stream.py 2 30 --warm 20" \
 "r06j_n4_r4|120|$R4 python3 tools/shard_stream.py 4 30 --warm 20" \
 "r06j_n8_r4|120|$R4 python3 tools/shard_stream.py 8 30 --warm 20" \
 "r06j_n1_base2|120|python3 tools/shard_stream.py 1 30 --warm 20" \
 "r06j_n1_ov4b|120|FR_FRAME_PIPE=2 $R4 python3 tools/shard_stream.py 1 30 --warm 20"
