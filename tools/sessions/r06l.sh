#!/bin/bash
# round 6: adaptive reserve (default) against a fixed reserve of 4, interleaved
S8="python3 tools/shard_stream.py 8 30 --warm 20 --shards 5,0"
S4="python3 tools/shard_stream.py 4 30 --warm 20 --shards 0"
S2="python3 tools/shard_stream.py 2 30 --warm 20 --shards 0"
tools/gpu_session.sh \
 "r06l_n8_a|120|$S8" "r06l_n8_f4|120|FR_FRAME_PIPE_RESERVE=4 $S8" "r06l_n8_a2|120|$S8" "r06l_n8_f4b|120|FR_FRAME_PIPE_RESERVE=4 $S8" \
 "r06l_n4_a|120|$S4" "r06l_n4_f4|120|FR_FRAME_PIPE_RESERVE=4 $S4" \
 "r06l_n2_a|120|$S2" "r06l_n2_f4|120|FR_FRAME_PIPE_RESERVE=4 $S2"
