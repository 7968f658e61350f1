#!/bin/bash
# round 6: the frame pipeline's reserve with one frame of streaming memory (default) against a
# fixed reserve of 4, interleaved; update() and N = 1 unchanged
S8="python3 tools/shard_stream.py 8 30 --warm 20 --shards 5,0"
S4="python3 tools/shard_stream.py 4 30 --warm 20 --shards 0"
S2="python3 tools/shard_stream.py 2 30 --warm 20 --shards 0"
tools/gpu_session.sh \
 "r06m_n8_a|120|$S8" "r06m_n8_f4|120|FR_FRAME_PIPE_RESERVE=4 $S8" "r06m_n8_a2|120|$S8" "r06m_n8_f4b|120|FR_FRAME_PIPE_RESERVE=4 $S8" \
 "r06m_n4_a|120|$S4" "r06m_n4_f4|120|FR_FRAME_PIPE_RESERVE=4 $S4" \
 "r06m_n2_a|120|$S2" "r06m_n2_f4|120|FR_FRAME_PIPE_RESERVE=4 $S2" \
 "r06m_n1|120|python3 tools/shard_stream.py 1 20 --warm 20" \
 "r06m_update|120|python3 tools/time_update.py"
