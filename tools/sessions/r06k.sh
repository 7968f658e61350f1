#!/bin/bash
# round 6: adaptive frame-pipeline reserve (4 of 8 slots for streamed overlapping traces, none
# for a frame whose predecessor has finished): every shard of N = 1/2/4/8 streamed, single
# frames of every BASELINE config, the bench line, the pipeline parity tests
tools/gpu_session.sh \
 "r06k_parity|600|python3 -u -m pytest tests/test_gpu_parity.py tests/test_scene_jit.py -k 'stream or pipelined or pass_pipeline or shard or mctx or update' -x -q --timeout 300 --timeout-method thread" \
 "r06k_shards1|120|python3 tools/shard_stream.py 1 20 --warm 20" \
 "r06k_shards2|120|python3 tools/shard_stream.py 2 20 --warm 20" \
 "r06k_shards4|120|python3 tools/shard_stream.py 4 20 --warm 20" \
 "r06k_shards8|120|python3 tools/shard_stream.py 8 20 --warm 20" \
 "r06k_configs|600|bash tools/time_all_configs.sh && cp gpurun_out/configs.jsonl gpurun_out/r06k_configs.jsonl" \
 "r06k_bench|300|python3 -u bench.py --no-cpu-baseline"
