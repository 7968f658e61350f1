#!/bin/bash
# round 6, final kernels: every BASELINE config, every shard of N = 1/2/4/8 streamed on one
# device (DESIGN.md §6's prediction), N = 2 and N = 8 rehearsals through torch.distributed.run
# on one device (frame_matches_n1)
R="python3 -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
tools/gpu_session.sh \
 "r06x_configs|600|bash tools/time_all_configs.sh && cp gpurun_out/configs.jsonl gpurun_out/r06x_configs.jsonl" \
 "r06x_shards1|120|python3 tools/shard_stream.py 1 20 --warm 20" \
 "r06x_shards2|120|python3 tools/shard_stream.py 2 20 --warm 20" \
 "r06x_shards4|120|python3 tools/shard_stream.py 4 20 --warm 20" \
 "r06x_shards8|120|python3 tools/shard_stream.py 8 20 --warm 20" \
 "r06x_rehearse2|300|FR_BENCH_DEVICE=0 $R --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2" \
 "r06x_rehearse8|300|FR_BENCH_DEVICE=0 $R --nproc-per-node 8 --master-port 29512 bench.py --gpus 8 --steps 10 --warmup 2"
