#!/bin/bash
# round 6 validation of the final tree: smoke, the bench line, every shard of N = 1/2/4/8
# streamed, an N = 2 and N = 8 rehearsal through torch.distributed.run on one
# device (frame_matches_n1), the whole GPU suite
R="python3 -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
tools/gpu_session.sh \
 "r06n_smoke|200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "r06n_bench|300|python3 -u bench.py" \
 "r06n_shards1|120|python3 tools/shard_stream.py 1 20 --warm 20" \
 "r06n_shards2|120|python3 tools/shard_stream.py 2 20 --warm 20" \
 "r06n_shards4|120|python3 tools/shard_stream.py 4 20 --warm 20" \
 "r06n_shards8|120|python3 tools/shard_stream.py 8 20 --warm 20" \
 "r06n_rehearse2|300|FR_BENCH_DEVICE=0 $R --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2" \
 "r06n_rehearse8|300|FR_BENCH_DEVICE=0 $R --nproc-per-node 8 --master-port 29512 bench.py --gpus 8 --steps 10 --warmup 2" \
 "r06n_gpu_suite|900|python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
