#!/bin/bash
# round 6 baseline: bench, counter-free kernel traces of C3 and C5, C5 PMC groups, the JIT eviction test
tools/gpu_session.sh \
 "r06a_bench|200|python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline" \
 "r06a_c3kt|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/r06a_c3kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc" \
 "r06a_c5kt|300|cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/r06a_c5kt -o kt --output-format csv -- python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 22" \
 "r06a_c5sq|200|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/r06a_c5sq -o p --output-format csv -- python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 3" \
 "r06a_c5sq2|200|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/r06a_c5sq2 -o p --output-format csv -- python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 3" \
 "r06a_c5w|200|rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/r06a_c5w -o p --output-format csv -- python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 3" \
 "r06a_c5f|200|rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/r06a_c5f -o p --output-format csv -- python3 tools/pmc_frame.py gen:10000:sphere 1920 1080 512 8 3" \
 "r06a_evict|200|python3 -u -m pytest tests/test_scene_jit.py -k eviction -x -v --timeout 150 --timeout-method thread"
