#!/bin/bash
# round 6: FR_KREJ_BVH 2 as the default: the BVH parity tests, every BASELINE config and the
# bundled BVH scenes
tools/gpu_session.sh \
 "r06ag_bvh_tests|900|python3 -u -m pytest tests -m gpu -x -q -k 'bvh or far or c5' --timeout 700 --timeout-method thread" \
 "r06ag_configs|600|bash tools/time_all_configs.sh && cp gpurun_out/configs.jsonl gpurun_out/r06ag_configs.jsonl"
