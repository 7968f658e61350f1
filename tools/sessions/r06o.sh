#!/bin/bash
# round 6: the class records across passes; the BVH and record-format tests again
tools/gpu_session.sh \
 "r06o_parity|600|python3 -u -m pytest tests/test_gpu_parity.py -k 'attenuation or bvh or record_formats' -x -q --timeout 300 --timeout-method thread"
