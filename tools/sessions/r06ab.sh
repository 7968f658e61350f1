#!/bin/bash
# round 6: the in-order (scene-kernel) loop against a forced BVH on the final kernels, for the
# BVH's size/cost threshold (tools/bvh_threshold.sh's scenes, with FR_SCENE_JIT=1 as the bench
# runs list scenes)
tools/gpu_session.sh \
 "r06ab_bvh_threshold|600|FR_SCENE_JIT=1 bash tools/bvh_threshold.sh"
