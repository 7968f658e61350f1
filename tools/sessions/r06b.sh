#!/bin/bash
# round 6: FR_SECCNT region entries and active lanes for C5 (BVH) and C3 (scene kernel)
tools/gpu_session.sh \
 "r06b_seccnt_c5|200|FORMA_RT_LIB=fo-rma_amd/build/ab/libforma_rt_seccnt.so python3 tools/seccnt_run.py gen:10000:sphere 1920 1080 512" \
 "r06b_seccnt_c3|200|FORMA_RT_LIB=fo-rma_amd/build/ab/libforma_rt_seccnt.so python3 tools/seccnt_run.py scene_08 1920 1080 256"
