set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp FR_SCENE_JIT=1 FR_NO_TORCH=1
for v in cur stg8; do
  if [ $v = cur ]; then unset FORMA_RT_LIB; else export FORMA_RT_LIB=fo-rma_amd/build/ab/libforma_rt_$v.so; fi
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/pmcw_$v -o w --output-format csv -- python3 tools/pmc_frame.py scene_08 1920 1080 256 8 2 > gpurun_out/pmcw_$v.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/pmcf_$v -o f --output-format csv -- python3 tools/pmc_frame.py scene_08 1920 1080 256 8 2 > gpurun_out/pmcf_$v.log 2>&1
done
