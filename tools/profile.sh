#!/bin/bash
# rocprofv3 collection for the bench workload (run on the GPU box via gpurun), or for
# PROF_CMD (a python3 command line, e.g. "python3 tools/time_config.py scene_04 1920 1080 64 8 1").
# Kernel trace + stats in one run; each PMC group in its own run (never combined
# with sys/runtime traces). Output under gpurun_out/prof/<tag>/.
tag="${1:-r01}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out="gpurun_out/prof/$tag"
mkdir -p "$out"
B="${PROF_CMD:-python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pmc}"
run() {  # name seconds args...
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" rocprofv3 "$@" -d "$out/$name" -o "$name" --output-format csv -- $B > "$out/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$out/$name.log"
  echo "rc=$rc"
  [ $rc -ge 124 ] && exit $rc
  return 0
}
run trace 300 --kernel-trace --stats
run pmc_fetch 300 --pmc FETCH_SIZE
run pmc_write 300 --pmc WRITE_SIZE
run pmc_sq 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU
run pmc_sq2 300 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE
exit 0
