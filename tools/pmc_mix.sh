#!/bin/bash
# Instruction mix, LDS and scalar-cache counters of one workload, one rocprofv3 PMC pass
# per group (each with at most 4 SQ counters, never combined with other traces):
#   tools/pmc_mix.sh TAG "python3 tools/pmc_frame.py scene_08 1920 1080 256 8 2"
# Output under gpurun_out/prof/<TAG>/mix_*; summarise with tools/pmc_summary.py.
tag="$1"; B="$2"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out="gpurun_out/prof/$tag"
mkdir -p "$out"
pass() {  # name counters...
  local name=$1; shift
  echo "=== $name: $*"
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace --stats -d "$out/$name" -o "$name" --output-format csv \
    -- $B > "$out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
pass mix_f32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32
pass mix_int SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU SQ_INSTS_SALU
pass mix_lds SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS
pass mix_sqc SQC_ICACHE_MISSES SQC_DCACHE_MISSES
exit 0
