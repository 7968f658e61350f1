#!/bin/bash
# PMC A/B: the same counter groups for several library variants (GPU box).
# usage: tools/pmc_ab.sh tag lib1.so lib2.so ...
#   PMC_FRAME="SCENE W H SPP DEPTH FRAMES": profile tools/pmc_frame.py on that configuration
#   instead of bench.py's headline frame (e.g. "gen:10000:sphere 1920 1080 512 8 2" for C5)
tag=$1; shift
if [ -n "$PMC_FRAME" ]; then prog="tools/pmc_frame.py $PMC_FRAME"; else prog="bench.py --steps 2 --warmup 1 --no-cpu-baseline"; fi
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename "$lib" .so)
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    g=$(echo $grp | cut -c1-12 | tr ' ' _)
    out="gpurun_out/prof/$tag/$name/pmc_$g"
    mkdir -p "$out"
    FORMA_RT_LIB=$(realpath "$lib") timeout -k 10 300 rocprofv3 --pmc $grp -d "$out" -o pmc --output-format csv -- \
      python3 $prog > "$out.log" 2>&1
    rc=$?; echo "$name $g rc=$rc"; [ $rc -ge 124 ] && exit $rc
  done
  FORMA_RT_LIB=$(realpath "$lib") timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof/$tag/$name/trace" -o trace --output-format csv -- \
      python3 $prog > "gpurun_out/prof/$tag/$name/trace.log" 2>&1
  rc=$?; echo "$name trace rc=$rc"; [ $rc -ge 124 ] && exit $rc
done
exit 0
