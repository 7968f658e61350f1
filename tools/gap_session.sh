#!/bin/bash
# rocprofv3 kernel traces of tools/gap_probe.py's modes; prints the per-frame gap analysis.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tag=${1:-gap}
for mode in gather u8 none; do
  d=gpurun_out/$tag/$mode
  mkdir -p "$d"
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run -- python3 tools/gap_probe.py $mode 12 > "$d.log" 2>&1
  rc=$?
  echo "== $mode rc=$rc"; tail -n 2 "$d.log"
  [ $rc -ne 0 ] && exit $rc
  python3 tools/gap_probe.py --analyze "$(find "$d" -name '*kernel_trace.csv' | head -1)" | tail -n 4
done
