#!/bin/bash
# round 6, the final tree as committed: smoke, the bench line, the whole GPU suite
tools/gpu_session.sh \
 "r06ai_smoke|200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "r06ai_bench|300|python3 -u bench.py" \
 "r06ai_gpu_suite|1000|python3 -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread"
