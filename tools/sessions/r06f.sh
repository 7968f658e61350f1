#!/bin/bash
# round 6: validation of the fma box test (a new box definition, product and oracle): smoke,
# the whole GPU suite, the bench line
tools/gpu_session.sh \
 "r06f_smoke|200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "r06f_bench|300|python3 -u bench.py" \
 "r06f_gpu_suite|900|python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
