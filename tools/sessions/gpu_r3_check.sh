#!/bin/bash
# Round 3 end-of-session check: smoke + whole GPU suite on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r3_check}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo SMOKE_OK || { tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
