#!/bin/bash
# MFMA NFA kernel: GPU == host twin, then context-feature engine A/B (dfa vs mfma) under rocprof
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nfa.py tests/test_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_nfa.log 2>&1 && echo NFA_TESTS_OK &&
cd /tmp && export TMPDIR=/tmp &&
ENGINE_CONTEXT_ENGINE=mfma timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_mfma -o run -- python3 $R/bench.py --steps 3 --warmup 1 --parse-requests 0 > $R/gpurun_out/ab_mfma.log 2>&1 && echo AB_MFMA_OK &&
ENGINE_CONTEXT_ENGINE=dfa timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_dfa -o run -- python3 $R/bench.py --steps 3 --warmup 1 --parse-requests 0 > $R/gpurun_out/ab_dfa.log 2>&1 && echo AB_DFA_OK
