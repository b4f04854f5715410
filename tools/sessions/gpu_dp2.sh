#!/bin/bash
# Multi-rank rehearsal on ONE GPU: GPU tests (incl. 2 ranks on cuda:0, host-staged gloo) and a
# 2-rank bench with --backend gloo. The real multi-GPU run (nccl = RCCL) is the driver's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --backend gloo --lines-per-gpu 2000000 --steps 3 --warmup 1 --parse-requests 0 > gpurun_out/bench_dp2_gloo.json 2> gpurun_out/bench_dp2_gloo.err && echo DP2_OK
