cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-include-regex "k_bpg_dedupe_all" -d gpurun_out/pmc_bpg/p1 -o run --output-format csv -- python3 tools/bpg_probe.py --lens 512 --reps 3 > gpurun_out/pmc_bpg_p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --kernel-include-regex "k_bpg_dedupe_all" -d gpurun_out/pmc_bpg/p2 -o run --output-format csv -- python3 tools/bpg_probe.py --lens 512 --reps 3 > gpurun_out/pmc_bpg_p2.log 2>&1
