# Why does the bench's H2D fall back from SDMA to a blit kernel? The HIP runtime's own log of the
# copies (AMD_LOG_LEVEL=3/4, all masks) during a short bench run -> gpurun_out/copy_log_*.txt
# Run: gpurun -- bash tools/gpu_copy_log.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lv in 3 4; do
  AMD_LOG_LEVEL=$lv timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --parse-requests 0 \
    > gpurun_out/copy_log_bench_$lv.out 2> /tmp/copy_log_$lv.err
  echo "level $lv rc=$? lines=$(wc -l < /tmp/copy_log_$lv.err)"
  grep -i -E "HSA copy|falling|blit|sdma" /tmp/copy_log_$lv.err | cut -c1-300 | tail -300 > gpurun_out/copy_log_$lv.txt || true
  grep -c -i "hipMemcpy" /tmp/copy_log_$lv.err || true
  head -c 3000 /tmp/copy_log_$lv.err > gpurun_out/copy_log_${lv}_head.txt
  rm -f /tmp/copy_log_$lv.err
done
wc -l gpurun_out/copy_log_3.txt gpurun_out/copy_log_4.txt
