cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/native/pinned_probe > gpurun_out/pinned_probe.json 2>&1; echo rc=$?
cat gpurun_out/pinned_probe.json
