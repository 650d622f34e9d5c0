cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k test_param_grid_fit_shares_ingest"
for cfg in "X=1" "ALBEDO_ROTATE_BF=0" "ALBEDO_GRAM_BF=0" "ALBEDO_ROTATE_BF=0 ALBEDO_GRAM_BF=0" "ALBEDO_LIGHT16=0"; do
  echo "== $cfg" >> gpurun_out/bisect.log
  env $cfg timeout -k 10 200 $T >> gpurun_out/bisect.log 2>&1
  echo "rc=$?" >> gpurun_out/bisect.log
done
exit 0
