cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "param_grid or cv_grid" > gpurun_out/grid.log 2>&1
