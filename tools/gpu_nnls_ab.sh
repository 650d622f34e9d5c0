#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/nnls_ab.py run 0 /tmp/nnls_a0.npz > gpurun_out/nnls_ab.txt 2> gpurun_out/nnls_ab0.err
timeout -k 10 400 python -u tools/nnls_ab.py run 1 /tmp/nnls_a1.npz >> gpurun_out/nnls_ab.txt 2> gpurun_out/nnls_ab1.err
timeout -k 10 400 python -u tools/nnls_ab.py run 1rs /tmp/nnls_rs.npz >> gpurun_out/nnls_ab.txt 2> gpurun_out/nnls_abr.err
echo all-ok
