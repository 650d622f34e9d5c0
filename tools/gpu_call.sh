#!/bin/bash
# One GPU call of this round: steps given as arguments are run in order, each under its own time
# limit; the call stops at the first failing step.  usage: tools/gpu_call.sh <step> [<step> ...]
#   bounds_c2 | bounds_c4 | tests_* | smoke | bench_c4 | bench_c2 | bench_c5 | prof_* | trace_* | probes
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
for s in "$@"; do
  echo "== $s $(date +%T)"
  case $s in
    bounds_c2) timeout -k 10 300 python -u tools/topk_bounds.py --config c2 --sweeps 10 --sample 16384 --out gpurun_out/bounds_c2_s10.json > gpurun_out/bounds_c2.log 2>&1 ;;
    bounds_c4) timeout -k 10 500 python -u tools/topk_bounds.py --config c4 --sweeps 25 --sample 16384 --out gpurun_out/bounds_c4_s25.json > gpurun_out/bounds_c4.log 2>&1 ;;
    tq_*) n=${s#tq_}; ALBEDO_ALS_LIB=$PWD/tools/ab/$n.so timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "half_sweep or golden or facade or albedo_protocol" > gpurun_out/$s.log 2>&1 ;;
    tests_quick) timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "half_sweep or golden or facade or albedo_protocol" > gpurun_out/tests_quick.log 2>&1 ;;
    tests_topk) timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_recommenders.py -k "topk or ndcg or recommend or transform or facade or albedo" > gpurun_out/tests_topk.log 2>&1 ;;
    tests_scale) timeout -k 10 900 $PYT tests/test_gpu_scale.py -s > gpurun_out/tests_scale.log 2>&1 ;;
    tests_c3) timeout -k 10 600 $PYT tests/test_gpu_scale.py -s -k "c2_scale or c3 or two_contexts" > gpurun_out/tests_c3.log 2>&1 ;;
    tests_all) timeout -k 10 1100 $PYT tests -m gpu > gpurun_out/tests_all.log 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 ;;
    bench_default) timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err ;;
    bench_trace) ALBEDO_TOPK_TRACE=1 timeout -k 10 900 python -u bench.py --no-cpu > gpurun_out/bench_trace.json 2> gpurun_out/bench_trace.err ;;
    bench_trace_zc) ALBEDO_TOPK_ZEROCOPY=1 ALBEDO_TOPK_TRACE=1 timeout -k 10 900 python -u bench.py --no-cpu > gpurun_out/bench_trace_zc.json 2> gpurun_out/bench_trace_zc.err ;;
    tests_topk_zc) ALBEDO_TOPK_ZEROCOPY=1 timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_recommenders.py -k "topk or ndcg or recommend or transform or facade or albedo" > gpurun_out/tests_topk_zc.log 2>&1 ;;
    bench_trace_zc2) ALBEDO_TOPK_ZEROCOPY=2 ALBEDO_TOPK_TRACE=1 timeout -k 10 900 python -u bench.py --no-cpu > gpurun_out/bench_trace_zc2.json 2> gpurun_out/bench_trace_zc2.err ;;
    tests_topk_zc2) ALBEDO_TOPK_ZEROCOPY=2 timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_recommenders.py -k "topk or ndcg or recommend or transform or facade or albedo" > gpurun_out/tests_topk_zc2.log 2>&1 ;;
    tests_c3_overlap) ALBEDO_TOPK_OVERLAP=1 timeout -k 10 600 $PYT tests/test_gpu_scale.py -s -k "c3_topk_passes" > gpurun_out/tests_c3_overlap.log 2>&1 ;;
    bench_c4) timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err ;;
    bench_c2) timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 5 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err ;;
    bench_c5cpu) timeout -k 10 600 python -u bench.py --config c5 --steps 2 --warmup 1 --topk-users 0 > gpurun_out/bench_c5cpu.json 2> gpurun_out/bench_c5cpu.err ;;
    bench_c5_s*) ALBEDO_NNLS_MIN_SLOTS=${s#bench_c5_s} timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu --topk-users 0 > gpurun_out/$s.json 2> gpurun_out/$s.err ;;
    repro_mrbig) timeout -k 10 600 python -u tools/repro_mrbig.py 16 /tmp/repro_mrbig > gpurun_out/repro_mrbig.log 2>&1 ;;
    tests_mrbig) timeout -k 10 900 $PYT tests/test_multi_rank.py -k c4_shaped > gpurun_out/tests_mrbig.log 2>&1 ;;
    batchtime4) (cd tools/probe && timeout -k 5 120 ./batchtime 256 16 500000 200000 6 && timeout -k 5 120 ./batchtime 256 8 500000 100000 12 && timeout -k 5 120 ./batchtime 256 4 500000 50000 24) > gpurun_out/batchtime4.txt 2>&1 ;;
    bench_c5) timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu --topk-users 0 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err ;;
    prof_c4) timeout -k 10 1100 tools/prof.sh c4 r03 16384 > gpurun_out/prof_c4.log 2>&1 ;;
    prof_c4r4) timeout -k 10 1100 tools/prof.sh c4 r04 16384 > gpurun_out/prof_c4r4.log 2>&1 ;;
    prof_c5r4) timeout -k 10 900 tools/prof.sh c5 r04 0 > gpurun_out/prof_c5r4.log 2>&1 ;;
    prof_c4r5) timeout -k 10 1100 tools/prof.sh c4 r05 0 > gpurun_out/prof_c4r5.log 2>&1 ;;
    prof_c4r6) timeout -k 10 1100 tools/prof.sh c4 r06 0 > gpurun_out/prof_c4r6.log 2>&1 ;;
    prof_c5r6) timeout -k 10 900 tools/prof.sh c5 r06 0 > gpurun_out/prof_c5r6.log 2>&1 ;;
    prof_c5r5) timeout -k 10 900 tools/prof.sh c5 r05 0 > gpurun_out/prof_c5r5.log 2>&1 ;;
    pmc_topk5) timeout -k 10 700 tools/pmc_topk5.sh r05 > gpurun_out/pmc_topk5.log 2>&1 ;;
    multi) # back-to-back processes on one box (each a fresh context on memory the previous one freed)
      for i in 1 2 3 4 5 6; do timeout -k 10 200 python -u bench.py --steps 2 --warmup 40 --no-cpu --topk-users 0 > gpurun_out/multi_$i.json 2> gpurun_out/multi_$i.err || { echo "multi run $i failed"; exit 1; }; done ;;
    det_c2) timeout -k 10 300 python -u tools/determinism.py --config c2 --rank 64 --halves 20 --out gpurun_out/det_c2.json > gpurun_out/det_c2.log 2>&1 ;;
    det_c2np) ALBEDO_L16_NOPAIR=1 timeout -k 10 300 python -u tools/determinism.py --config c2 --rank 64 --halves 20 --out gpurun_out/det_c2np.json > gpurun_out/det_c2np.log 2>&1 ;;
    det_c2ab_*) n=${s#det_c2ab_}; ALBEDO_ALS_LIB=$PWD/tools/ab/$n.so timeout -k 10 300 python -u tools/determinism.py --config c2 --rank 64 --halves 20 --out gpurun_out/$s.json > gpurun_out/$s.log 2>&1 ;;
    det_c4) timeout -k 10 400 python -u tools/determinism.py --config c4 --rank 128 --halves 12 --out gpurun_out/det_c4.json > gpurun_out/det_c4.log 2>&1 ;;
    stress) timeout -k 10 300 python -u bench.py --steps 5 --warmup 300 --no-cpu --topk-users 0 > gpurun_out/stress.json 2> gpurun_out/stress.err ;;
    prof_c5) timeout -k 10 900 tools/prof.sh c5 r03 0 > gpurun_out/prof_c5.log 2>&1 ;;
    prof_c2) timeout -k 10 600 tools/prof.sh c2 r03 16384 > gpurun_out/prof_c2.log 2>&1 ;;
    trace_c4) mkdir -p gpurun_out/trace_c4 && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_c4 -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu --topk-users 16384 > gpurun_out/trace_c4/bench.json 2> gpurun_out/trace_c4/bench.err ;;
    trace_topk) mkdir -p gpurun_out/trace_topk && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_topk -o run -- python3 -u bench.py --steps 1 --warmup 24 --no-cpu > gpurun_out/trace_topk/bench.json 2> gpurun_out/trace_topk/bench.err ;;
    trace_topk4) mkdir -p gpurun_out/trace_topk4 && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_topk4 -o run -- python3 -u bench.py --no-cpu > gpurun_out/trace_topk4/bench.json 2> gpurun_out/trace_topk4/bench.err ;;
    trace_topkcp) mkdir -p gpurun_out/trace_topkcp && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/trace_topkcp -o run -- python3 -u bench.py --no-cpu --steps 1 --warmup 0 > gpurun_out/trace_topkcp/bench.json 2> gpurun_out/trace_topkcp/bench.err ;;
    tests_solve) timeout -k 10 700 $PYT tests/test_gpu_parity.py tests/test_gpu_heavy_tail.py tests/test_gpu_scale.py -k "half_sweep or golden or facade or albedo_protocol or column_scaling or positive_definite or heavy or c4_scale_rows or c2_scale" > gpurun_out/tests_solve.log 2>&1 ;;
    tests_nnls) timeout -k 10 700 $PYT tests/test_gpu_parity.py tests/test_gpu_heavy_tail.py tests/test_gpu_c5_rows.py -k "nnls or c5 or million" > gpurun_out/tests_nnls.log 2>&1 ;;
    nnlsrow) (for dg in "2048 200" "512 2000" "4096 60"; do set -- $dg; echo "## 512-thread rows $1 deg $2"; timeout -k 5 60 tools/probe/nnlstime 256 100000 $1 $2 || exit 1; echo "## 1024-thread rows $1 deg $2"; ALBEDO_NNLS_ROW=1024 timeout -k 5 60 tools/probe/nnlstime 256 100000 $1 $2 || exit 1; done) > gpurun_out/nnlsrow.txt 2>&1 ;;
    nnlsph) (for b in ${NNLS_PROBES:-nnlstime}; do for dg in "2048 200" "4096 60" "512 2000"; do set -- $dg; echo "## $b rows $1 deg $2"; timeout -k 5 60 tools/probe/$b 256 100000 $1 $2 || exit 1; done; done) > gpurun_out/nnlsph.txt 2>&1 ;;
    bench_ab_*) n=${s#bench_ab_}; ALBEDO_ALS_LIB=$PWD/tools/ab/$n.so timeout -k 10 900 python -u bench.py > gpurun_out/$s.json 2> gpurun_out/$s.err ;;
    bench_c5_old) ALBEDO_NNLS_ROW=1024 timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu --topk-users 0 > gpurun_out/bench_c5_old.json 2> gpurun_out/bench_c5_old.err ;;
    batchtime) (cd tools/probe && timeout -k 5 120 ./batchtime 256 16 500000 200000 6 && timeout -k 5 120 ./batchtime 256 8 500000 100000 12) > gpurun_out/batchtime.txt 2>&1 ;;
    nnlsab) (timeout -k 5 60 tools/probe/nnlstime_base 256 100000 2048 200 && timeout -k 5 60 tools/probe/nnlstime 256 100000 2048 200 && timeout -k 5 60 tools/probe/nnlstime_base 256 100000 2048 200 && timeout -k 5 60 tools/probe/nnlstime 256 100000 2048 200) > gpurun_out/nnlsab.txt 2>&1 ;;
    nnlsab2) (for b in nnlstime_base nnlstime_u1 nnlstime_u2 nnlstime_base nnlstime_u1 nnlstime_u2; do echo "## $b"; timeout -k 5 60 tools/probe/$b 256 100000 2048 200 || exit 1; done; for b in nnlstime_base nnlstime_u1 nnlstime_u2; do echo "## $b 128"; timeout -k 5 60 tools/probe/$b 128 100000 2048 200 || exit 1; done) > gpurun_out/nnlsab2.txt 2>&1 ;;
    nnlstime) timeout -k 5 60 tools/probe/nnlstime 256 100000 2048 200 > gpurun_out/nnlstime.txt 2>&1 ;;
    tests_gram) timeout -k 10 300 $PYT tests/test_gpu_heavy_tail.py -k "gram" > gpurun_out/tests_gram.log 2>&1 ;;
    trace_c5) mkdir -p gpurun_out/trace_c5 && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_c5 -o run -- python3 -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu --topk-users 0 > gpurun_out/trace_c5/bench.json 2> gpurun_out/trace_c5/bench.err ;;
    tests_mr) timeout -k 10 900 $PYT tests/test_multi_rank.py > gpurun_out/tests_mr.log 2>&1 ;;
    wavetime) (cd tools/probe && timeout -k 5 120 ./wavetime 20000000 80,160,320,640,1280,4096 200000000 && timeout -k 5 120 ./wavetime_bo 20000000 80,160,320,640,1280,4096 200000000) > gpurun_out/wavetime.txt 2>&1 ;;
    wavetime1) (cd tools/probe && timeout -k 5 120 ./wavetime 20000000 80,160,320,640,1280,4096 200000000) > gpurun_out/wavetime1.txt 2>&1 ;;
    c4ingest) timeout -k 10 900 python -u tools/c1p_job.py --config c4 --rank 128 --ingest-only --out gpurun_out/c4_ingest.json > gpurun_out/c4_ingest.log 2>&1 ;;
    c1p) timeout -k 10 900 python -u tools/c1p_job.py --out gpurun_out/c1p_job.json > gpurun_out/c1p_job.log 2>&1 ;;
    tests_eig) timeout -k 10 300 $PYT tests/test_gpu_parity.py -k "device_eigensolver or half_sweep_ranks or orthogonal" > gpurun_out/tests_eig.log 2>&1 ;;
    pmc_topk4) timeout -k 10 600 tools/pmc_topk4.sh r04 > gpurun_out/pmc_topk4.log 2>&1 ;;
    bench_topk_g8) ALBEDO_TOPK_GMAX=8 timeout -k 10 400 python -u bench.py --steps 1 --warmup 24 --no-cpu > gpurun_out/bench_topk_g8.json 2> gpurun_out/bench_topk_g8.err ;;
    tests_topk_g8) ALBEDO_TOPK_GMAX=8 timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_recommenders.py -k "topk or ndcg or recommend or transform or facade or albedo" > gpurun_out/tests_topk_g8.log 2>&1 ;;
    bench_topk_g4) ALBEDO_TOPK_GMAX=4 timeout -k 10 400 python -u bench.py --steps 1 --warmup 24 --no-cpu > gpurun_out/bench_topk_g4.json 2> gpurun_out/bench_topk_g4.err ;;
    topkph_g4) ALBEDO_TOPK_GMAX=4 timeout -k 10 400 python -u tools/topk_phases.py --lib tools/ab/topkph.so --out gpurun_out/topkph_g4.json > gpurun_out/topkph_g4.log 2>&1 ;;
    bench_topk_tr) ALBEDO_TOPK_TRACE=1 timeout -k 10 400 python -u bench.py --steps 1 --warmup 24 --no-cpu > gpurun_out/bench_topk_tr.json 2> gpurun_out/bench_topk_tr.err ;;
    bench_topk_p*) ALBEDO_TOPK_PASS=${s#bench_topk_p} timeout -k 10 400 python -u bench.py --steps 1 --warmup 24 --no-cpu > gpurun_out/$s.json 2> gpurun_out/$s.err ;;
    bench_topk_d*) ALBEDO_TOPK_DIRSPLIT=${s#bench_topk_d} timeout -k 10 400 python -u bench.py --steps 1 --warmup 24 --no-cpu > gpurun_out/$s.json 2> gpurun_out/$s.err ;;
    bench_topk_kt*) ALBEDO_TOPK_KTX=${s#bench_topk_kt} timeout -k 10 400 python -u bench.py --steps 1 --warmup 24 --no-cpu > gpurun_out/$s.json 2> gpurun_out/$s.err ;;
    bench_topk) timeout -k 10 400 python -u bench.py --steps 1 --warmup 24 --no-cpu > gpurun_out/bench_topk.json 2> gpurun_out/bench_topk.err ;;
    bench_c4q) timeout -k 10 400 python -u bench.py --steps 3 --warmup 5 --no-cpu --topk-users 0 > gpurun_out/bench_c4q.json 2> gpurun_out/bench_c4q.err ;;
    bench_c4q_l*) timeout -k 10 400 python -u bench.py --steps 3 --warmup 5 --no-cpu --topk-users 0 --light ${s#bench_c4q_l} > gpurun_out/$s.json 2> gpurun_out/$s.err ;;
    abtk_*) # A/B of top-k: the 25-sweep + all-users top-30 bench on tools/ab/<name>.so, then restored
      n=${s#abtk_}; cp albedo_amd/libalbedo_als.so /tmp/albedo_main.so && cp tools/ab/$n.so albedo_amd/libalbedo_als.so && \
      { timeout -k 10 400 python -u bench.py --steps 1 --warmup 24 --no-cpu > gpurun_out/abtk_$n.json 2> gpurun_out/abtk_$n.err; r=$?; cp /tmp/albedo_main.so albedo_amd/libalbedo_als.so; [ $r -eq 0 ]; } ;;
    ab_*) # A/B: the quick c4 bench on tools/ab/<name>.so in place of the built library, then restored
      n=${s#ab_}; cp albedo_amd/libalbedo_als.so /tmp/albedo_main.so && cp tools/ab/$n.so albedo_amd/libalbedo_als.so && \
      { timeout -k 10 400 python -u bench.py --steps 3 --warmup 5 --no-cpu --topk-users 0 > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err; r=$?; cp /tmp/albedo_main.so albedo_amd/libalbedo_als.so; [ $r -eq 0 ]; } ;;
    debug_eig) timeout -k 10 600 python -u tools/debug_eig.py > gpurun_out/debug_eig.log 2>&1; r=$?; echo "debug_eig rc $r"; [ $r -le 1 ] ;;
    debug_c1) timeout -k 10 300 python -u tools/debug_c1.py > gpurun_out/debug_c1.log 2>&1; r=$?; echo "debug_c1 rc $r"; [ $r -le 1 ] ;;
    protocol_eu) { timeout -k 10 300 python -u tools/protocol_eu.py main; } > gpurun_out/protocol_eu.log 2>&1 ;;
    permlane) (cd tools/probe && timeout -k 5 60 ./permlane_probe) > gpurun_out/permlane.txt 2>&1 ;;
    factortime)(cd tools/probe && timeout -k 5 120 ./factortime 1000000) > gpurun_out/factortime.txt 2>&1 ;;
    prot_*) n=${s#prot_}; { ALBEDO_ALS_LIB=$PWD/tools/ab/$n.so timeout -k 10 300 python -u tools/protocol_eu.py $n; } > gpurun_out/prot_$n.log 2>&1 ;;
    topkph) timeout -k 10 400 python -u tools/topk_phases.py --lib tools/ab/topkph.so --out gpurun_out/topkph.json > gpurun_out/topkph.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo all-ok
