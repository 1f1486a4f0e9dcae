# usage: bash tools/gpu_model_pairs_ab.sh TAG — the pair / screen / bit-identity GPU tests, then the
# C3 bench (no CPU baseline, no other configs) with PICARD_MODEL_PAIRS=1 / 0 alternating twice
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/mpairs_$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_screen_pair.py tests/test_gpu_int8.py tests/test_gpu_group.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  for mp in 1 0; do
    PICARD_TRACE=1 PICARD_MODEL_PAIRS=$mp timeout -k 10 400 python -u bench.py --configs 0 --cpu-baseline 0 > $O/c3_mp${mp}_$rep.json 2> $O/c3_mp${mp}_$rep.err || { tail -20 $O/c3_mp${mp}_$rep.err; exit 1; }
    echo "MODEL_PAIRS=$mp rep $rep: $(python3 tools/bench_summary.py $O/c3_mp${mp}_$rep.json | head -1)"
    rm -f $O/c3_mp${mp}_$rep.err.big
  done
done
