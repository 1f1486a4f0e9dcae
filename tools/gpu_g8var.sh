cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "" "PICARD_G8_DBG=1" "PICARD_G8_DBG=2" "PICARD_G8=0"; do
  echo "== $v"; env $v timeout -k 10 120 python -u tools/bench_pass.py 128 2e7 tanh 5 || exit 1
done
