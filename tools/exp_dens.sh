cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in tanh exp cube; do timeout -k 10 120 python tools/bench_split.py 128 5e7 3 $d || exit 1; done
PICARD_NO_YSTORE=1 timeout -k 10 120 python tools/bench_split.py 128 5e7 3 tanh || exit 1
PICARD_NO_YSTORE=1 timeout -k 10 120 python tools/bench_split.py 128 5e7 3 cube || exit 1
