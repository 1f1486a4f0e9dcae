# usage: bash tools/exp_nw.sh — time fused/loss/fromy for density interleave-width variants (rebuilds the library)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "2 1 1" "2 2 2" "1 1 1" "4 2 1"; do
  set -- $cfg
  make -s -C picard-ica_amd clean && make -s -C picard-ica_amd -j16 EXTRA_HIPFLAGS="-DPC_FUSED_NW=$1 -DPC_LOSS_NW=$2 -DPC_FROMY_NW=$3" > /dev/null || exit 1
  echo "== NW fused=$1 loss=$2 fromy=$3"
  timeout -k 10 120 python tools/bench_split.py 128 5e7 3 || exit 1
done
make -s -C picard-ica_amd clean && make -s -C picard-ica_amd -j16 > /dev/null
