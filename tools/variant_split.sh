# usage: bash tools/variant_split.sh N T v1 v2 ... — time fused/loss passes for each variants/<v>.so
N=$1; T=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PICARD_NO_YSTORE=1  # loss-only passes as the orthogonal solver runs them
cp picard-ica_amd/libpicard_mi355x.so /tmp/orig.so
for v in "$@"; do
  cp variants/$v.so picard-ica_amd/libpicard_mi355x.so
  echo "== $v"
  timeout -k 10 120 python tools/bench_split.py $N $T 5 tanh 0.3 || { cp /tmp/orig.so picard-ica_amd/libpicard_mi355x.so; exit 1; }
done
cp /tmp/orig.so picard-ica_amd/libpicard_mi355x.so
