# usage: bash tools/gpu_c4chunk.sh TAG — the C4-shape tiled passes (256 × 1e7) with T chunks whose
# y/ψ fragments fit PICARD_TILED_CHUNK_MB (Infinity Cache experiment) against one chunk
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/c4c_$TAG
mkdir -p $O
for MB in 0 192 512 2048; do
  if [ $MB = 0 ]; then E=""; else E="PICARD_TILED_CHUNK_MB=$MB"; fi
  env $E timeout -k 10 180 python3 tools/bench_tiled.py 256 1e7 3 > $O/mb$MB.txt 2>&1 || { cat $O/mb$MB.txt; exit 1; }
  echo "== chunk MB $MB"; grep -E "full|multi na=11" $O/mb$MB.txt
done
# C4 end to end: the bounded multi-try pass until its first wasted full pass (default) against
# exact tries only (PICARD_MULTI_F32=0)
for M in 1 0; do
  PICARD_MULTI_F32=$M timeout -k 10 200 python3 tools/run_configs.py C4 > $O/c4_m$M.json 2>&1 || { cat $O/c4_m$M.json; exit 1; }
  echo "== C4 PICARD_MULTI_F32=$M"; python3 -c "import json,sys; d=json.loads(open('$O/c4_m$M.json').read().strip().splitlines()[-1]); print({k: d[k] for k in d if k in ('iterations_s','n_iterations','converged','n_evaluations','amari')})"
done
