# usage: bash tools/gpu_hostspikes.sh TAG [all] — the one-rank-of-8 proxy (bench.py --t 1.25e7, C3 only)
# three times each under three OpenMP settings, with the per-iteration trace: host-time spikes
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, env...
  name=$1; shift
  for i in 1 2; do
    env "$@" PICARD_TRACE=1 timeout -k 10 120 python -u bench.py --t 1.25e7 --configs 0 --cpu-baseline 0 \
      > gpurun_out/hs_${TAG}_${name}_$i.json 2> gpurun_out/hs_${TAG}_${name}_$i.log || return 1
    grep step_ms gpurun_out/hs_${TAG}_${name}_$i.log | sed -E 's/.*step_ms ([0-9.]+) eval_ms ([0-9.]+) host_ms ([0-9.]+).*/\3/' \
      | sort -n | awk -v nm="$name $i" '{h[NR]=$1; s+=$1} END {printf "%s: n %d host mean %.3f median %.3f p90 %.3f max %.3f\n", nm, NR, s/NR, h[int(NR/2)+1], h[int(NR*0.9)], h[NR]}'
    python3 tools/bench_summary.py gpurun_out/hs_${TAG}_${name}_$i.json | head -2
  done
}
echo "nproc $(nproc) OMP_NUM_THREADS=$OMP_NUM_THREADS"
if [ "$2" = all ]; then
  run default OMP_DUMMY=1 && run passive OMP_WAIT_POLICY=passive && run omp8 OMP_NUM_THREADS=8
else
  run default OMP_DUMMY=1
fi
