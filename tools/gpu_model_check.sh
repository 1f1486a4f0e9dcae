# usage: bash tools/gpu_model_check.sh TAG — the later-try model policy on the bit-identity fits
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PICARD_TRACE=1 timeout -k 10 300 python -u tools/model_policy_check.py > gpurun_out/model_$1.txt 2> gpurun_out/model_$1.err || { tail -20 gpurun_out/model_$1.err; exit 1; }
cat gpurun_out/model_$1.txt
awk '/^=== fit/ {k=$0} /\[picard-model\]/ {c[k]++} END {for (k in c) print c[k], k}' gpurun_out/model_$1.err
