# usage: bash tools/isa_hist.sh <mangled-kernel-prefix>  — VALU/MFMA histogram of the kernel's innermost loop(s)
cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=on -Wno-unused-function -Wno-unused-variable --cuda-device-only -S -o /tmp/device.s $GRAFT_SRC 2>/dev/null
awk -v k="$1" 'index($0,k)==1 && /:/ {on=1} on {print} on && /^\.Lfunc_end/ {exit}' /tmp/device.s > /tmp/kern.s
awk '/Inner Loop Header/ {on=1} on {print} on && /s_cbranch_vccnz/ {on=0}' /tmp/kern.s | grep -v "^\s*;" | awk '{print $1}' | sort | uniq -c | sort -rn | head -${2:-25}
grep -E "^\s+\.(vgpr|agpr|sgpr)_count|vgpr_spill" /tmp/device.s | head -0
