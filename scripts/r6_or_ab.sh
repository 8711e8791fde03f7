# the OR-tested softmax step (v6_softmax_p) vs the previous tree's library: attention kernels 1 (V rows) and 3 (V^T)
# at the config-2 launch, alternating processes; libstableavatar_hip_old.so = the library built from the previous commit
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  for lib in old new; do
    f=stableavatar_amd/libstableavatar_hip.so
    [ $lib = old ] && f=stableavatar_amd/libstableavatar_hip_old.so
    SA_LIB=$f SA_KB_AVARS=3,1 scripts/gpustep.sh 300 gpurun_out/kb_or_${lib}_$i.log python -u -m stableavatar_amd.kbench attnvar || exit 1
    echo "$lib $(grep attn_self gpurun_out/kb_or_${lib}_$i.log)"
  done
done
