# attention kernels of the working tree's library vs libstableavatar_hip_old.so (built from the previous commit):
# kbench attnvar (kernels 3 and 1 at the config-2 launch) and cross3, alternating processes, 3 rounds
set -u
mkdir -p gpurun_out
tag=${1:-ab}
for i in 1 2 3; do
  for lib in old new; do
    f=stableavatar_amd/libstableavatar_hip.so
    [ $lib = old ] && f=stableavatar_amd/libstableavatar_hip_old.so
    SA_LIB=$f SA_KB_AVARS=3,1 scripts/gpustep.sh 300 gpurun_out/kb_${tag}_${lib}_$i.log python -u -m stableavatar_amd.kbench attnvar cross3 || exit 1
    grep -h '"kernel": "attn_' gpurun_out/kb_${tag}_${lib}_$i.log | sed "s/^/$lib $i /"
  done
done
