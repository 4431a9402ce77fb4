# Same-box A/B of prebuilt library sets (run via gpurun from the repo root):
#   bash tools/ab_libs.sh ROUNDS "CMD" DIR1 DIR2 ...
# Each DIR holds a libdmdqn_hip.so + libdmdqn_torch.so built here (e.g. from
# another revision of a kernel); every round copies each set over
# dmdqn_amd/lib/ in turn and runs CMD (alternating, so box drift hits all
# sets alike).  The current build is restored at the end.
set -e
R=$1; CMD=$2; shift 2
L=dmdqn_amd/lib
mkdir -p /tmp/_ab_cur && cp $L/libdmdqn_hip.so $L/libdmdqn_torch.so /tmp/_ab_cur/
for r in $(seq 1 $R); do
  for d in "$@"; do
    cp $d/libdmdqn_hip.so $d/libdmdqn_torch.so $L/
    echo "== round $r $d"
    timeout -k 10 300 bash -c "$CMD"
  done
done
cp /tmp/_ab_cur/*.so $L/
