#!/bin/bash
# Link a diagnostic variant of libnfx.so: recompile the named translation units with extra flags,
# reuse every other object of the main build (normalizing-flows-study_amd/build/).
#   bash tools/quick_variant.sh <name> "<flags>" nfx_made_wgrad.hip [...]  -> nfs_amd/libnfx_<name>.so
set -e
name=$1; flags=$2; shift 2
P=$(cd "$(dirname "$0")/.." && pwd)/normalizing-flows-study_amd
T=$(mktemp -d)
objs=""
for o in $P/build/*.o; do
  b=$(basename $o .o)
  skip=0
  for tu in "$@"; do [ "$b" = "${tu%.hip}" ] && skip=1; done
  [ $skip = 0 ] && objs="$objs $o"
done
for tu in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I$P/../include -I$P/csrc \
    -mllvm -amdgpu-mfma-vgpr-form=1 $flags -c $P/csrc/$tu -o $T/${tu%.hip}.o
  objs="$objs $T/${tu%.hip}.o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $P/nfs_amd/libnfx_$name.so $objs
rm -rf $T
echo "linked $P/nfs_amd/libnfx_$name.so"
