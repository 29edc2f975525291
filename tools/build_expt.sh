#!/bin/bash
# Build libnfx variants with the spline backward compiled under -DNFX_SBWD_EXPT=<n> into expt/.
set -e
R=/root/repo; P=$R/normalizing-flows-study_amd; mkdir -p $R/expt
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$P/csrc -mllvm -amdgpu-mfma-vgpr-form=1"
for n in "$@"; do
  for t in nfx_spline_bwd_h2; do /opt/rocm/bin/hipcc $F -DNFX_SBWD_EXPT=$n -c $P/csrc/$t.hip -o $R/expt/${t}_$n.o & done
done
wait
for n in "$@"; do
  objs=$(ls $P/build/*.o | grep -v nfx_spline_bwd_h2.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $R/expt/libnfx_$n.so $objs $R/expt/nfx_spline_bwd_h2_$n.o
done
