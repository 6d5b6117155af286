#!/bin/bash
# tools/ab_build.sh <exp> -- a variant libcgx.so for same-box A/B timing:
# every source compiled with -DCGX_EXP=<exp>; an experiment puts its variant
# behind `#if CGX_EXP & bit` while it is measured (the product never defines
# CGX_EXP; round 3's experiments -- p_new stores, CSR tiling -- were removed
# after their A/B); output ab/<exp>/libcgx.so.  Use it through
# cgx.py's CGX_LIB, or tools/ab_probe.sh.  To compare against the last commit:
# copy its libcgx.so to ab/0/ before rebuilding.
set -eu
cd "$(dirname "$0")/../conjugate-gradient_amd"
exp=$1
out=../ab/$exp
mkdir -p $out
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -Icsrc -DCGX_EXP=$exp"
objs=""
for src in csrc/cgx_kernels.hip csrc/cgx_matrix.cpp csrc/cgx_solver.cpp csrc/cgx_mvops.cpp \
           csrc/cgx_gen.cpp csrc/cgx_partition.cpp csrc/cgx_dist.cpp csrc/cgx_io.cpp; do
  o=$out/$(basename "${src%.*}").o
  /opt/rocm/bin/hipcc $F -c $src -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -o $out/libcgx.so $objs -shared \
  -Wl,--version-script=csrc/libcgx.map -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lamdhip64
echo "built $out/libcgx.so"
