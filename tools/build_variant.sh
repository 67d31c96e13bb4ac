#!/bin/bash
# dev: build libraysnail_hip with extra -D flags into raysnail_amd/lib/var_<name>.so (the same
# translation units as raysnail_amd/csrc/Makefile, compiled in parallel)
# usage: tools/build_variant.sh <name> [flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
B=/tmp/rs_var_$N; mkdir -p $B
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math $*"
for t in -1 0 1 2 3 4; do
  /opt/rocm/bin/hipcc $F -DRS_TU=$t -c $R/raysnail_amd/csrc/rs_kernels.hip -o $B/k$t.o &
done
/opt/rocm/bin/hipcc $F -x hip -c $R/raysnail_amd/csrc/rs_host.cpp -o $B/h.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/raysnail_amd/lib/var_$N.so $B/k*.o $B/h.o
echo built var_$N.so
