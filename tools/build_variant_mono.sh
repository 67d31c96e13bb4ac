#!/bin/bash
# dev: build libraysnail_hip as ONE translation unit with extra -D flags (debug builds whose device
# globals must be shared by all kernels, e.g. -DRS_TRAV_STATS) into raysnail_amd/lib/var_<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
B=/tmp/rs_var_$N; mkdir -p $B
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math $*"
/opt/rocm/bin/hipcc $F -c $R/raysnail_amd/csrc/rs_kernels.hip -o $B/k.o &
/opt/rocm/bin/hipcc $F -x hip -c $R/raysnail_amd/csrc/rs_host.cpp -o $B/h.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/raysnail_amd/lib/var_$N.so $B/k.o $B/h.o
echo built var_$N.so
