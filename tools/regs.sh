#!/bin/bash
# dev: VGPRs / scratch / occupancy of kernels matching $1, with extra hipcc flags $2...
R=$(cd "$(dirname "$0")/.." && pwd)
pat=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off "$@" -c $R/raysnail_amd/csrc/rs_kernels.hip -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | grep -E "remark: +(Function Name|VGPRs|ScratchSize|Occupancy)" | sed -E 's/.*remark: +//; s/ \[-Rpass.*//' \
 | awk -v p="$pat" '/Function Name/{n=$3; show=(n ~ p)} show && !/Function Name/{printf "%s %s  ", $1, $NF} /Occupancy/ && show {print n}'
rm -f /tmp/regs_$$.o
