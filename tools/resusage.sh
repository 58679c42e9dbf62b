#!/bin/bash
# k_raster resource usage for a config: tools/resusage.sh "<attr or x>" [hipcc -D flags...]
attr=$1; shift
src=/root/repo/constructionsceneposeestimation_amd/csrc
a=""; [ "$attr" != x ] && a="__attribute__(($attr))"
sed "s/CSG_RASTER_ATTR void k_raster/$a void k_raster/" $src/csg_kernels.hip > $src/_tmp.hip
cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 "$@" -c $src/_tmp.hip -o /tmp/_k.o -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "error|8k_raster" -A12 | grep -E "error|VGPRs:|VGPRs Spill|ScratchSize|Occupancy|LDS" | sed "s/.*remark: *//;s/ \[-R.*//" | tr '\n' ' '; echo " <- $attr $*"
rm -f $src/_tmp.hip
