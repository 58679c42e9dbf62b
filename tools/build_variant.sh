#!/bin/bash
# Build an A/B variant of libcsg.so into constructionsceneposeestimation_amd/libcsg_<name>.so:
# the kernels (csg_kernels.hip/.h) from git revision <rev> ("-" = working tree)
# with the working tree's C-ABI host code, plus extra hipcc flags.
#   tools/build_variant.sh base HEAD          tools/build_variant.sh occ6 - -DCSG_OCC=6
# Use with CSG_LIB=<path> (see _lib.py).
set -e
cd "$(dirname "$0")/.."
name=$1; rev=${2:--}; shift 2 || true
src=constructionsceneposeestimation_amd/csrc
tmp=$(mktemp -d)
mkdir -p $tmp/pkg/csrc $tmp/include
cp include/csg_api.h $tmp/include/
cp $src/csg_api.cpp $src/csg_kernels.hip $src/csg_kernels.h $src/csg_encode.hip $src/csg_encode.h $src/csg_deflate.h $src/csg_widen.h $tmp/pkg/csrc/
if [ "$rev" != "-" ]; then
  for f in csg_kernels.hip csg_kernels.h; do git show $rev:$src/$f > $tmp/pkg/csrc/$f; done
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 -Wall -pthread "$@" \
  -o constructionsceneposeestimation_amd/libcsg_$name.so $tmp/pkg/csrc/csg_kernels.hip $tmp/pkg/csrc/csg_encode.hip $tmp/pkg/csrc/csg_api.cpp
rm -rf $tmp
echo built constructionsceneposeestimation_amd/libcsg_$name.so
