#!/bin/bash
# Build the product library of a git revision into scann_amd/lib/libscann_mi355x_<name>.so
# (for same-box A/Bs with tools/ab_libs.sh):  bash tools/build_rev.sh <rev> <name>
set -e
REV=$1; NAME=$2
ROOT=$(cd $(dirname $0)/.. && pwd)
T=$(mktemp -d)
mkdir -p $T/scann_amd/csrc $T/include
for f in smx_kernels.hip smx_searcher.hip smx_builder.hip smx_sort.hip smx_internal.h; do
  git -C $ROOT show $REV:scann_amd/csrc/$f > $T/scann_amd/csrc/$f
done
git -C $ROOT show $REV:include/scann_mi355x.h > $T/include/scann_mi355x.h
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wall \
  -o $ROOT/scann_amd/lib/libscann_mi355x_$NAME.so $T/scann_amd/csrc/smx_kernels.hip \
  $T/scann_amd/csrc/smx_searcher.hip $T/scann_amd/csrc/smx_builder.hip $T/scann_amd/csrc/smx_sort.hip
rm -rf $T
echo $ROOT/scann_amd/lib/libscann_mi355x_$NAME.so
