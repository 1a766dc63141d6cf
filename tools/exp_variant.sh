#!/bin/bash
# Build an experiment variant of libhikari_amd.so from a copy of the sources with sed edits applied
# (CPU, this container): the product sources keep no experiment switches.
# usage: bash tools/exp_variant.sh <name> 'sed-expr-for-hk_kernels.hip' ['sed-expr-for-hk_runtime.hip']
#                                  ['sed-expr-for-hk_device.h'] ['sed-expr-for-hk_launch.h']
#   -> exp_lib/libhk_<name>.so (load it with HK_LIB, tools/ab.sh)
set -e
NAME=$1; KS=$2; RS=${3:-}; DS=${4:-}; LS=${5:-}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$R/exp_build/$NAME
rm -rf $T && mkdir -p $T
cp -r $R/include $T/include
mkdir -p $T/pkg && cp -r $R/bevy-hikari_amd/csrc $R/bevy-hikari_amd/Makefile $T/pkg/
[ -n "$KS" ] && sed -i "$KS" $T/pkg/csrc/hk_kernels.hip
[ -n "$RS" ] && sed -i "$RS" $T/pkg/csrc/hk_runtime.hip
[ -n "$DS" ] && sed -i "$DS" $T/pkg/csrc/hk_device.h
[ -n "$LS" ] && sed -i "$LS" $T/pkg/csrc/hk_launch.h
diff -q $R/bevy-hikari_amd/csrc/hk_kernels.hip $T/pkg/csrc/hk_kernels.hip > /dev/null && [ -z "$RS" ] && [ -z "$DS" ] && [ -z "$LS" ] && { echo "no edit applied"; exit 1; }
make -s -C $T/pkg -j8 OUT=libhk.so
mkdir -p $R/exp_lib && cp $T/pkg/libhk.so $R/exp_lib/libhk_$NAME.so
echo exp_lib/libhk_$NAME.so
