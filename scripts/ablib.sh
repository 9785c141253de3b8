#!/bin/bash
# Dev helper: build ab_libs/NAME.so = the in-tree objects with the units matching ONLY
# (default fwd_bf16_d128) recompiled under extra hipcc FLAGS.  usage: ablib.sh NAME "FLAGS" [ONLY]
set -e
NAME=$1; FLAGS=$2; ONLY=${3:-fwd_bf16_d128}
D=ab_libs/$NAME
rm -rf $D && mkdir -p $D && cp -p fa2_triton_amd/_build/*.o $D/
for tok in ${ONLY//,/ }; do rm -f $D/*${tok}*.o; done
FA2_BUILD_ONLY=$ONLY FA2_HIPCC_FLAGS="$FLAGS" FA2_BUILD_DIR=$PWD/$D FA2_LIB_OUT=$PWD/ab_libs/$NAME.so python -m fa2_triton_amd.build -j 8 > /dev/null
ls -la ab_libs/$NAME.so
