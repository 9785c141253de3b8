#!/bin/bash
# Dev helper: build ab_libs/NAME.so for each NAME=ABL1+ABL2 argument: the hand-placed streams
# regenerated with FA2_HPGEN_ABL (timing ablations, wrong outputs) and the units matching ONLY
# (default bwd_bf16_d128) recompiled; the default headers are restored (mtimes kept) at the end.
# usage: ONLY=bwd_bf16_d128 bash scripts/hpabl.sh base= novm=dk_novm nobar=dk_novm+dk_nobar
set -e
ONLY=${ONLY:-bwd_bf16_d128}
python -m fa2_triton_amd.build > /dev/null
SAVE=$(mktemp -d); cp -p fa2_triton_amd/csrc/gen/*_hp_body.h $SAVE/
trap 'cp -p $SAVE/*_hp_body.h fa2_triton_amd/csrc/gen/; rm -rf $SAVE' EXIT
for spec in "$@"; do
  NAME=${spec%%=*}; ABL=${spec#*=}; ABL=${ABL//+/,}
  D=ab_libs/$NAME
  rm -rf $D && mkdir -p $D && cp -p fa2_triton_amd/_build/*.o $D/
  for tok in ${ONLY//,/ }; do rm -f $D/*${tok}*.o; done
  FA2_HPGEN_ABL=$ABL python -m fa2_triton_amd.hp_gen > /dev/null
  FA2_HPGEN_ABL=$ABL FA2_BUILD_ONLY=$ONLY FA2_BUILD_DIR=$PWD/$D FA2_LIB_OUT=$PWD/ab_libs/$NAME.so \
    python -m fa2_triton_amd.build -j 8 > /dev/null
  rm -rf $D
  echo "ab_libs/$NAME.so ($ABL)"
done
