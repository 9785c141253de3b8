#!/bin/bash
# Dev helper: s_memtime stamp builds of the hand-placed forward (-DFA2_HP_STAMPS=1), each
# NAME=ABL1+ABL2 argument regenerated with FA2_HPGEN_ABL (fw_* timing ablations of the class-A
# period: wrong outputs, cycles only) -> ab_libs/st_NAME.so; only api.hip and the bf16 D = 128
# forward unit are recompiled, the default headers are restored (mtimes kept) at the end.
# usage: bash scripts/fwd_stamp_abl.sh base= nodma=fw_nodma novalu=fw_novalu+fw_nodma
#        then (GPU) python scripts/hp_stamps.py ab_libs/st_base.so ab_libs/st_nodma.so ...
set -e
python -m fa2_triton_amd.build > /dev/null
SAVE=$(mktemp -d); cp -p fa2_triton_amd/csrc/gen/*_hp_body.h $SAVE/
trap 'cp -p $SAVE/*_hp_body.h fa2_triton_amd/csrc/gen/; rm -rf $SAVE' EXIT
for spec in "$@"; do
  NAME=st_${spec%%=*}; ABL=${spec#*=}; ABL=${ABL//+/,}
  D=$PWD/ab_libs/$NAME
  rm -rf $D && mkdir -p $D && cp -p fa2_triton_amd/_build/*.o $D/
  rm -f $D/api.o $D/fwd_bf16_d128.o
  FA2_HPGEN_ABL=$ABL python -m fa2_triton_amd.hp_gen > /dev/null
  FA2_HIPCC_FLAGS=-DFA2_HP_STAMPS=1 FA2_HPGEN_ABL=$ABL FA2_BUILD_ONLY=api,fwd_bf16_d128 FA2_BUILD_DIR=$D \
    FA2_LIB_OUT=$PWD/ab_libs/$NAME.so python -m fa2_triton_amd.build -j 8 > /dev/null
  rm -rf $D
  echo "ab_libs/$NAME.so ($ABL)"
done
