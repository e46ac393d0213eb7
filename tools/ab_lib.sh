#!/bin/bash
# A/B of variant builds of the library (tools/build.py --variant NAME DEFS):
# for each LIB[:MODE] entry, the on-device C4 verify time (tools/sweep_modes.py,
# MODE one of its bgv_cfg override sets, default "default").
#   LIBS="libbgv.so libbgv_mw2.so:serial" bash tools/ab_lib.sh
set -e
mkdir -p gpurun_out
for spec in $LIBS; do
  lib=${spec%%:*}; mode=default
  [ "$spec" != "$lib" ] && mode=${spec#*:}
  ( export BGV_LIB=$PWD/lodestar_amd/$lib;
    timeout -k 10 300 python -u tools/sweep_modes.py --sizes ${SIZES:-100352} --modes $mode --reps 7 | sed "s|^|$spec |" ) >> gpurun_out/ab.txt
done
