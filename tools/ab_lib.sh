#!/bin/bash
# A/B of variant builds of the library (tools/build.py --variant NAME DEFS):
# for each LIB:ENV pair, the on-device C4 verify time (tools/sweep_modes.py).
#   LIBS="libbgv.so: libbgv_mw2.so:BGV_PAIRS=1" bash tools/ab_lib.sh
set -e
mkdir -p gpurun_out
for spec in $LIBS; do
  lib=${spec%%:*}; envs=${spec#*:}
  ( export BGV_LIB=$PWD/lodestar_amd/$lib; [ -n "$envs" ] && export ${envs//,/ };
    timeout -k 10 300 python -u tools/sweep_modes.py --sizes ${SIZES:-100352} --modes default --reps 7 | sed "s|^|$spec |" ) >> gpurun_out/ab.txt
done
