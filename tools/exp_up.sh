#!/bin/bash
# Experiment build for upload: bash tools/exp_up.sh NAME "-DFLAG=1 ..." -> exp_up/NAME/lib
# (git-ignored, not gpurun-ignored: the box runs it with R3DG_LIB_DIR=exp_up/NAME/lib, e.g. via
# tools/ab_libs.sh TAG ROUNDS NAME=exp_up/NAME/lib). Objects go to exp/NAME/obj (not uploaded).
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2
rm -rf "exp/$NAME" "exp_up/$NAME"
R3DG_LIB_DIR=exp_up/$NAME/lib R3DG_OBJ_DIR=exp/$NAME/obj R3DG_EXTRA_HIPFLAGS="$FLAGS" python relightable3dgaussian_amd/build.py
