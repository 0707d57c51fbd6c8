#!/bin/bash
# Experiment build: bash tools/exp_build.sh NAME "-DFLAG=1 ..." -> exp/NAME/lib/{libr3dg_hip.so,_C.so}
# Run against it with R3DG_LIB_DIR=exp/NAME/lib (timing-only variants; results may be invalid).
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2
rm -rf "exp/$NAME"  # build.py rebuilds by source mtime only: a flag change needs a clean directory
R3DG_LIB_DIR=exp/$NAME/lib R3DG_OBJ_DIR=exp/$NAME/obj R3DG_EXTRA_HIPFLAGS="$FLAGS" python relightable3dgaussian_amd/build.py
