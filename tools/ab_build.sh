#!/bin/bash
# Build an A/B variant of libqattn.so with one source compiled under extra -D flags (dev tool).
#   tools/ab_build.sh <source.hip> <variant-name> [-DFOO=1 ...]   -> _ab/libqattn_<variant-name>.so
#   (<source.hip>: a file of csrc/, or a path to another version of one, e.g. from git show)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
SRC=$1; NAME=$2; shift 2
python3 -c "import sys; sys.path.insert(0, '$R'); from quantizedattention_amd import build; build.build(verbose=False)"
mkdir -p $R/_ab/obj
OBJ=$R/_ab/obj/$(basename $SRC .hip)_$NAME.o
case $SRC in /*) SRCP=$SRC ;; *) SRCP=$R/quantizedattention_amd/csrc/$SRC ;; esac
# the product build's per-source flags (build.FILE_FLAGS), so a variant differs only by "$@"
FF=$(python3 -c "import sys; sys.path.insert(0, '$R'); from quantizedattention_amd import build; print(' '.join(build.FILE_FLAGS.get('$(basename $SRC)', [])))")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt \
  -fno-gpu-rdc -Wno-unused-result -Wno-unused-value -I$R/include -I$R/quantizedattention_amd/csrc $FF "$@" -c $SRCP -o $OBJ
OTHERS=$(ls $R/quantizedattention_amd/_build/*.o | grep -v "/dev_" | grep -v "/$(basename $SRC .hip).o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/_ab/libqattn_$NAME.so $OTHERS $OBJ
echo "built _ab/libqattn_$NAME.so"
