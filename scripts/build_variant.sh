#!/usr/bin/env bash
# Build an A/B variant of libmvs.so: the in-tree sources with some files
# replaced.  scripts/build_variant.sh TAG ncc.hip=/path/to/variant.hip [...]
#   -> ab/libmvs_TAG.so  (NAME=PATH replaces csrc/NAME by PATH)
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; shift
T=$(mktemp -d /tmp/mvsvar.XXXX)
mkdir -p $T/cl_multiview_stereo_amd/host $T/include $T/tests/adapter
cp -r $ROOT/cl_multiview_stereo_amd/csrc $T/cl_multiview_stereo_amd/
cp $ROOT/cl_multiview_stereo_amd/host/* $T/cl_multiview_stereo_amd/host/
cp $ROOT/include/* $T/include/
for f in "$@"; do  # NAME=PATH: csrc/NAME, or include/NAME for an include/ header
  n="${f%%=*}"
  case $n in include/*) cp "${f#*=}" $T/"$n" ;; *) cp "${f#*=}" $T/cl_multiview_stereo_amd/csrc/"$n" ;; esac
done
make -s -j8 -C $T/cl_multiview_stereo_amd/csrc ../libmvs.so 2>&1 | grep -v dot6 || true
mkdir -p $ROOT/ab
cp $T/cl_multiview_stereo_amd/libmvs.so $ROOT/ab/libmvs_$TAG.so
rm -rf $T
echo "built ab/libmvs_$TAG.so"
