#!/bin/bash
# Twin of the in-tree libmidiseq.so with one source compiled under extra flags
# (ablation / diagnostic builds). usage: tools/build_var.sh <csrc/file.hip> <out.so> <flags...>
set -e
src=$1; out=$2; shift 2
P=deep-learning-based-sequence-models-for-music-generation_amd
tmp=$(mktemp -d /tmp/varXXXX)
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I include -Wno-unused-result "$@" -c "$P/$src" -o "$tmp/v.o"
objs=$(ls $P/build/*.o | grep -v "/$(basename $src).o$")
mkdir -p "$(dirname $out)"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$out" $objs "$tmp/v.o"
rm -rf "$tmp"
echo "built $out ($src $*)"
