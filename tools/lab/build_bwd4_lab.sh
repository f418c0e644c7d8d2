#!/bin/bash
# Builds tools/lab/attn_bwd4_lab (v3 vs v4 key/value pass comparison + timing);
# extra arguments go to the v4 compile (e.g. -DKV4_SCHED=1), $OUT names the binary
set -e
cd "$(dirname "$0")/../.."
C=deep-learning-based-sequence-models-for-music-generation_amd/csrc
OUT=${OUT:-tools/lab/attn_bwd4_lab}
[ -f /tmp/kv3_lab.o ] || hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -c $C/attn_bwd3.hip -o /tmp/kv3_lab.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include "$@" -c tools/lab/attn_bwd4_lab.hip -o /tmp/kv4_lab_$$.o
hipcc --offload-arch=gfx950 /tmp/kv4_lab_$$.o /tmp/kv3_lab.o -o $OUT
