#!/bin/bash
# Build the committed (HEAD, or REV=<rev>) library (kernels and host code) as sam2consensus_amd/libs2c_prev.so — the "before" side
# of an A/B on the GPU box (scripts/run.sh ab:WL with LIBS="libs2c.so libs2c_prev.so").
set -e
cd "$(dirname "$0")/.."
T=$(mktemp -d)
S=$T/sam2consensus_amd/csrc
mkdir -p $S $T/include
for f in s2c_dense.hip s2c_tile.hip s2c_reads.hip s2c_common.h s2c_host.cpp s2c_synth.cpp; do git show ${REV:-HEAD}:sam2consensus_amd/csrc/$f > $S/$f; done
git show ${REV:-HEAD}:include/s2c.h > $T/include/s2c.h
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$T/include -Wno-unused-result"
for k in s2c_dense s2c_tile s2c_reads; do /opt/rocm/bin/hipcc $F -c $S/$k.hip -o $T/$k.o & done
for k in s2c_host s2c_synth; do g++ -O3 -std=c++17 -fPIC -pthread -I$T/include -c $S/$k.cpp -o $T/$k.o & done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $T/s2c_host.o $T/s2c_synth.o $T/s2c_reads.o $T/s2c_tile.o $T/s2c_dense.o -lz -lpthread -o sam2consensus_amd/libs2c_prev.so
rm -rf $T
echo built sam2consensus_amd/libs2c_prev.so
