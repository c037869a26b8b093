#!/bin/bash
# Build the committed (HEAD, or REV=<rev>) library (kernels and host code) as sam2consensus_amd/libs2c_prev.so — the "before" side
# of an A/B on the GPU box (scripts/run.sh ab:WL with LIBS="libs2c.so libs2c_prev.so").
set -e
cd "$(dirname "$0")/.."
T=$(mktemp -d)
S=$T/sam2consensus_amd/csrc
mkdir -p $S $T/include
K="s2c_dense s2c_tile s2c_reads"
git cat-file -e ${REV:-HEAD}:sam2consensus_amd/csrc/s2c_bodies.hip 2>/dev/null && K="$K s2c_bodies"   # (ABI 14+)
for f in s2c_common.h s2c_host.cpp s2c_synth.cpp; do git show ${REV:-HEAD}:sam2consensus_amd/csrc/$f > $S/$f; done
for k in $K; do git show ${REV:-HEAD}:sam2consensus_amd/csrc/$k.hip > $S/$k.hip; done
git show ${REV:-HEAD}:include/s2c.h > $T/include/s2c.h
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$T/include -Wno-unused-result"
for k in $K; do /opt/rocm/bin/hipcc $F -c $S/$k.hip -o $T/$k.o & done
for k in s2c_host s2c_synth; do g++ -O3 -std=c++17 -fPIC -pthread -I$T/include -c $S/$k.cpp -o $T/$k.o & done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $T/s2c_host.o $T/s2c_synth.o $(for k in $K; do echo $T/$k.o; done) -lz -lpthread -o sam2consensus_amd/libs2c_prev.so
rm -rf $T
echo built sam2consensus_amd/libs2c_prev.so
