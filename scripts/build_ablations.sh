#!/bin/bash
# Timing-only variant builds of libdal.so with gram_split.hip compiled under
# extra defines, into build/<name>/libdal.so (the other objects are the
# product build's).  usage: build_ablations.sh name1 "-DX=1" [name2 "-DY=2" ...]
# e.g. ablations of the super-block Gram: abl3 "-DDAL_SYM2_ABL=3" (results WRONG).
set -e
cd "$(dirname "$0")/../distributed-active-learning_amd/csrc"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  d=../../build/$name
  mkdir -p $d/obj
  for f in abi normalize gram forest topk maxcos ingest rf_train plan; do cp ../../build/csrc/$f.o $d/obj/$f.o; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include \
    $defs -c gram_split.hip -o $d/obj/gram_split.o &
done
wait
cd ../../build
for d in */obj; do
  n=${d%/obj}
  [ -f $n/obj/gram_split.o ] && /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $n/libdal.so $n/obj/*.o
done
