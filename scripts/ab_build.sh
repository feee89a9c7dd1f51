#!/bin/bash
# Build an A/B variant of libdal.so into ab/NAME/libdal.so (objects in
# build/ab_NAME), with extra compile flags (tuning-constant overrides), from
# the in-tree sources; the product library is untouched.
#   bash scripts/ab_build.sh NAME "-DDAL_X=1 -DDAL_Y=2"
set -eu
name=$1
extra=${2:-}
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/ab/$name"
make -s -C "$root/distributed-active-learning_amd/csrc" -j8 OUT="$root/ab/$name/libdal.so" \
  OBJDIR="$root/build/ab_$name" EXTRA="$extra"
echo "built ab/$name/libdal.so ($extra)"
