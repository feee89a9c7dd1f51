#!/bin/bash
# Host AddressSanitizer + UndefinedBehaviorSanitizer build of the pool-ingest
# parser (csrc/ingest.hip, host code only) with its driver
# (scripts/asan/ingest_asan_driver.cpp).  CPU only: host compilation
# (--cuda-host-only), each -fsanitize= after -Xarch_host, nothing for the GPU.
#
#   bash scripts/asan/build.sh [OUT]      (default build/asan/ingest_asan_driver)
#
# Run the checks: python -m pytest tests/test_ingest_asan.py -v
set -euo pipefail
REPO="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="${1:-$REPO/build/asan/ingest_asan_driver}"
mkdir -p "$(dirname "$OUT")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN=(-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all)
"$HIPCC" -x hip --cuda-host-only --offload-arch=gfx950 -O1 -g -fno-omit-frame-pointer -std=c++17 "${SAN[@]}" \
  -I"$REPO/include" -c "$REPO/distributed-active-learning_amd/csrc/ingest.hip" -o "$OUT.ingest.o"
"$HIPCC" -x c++ -O1 -g -fno-omit-frame-pointer -std=c++17 "${SAN[@]}" -I"$REPO/include" \
  -c "$REPO/scripts/asan/ingest_asan_driver.cpp" -o "$OUT.driver.o"
"$HIPCC" "${SAN[@]}" -o "$OUT" "$OUT.driver.o" "$OUT.ingest.o" -lpthread
echo "$OUT"
