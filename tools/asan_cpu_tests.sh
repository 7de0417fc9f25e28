#!/bin/bash
# The CPU test suite against a host-sanitizer build of libmpi.so (AddressSanitizer + UBSan on the
# host C++; the device objects are the regular ones and no GPU code runs).  Here only, not on the
# GPU box: gcc's sanitizer runtimes are preloaded into python, the library is picked through
# MV2AMD_LIBMPI.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -C "$ROOT/mvapich2_amd/csrc" asan -j8
cd /tmp
LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" \
ASAN_OPTIONS=detect_leaks=0 MV2AMD_LIBMPI="$ROOT/build/asan/libmpi.so" \
  python -m pytest "$ROOT/tests" -x -q -m "not gpu" -p no:cacheprovider "$@"
