#!/bin/bash
# Build an A/B variant of the checksum library (libaws-checksums-amd.so) into ab/lib<NAME>.so with extra compile flags (own build dir).
#   scripts/build_variant.sh B "-DAMDCRC_LIST_STREAM=0"
set -e
cd "$(dirname "$0")/../aws-crt-cpp_amd"
n=$1; shift
rm -rf build_$n  # make does not track flags: a variant dir left from other flags would be reused
make -s -j8 BUILD=build_$n ENGINE=../ab/lib$n.so HIPFLAGS_EXTRA="-DAMDCRC_VARIANT_BUILD=1 $*" ../ab/lib$n.so
