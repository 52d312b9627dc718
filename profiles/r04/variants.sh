#!/bin/bash
# build a libmmadmm variant: variants.sh <name> "<extra flags>"  ->  dev/lib_<name>/libmmadmm.so
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
make -s -j8 -C "$ROOT/mm-admm_amd" "$ROOT/dev/lib_$1/libmmadmm.so" BUILD="$ROOT/dev/build_$1" LIB="$ROOT/dev/lib_$1/libmmadmm.so" EXTRA="$2"
