#!/bin/bash
# Build library variants (compile-time geometry knobs) as lib/libimgrec_<name>.so.
# Usage: bash tools/build_variants.sh name1 "flags1" name2 "flags2" ...
set -eu
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  IMGREC_EXTRA_FLAGS="$flags" IMGREC_OBJ_SUFFIX="_$name" IMGREC_LIB_NAME="libimgrec_$name.so" \
    python -m image_recommender_amd.build --jobs 4 2>&1 | tail -1
done
