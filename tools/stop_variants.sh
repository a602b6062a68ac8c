#!/bin/bash
# Build the -DMPCR_STOP_AFTER=k attribution variants (CPU container).
cd "$(dirname "$0")/.."
for k in 0 1 2 3 4 5 6 7 8 13 9; do
  python tools/build_variant.py stop$k -DMPCR_STOP_AFTER=$k > /dev/null || exit 1
done
python tools/build_variant.py full > /dev/null
ls build_variants/
