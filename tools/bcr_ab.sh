#!/bin/bash
# timing experiments of the BCR elimination loop (PLBA_DIAG bits; results are wrong in 16/32)
set -eo pipefail
for dg in 8 24 40 56; do
  echo "== PLBA_DIAG=$dg"
  PLBA_DIAG=$dg timeout -k 5 120 python tools/bcr_stamps.py ${1:-C3} | sed -n '2,4p'
done
