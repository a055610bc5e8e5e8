#!/usr/bin/env bash
# k_schur / LM step of config 3 under the camera-major observation orders and Schur work orders, each in its own
# process (the switches are read once per process).  usage: tools/order_probe.sh ORDER:XCD[:CHUNK] ...
#   ORDER = INSFM_SCHUR_ORDER (0 partner count, 1 point-order chunks), XCD = INSFM_SCHUR_XCD (rows per XCD run),
#   CHUNK = INSFM_SCHUR_CHUNK (k_schur rounds per chunk)
set -e
cd "$(dirname "$0")/.."
for spec in "$@"; do
  IFS=: read -r o x c <<< "$spec"
  echo -n "order=$o xcd=$x chunk=${c:-4}  "
  INSFM_SCHUR_ORDER=$o INSFM_SCHUR_XCD=$x INSFM_SCHUR_CHUNK=${c:-4} timeout -k 10 150 python -u tools/schur_probe.py 2>&1 | grep -v amdgpu.ids
done
