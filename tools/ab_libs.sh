#!/usr/bin/env bash
# Same-box A/B of library builds: alternates tools/schur_probe.py (config-3 k_schur time and LM step time) over the
# in-tree library ("default") and tools/lib_<name>.so builds, `rounds` times.  usage: tools/ab_libs.sh rounds name...
set -e
cd "$(dirname "$0")/.."
rounds=$1; shift
for r in $(seq "$rounds"); do
  timeout -k 10 120 python -u tools/schur_probe.py
  for v in "$@"; do
    INSFM_LIB=tools/lib_$v.so timeout -k 10 120 python -u tools/schur_probe.py
  done
done
