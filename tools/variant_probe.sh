#!/usr/bin/env bash
# tools/schur_probe.py (config 3: k_schur and the LM step) once per environment setting, each in its own process.
# usage: tools/variant_probe.sh "NAME=VAL NAME2=VAL2" "..."   ("-" = defaults)
set -e
cd "$(dirname "$0")/.."
for spec in "$@"; do
  echo -n "[$spec]  "
  if [ "$spec" = "-" ]; then spec=""; fi
  env $spec timeout -k 10 150 python -u tools/schur_probe.py 2>&1 | grep -v amdgpu.ids
done
