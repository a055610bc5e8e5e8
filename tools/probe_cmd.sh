set -e
for v in "$@"; do
  INSFM_LIB=tools/lib_$v.so timeout -k 10 120 python -u tools/schur_probe.py
done
