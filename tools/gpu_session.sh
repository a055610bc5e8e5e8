#!/usr/bin/env bash
# Run GPU steps in order, each under its own time limit; stop at the first fault-class exit
# (abort 134, segfault 139, timeout 124/137) so nothing else touches the GPU after a fault.
# usage: tools/gpu_session.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
status=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 15 "gpurun_out/$name.log"
  case $rc in
    0) ;;
    134|139|124|137|136|135) echo "fault-class exit $rc: stopping the session"; exit $rc ;;
    *) status=$rc ;;
  esac
done
exit $status
