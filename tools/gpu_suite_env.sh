#!/bin/bash
# The GPU suite under an environment setting, repeated: gpurun -- bash tools/gpu_suite_env.sh <tag> <runs> VAR=VALUE ...
# A run whose tests fail (pytest exit 1) does not stop the next; anything else (a time limit,
# a crash, an abort) ends the script there.  PYTEST_EXTRA adds pytest options; STOP_ON_FAIL=1
# ends the repeats at the first failing run.
set -o pipefail
tag=${1:-run}
runs=${2:-1}
shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for kv in "$@"; do export "${kv?}"; done
for i in $(seq 1 "$runs"); do
  timeout -k 10 400 python -u -m pytest tests -m gpu -v ${PYTEST_EXTRA:-} --timeout 120 --timeout-method thread \
    > "gpurun_out/suite_${tag}_${i}.txt" 2>&1
  rc=$?
  echo "run $i: exit $rc; $(tail -1 "gpurun_out/suite_${tag}_${i}.txt")"
  grep -E "^(FAILED|ERROR)|bytes differ" "gpurun_out/suite_${tag}_${i}.txt" | head -20
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  [ $rc -eq 1 ] && [ -n "${STOP_ON_FAIL:-}" ] && break
done
exit 0
