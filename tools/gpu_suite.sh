#!/bin/bash
# The GPU test suite and smoke() on the box, each under its own time limit; logs under
# gpurun_out/suite_<tag>/.   gpurun -- bash tools/gpu_suite.sh <tag> [pytest -k expression]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-run}; O=gpurun_out/suite_$tag; mkdir -p "$O"
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$O/pytest_gpu.txt" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 && tail -1 "$O/smoke.txt"
