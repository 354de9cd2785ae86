#!/bin/bash
# GPU test pass: pytest -m gpu (optionally a subset: PYTEST_TARGETS), each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-tests}
mkdir -p "$OUT"
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_TARGETS:-tests} -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -15 "$OUT/pytest_gpu.log"
exit $rc
