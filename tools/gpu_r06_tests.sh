#!/bin/bash
# Round 6: run the given pytest node ids (the -m gpu suite's new / changed tests) on the box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LOG=gpurun_out/${TESTLOG:-r06_tests}.log
timeout -k 10 ${TESTTIME:-1100} python -u -m pytest -m gpu ${XFLAG--x} -v -p no:cacheprovider --timeout 450 \
  --timeout-method thread "$@" > "$LOG" 2>&1; rc=$?
tail -25 "$LOG"
exit $rc
