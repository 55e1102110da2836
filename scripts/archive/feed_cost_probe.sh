#!/bin/bash
# Where the H2D feed's ~4 % goes under the run-ahead bound: default feed vs augment-from-slots
# without copies (FEED=nocopy) vs no feeder at all (NOFEED=1), in-stream 10-step slices.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in "X=1" "FEED=nocopy" "NOFEED=1" "X=1" "FEED=nocopy" "NOFEED=1"; do
  env $v timeout -k 10 300 python scripts/stability.py 2>&1 | grep -E "chunks" | sed "s/^/$v /" || exit 1
done
