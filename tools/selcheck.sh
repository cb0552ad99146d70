#!/bin/bash
# selcheck over the residual modes (tools/selcheck.hip); stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for args in "1000000 20 0 3.0" "1000000 10 0 0.95" "1000000 10 0 1.3" "100000 8 1 3.0" \
            "200000 8 2 3.0" "300000 8 3 0.95" "1000000 8 4 3.0" "1000000 8 5 3.0" "3000 8 0 3.0" "8000000 8 0 3.0"; do
    timeout -k 5 60 ./tools/selcheck $args || { echo "selcheck $args rc=$?"; exit 1; }
done
