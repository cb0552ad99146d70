#!/bin/bash
# selcheck over the residual modes (tools/selcheck.hip); stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for args in "1000000 20 0 3.0" "1000000 10 0 0.95" "1000000 10 0 1.3" "100000 5 1 3.0" \
            "200000 3 2 3.0" "300000 3 3 0.95" "1000000 5 4 3.0" "1000000 5 5 3.0" "3000 5 0 3.0" "8000000 5 0 3.0"; do
    timeout -k 5 60 ./tools/selcheck $args || { echo "selcheck $args rc=$?"; exit 1; }
done
