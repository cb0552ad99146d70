#!/bin/bash
# wincheck over the residual modes (tools/wincheck.hip): the window selection path on
# every distribution, window size and threshold placement; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for args in "1000000 0 3.0" "1000000 0 0.95" "1000000 0 1.3" "100000 1 3.0" "200000 2 3.0" \
            "300000 3 0.95" "1000000 4 3.0" "1000000 5 3.0" "3000 0 3.0" "8000000 0 3.0" \
            "1000000 6 3.0" "1000000 7 3.0" "1000000 8 0.95"; do
    timeout -k 5 120 ./tools/wincheck $args || { echo "wincheck $args rc=$?"; exit 1; }
done
