cd $GRAFT_REPO_ROOT
for a in "1000000 20 0 3.0" "3000 5 0 3.0" "1000000 10 0 1.3"; do timeout -k 5 60 ./tools/selcheck $a || exit 1; done
