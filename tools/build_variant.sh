#!/bin/bash
# Build a variant of libficp.so with extra compile flags, for A/B runs through FICP_LIB:
# usage: tools/build_variant.sh <name> <flags...>  ->  tools/abv/libficp_<name>.so (objects in tools/ab/)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=tools/ab/build_$name
mkdir -p $out tools/abv
# VARIANT_SRC=<dir>: build from another copy of csrc (e.g. a git checkout of an older round)
cd "${VARIANT_SRC:-coregistrationgame_amd/csrc}"
SRCS=$(sed -n 's/^SRCS = //p' Makefile)
pids=""
for f in $SRCS; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-fast-math \
    -I"$OLDPWD/include" "$@" -c $f -o "$OLDPWD/$out/${f%.hip}.o" &
  pids="$pids $!"
done
for p in $pids; do wait $p || { echo "compile failed"; exit 1; }; done
cd "$OLDPWD"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o tools/abv/libficp_$name.so $out/*.o
echo tools/abv/libficp_$name.so
