#!/bin/bash
# Build round_amd/<name>.so for A/B runs (PSG_LIB=round_amd/<name>.so).
#   scripts/build_variant.sh NAME [GIT_REF|-] [extra HIPFLAGS...]
# GIT_REF: build the kernels of that commit (e.g. HEAD = the last commit); "-": the working tree.
set -e
NAME=$1; REF=${2:--}; shift 2 || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT
if [ "$REF" != "-" ]; then
  SRC=$(mktemp -d /tmp/psgv.XXXX)
  git -C "$ROOT" archive "$REF" round_amd/csrc include | tar -x -C "$SRC"
fi
make -s -j8 -C "$SRC/round_amd/csrc" OUT="$ROOT/round_amd/$NAME.so" BUILD="$ROOT/build/ab_$NAME" \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*"
[ "$REF" != "-" ] && rm -rf "$SRC"
echo "built round_amd/$NAME.so"
