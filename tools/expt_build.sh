#!/bin/bash
# Build alternative variants of libmdqt.so for kernel A/B timing (not the product build).
#   tools/expt_build.sh name "EXTRA flags" [name "flags" ...]  ->  expt/<name>/lib/libmdqt.so
# (FORCESFLAGS=... / QTSCHED=... in the environment override those files' own flags)
# Run a variant with MDQT_LIB=expt/<name>/lib/libmdqt.so python bench.py ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -s -C "$ROOT/mdqtplasmasims_amd/csrc" -j4 "$ROOT/expt/$name/lib/libmdqt.so" \
    OBJDIR="$ROOT/expt/$name/obj" LIBDIR="$ROOT/expt/$name/lib" EXTRA="$flags" ${FORCESFLAGS+FORCESFLAGS="$FORCESFLAGS"} ${QTSCHED+QTSCHED="$QTSCHED"}
done
