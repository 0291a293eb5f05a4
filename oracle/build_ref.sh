#!/bin/bash
# TEST INFRASTRUCTURE ONLY. Builds the reference's own host code into oracle/_ref/ (git- but
# not gpurun-ignored) from the sources where they lie under $REF (default /root/reference).
#
# What is compiled from the reference, unmodified:
#   * src/gridscheduler.c (whole file, its own header);
#   * qrdecomp.c with two ranges of lines left out: line 15 (`#include "include/cycle.h"`,
#     a header that exists neither in the reference nor in this image) and lines 27-230
#     (main, tiledQR and taskQRP_threads, the only functions that use cycle.h's rdtsc
#     `ticks`/`getticks`, and tiledQR also calls the CUDA entry point). No stand-in header is
#     written; the source is piped to gcc, never copied into the repository. oracle/ref_harness.c
#     re-does taskQRP_threads' thread setup around the reference's own pthr_doTasks.
#   * libref_*_fix: the same plus the one-line fix of qrdecomp.c:506 (`j < 32` -> `j < n`),
#     without which the reference GEQRT is wrong for every tile size but 32.
# fp64 = the unmodified source with -Dfloat=double.
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
[ -f "$REF/qrdecomp.c" ] || { echo "build_ref: no reference at $REF, skipping"; exit 0; }
mkdir -p "$OUT"
CFLAGS="-O2 -ffp-contract=off -fPIC -w"
build() { # name fix(0/1) extra-cflags
    local name=$1 fix=$2 extra=$3
    local -a script=(-e '15d' -e '27,230d')
    [ "$fix" = 1 ] && script+=(-e '506s/j < 32/j < n/')
    sed "${script[@]}" "$REF/qrdecomp.c" | gcc -x c $CFLAGS $extra -I"$REF" -c - -o "$OUT/$name.qr.o"
    gcc $CFLAGS $extra -c "$REF/src/gridscheduler.c" -o "$OUT/$name.gs.o"
    gcc $CFLAGS $extra -I"$REF" -c "$HERE/ref_harness.c" -o "$OUT/$name.h.o"
    gcc -shared -o "$OUT/lib$name.so" "$OUT/$name.qr.o" "$OUT/$name.gs.o" "$OUT/$name.h.o" -lm -lpthread
    rm -f "$OUT/$name".*.o
}
build ref_f32     0 ""
build ref_f64     0 "-Dfloat=double"
build ref_f32_fix 1 ""
build ref_f64_fix 1 "-Dfloat=double"
echo "build_ref: built $(ls "$OUT"/*.so | wc -l) libraries in $OUT"
