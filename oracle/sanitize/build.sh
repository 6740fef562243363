#!/bin/sh
# TEST INFRASTRUCTURE ONLY: the CPU restatement and the host emulation of the HIP
# path's in-place schedules under AddressSanitizer + UndefinedBehaviorSanitizer
# (SURVEY.md §5). Host code only: no GPU sanitizer is involved.
#   sh oracle/sanitize/build.sh [out]      -> oracle/sanitize/sanitize_bin
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=${1:-$HERE/sanitize_bin}
gcc -std=c11 -O1 -g -fopenmp -fno-omit-frame-pointer \
    -fsanitize=address,undefined -fno-sanitize-recover=all \
    -Wall -Wextra -Wno-unused-parameter \
    -o "$OUT" "$HERE/sanitize_main.c" "$HERE/../pmenv_oracle.c" -lm
echo "$OUT"
