#!/bin/bash
# One library per process, interleaved rounds: tools/ab_proc.sh ROUNDS LIB.so...
# (in-process A/B of several libraries is biased by library position)
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for lib in "$@"; do
    timeout -k 10 300 python tools/ab_quad.py "$lib" 2>&1 | grep -v "amdgpu\|^round" || exit $?
  done
done
