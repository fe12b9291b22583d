#!/bin/bash
# Time A/B library variants with one timing script (dev tool, runs on the GPU box):
#   tools/ab_run.sh <script.py> <variant> [<variant> ...]     (variant "default" = the in-tree build)
S=$1; shift
for v in "$@"; do
  if [ "$v" = default ]; then
    timeout -k 10 90 python "$S" || exit 1
  else
    QATTN_AB=$PWD/_ab/libqattn_$v.so timeout -k 10 90 python "$S" || exit 1
  fi
done
