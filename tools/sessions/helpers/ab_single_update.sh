#!/bin/bash
# A/B of tools/time_single_update.py over variant libraries.
set -u
for v in "$@"; do
  echo -n "$v: "
  UWVK_LIB=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so timeout -k 10 200 python tools/time_single_update.py || exit 1
done
