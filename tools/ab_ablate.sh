#!/bin/bash
set -u
for v in 0 1 3 4 0; do
  echo "== AANET_ABLATE=$v"
  AANET_ABLATE=$v timeout -k 10 300 python tools/conv_microbench.py 20 conv3x3,dcn,offset_conv,conv1x1 || exit $?
done
