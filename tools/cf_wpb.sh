#!/bin/bash
# composite kernels with 1/2/4/8/16 waves (rays) per workgroup (tools/build_loss_variants.sh CF_WPB=...)
for so in normal-clustering-nerf_amd/ncnerf_amd/libncnerf.so tools/_build/lib_cf_wpb_*.so; do
  echo "== $so"
  NCN_LIB_PATH=$PWD/$so timeout -k 10 100 python tools/composite_lab.py 8192 , 2>&1 | grep -E "^main" || exit $?
done
