#!/bin/bash
# time the clustering kernel of every tools/_build/lib_ncn_diag_cl_times*.so (tools/cluster_probe.py)
for so in tools/_build/lib_ncn_diag_cl_times*.so; do
  echo "== $so"
  NCN_CL_PROBE_SO=$so timeout -k 10 60 python tools/cluster_probe.py 2>&1 | grep -E "compaction |it  0|it 10|^total" || exit $?
done
