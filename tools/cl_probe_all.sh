#!/bin/bash
# cluster_probe.py over the NCN_DIAG_CL_TIMES builds in tools/_build (one line of totals each)
for so in tools/_build/lib_ncn_diag_cl_times*.so; do
  echo "== $so"
  NCN_CL_PROBE_SO=$so timeout -k 10 60 python tools/cluster_probe.py | grep -E "compaction|it  5|it 15|total|end" || exit $?
done
