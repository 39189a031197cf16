#!/bin/bash
# PMC passes over tools/scatter_probe.py (main library only), one counter group per pass
# (summarise: python3 tools/pmc_summary.py gpurun_out/pmc_scatter field_scatter)
export TMPDIR=/tmp SCATTER_PROBE_MAIN_ONLY=1
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_scatter/p$i -o p -- python3 tools/scatter_probe.py > gpurun_out/pmc_scatter_$i.log 2>&1 || exit $?
done
