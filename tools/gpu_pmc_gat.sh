#!/bin/bash
# PMC passes (one counter group per run) over tools/gat_h8_probe.py: wave-state breakdown
# of the 8-head GAT forward vs the weighted SpMM of the same shape.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_gat -o run -- python3 $R/tools/gat_h8_probe.py > $R/gpurun_out/pmc_gat.log 2>&1
