#!/bin/bash
# kernel trace + PMC passes (one counter group per run) over tools/gat_fwd_probe.py
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_gatfwd
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/gat_fwd_probe.py > $O/trace.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 $R/tools/gat_fwd_probe.py > $O/fetch.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python3 $R/tools/gat_fwd_probe.py > $O/write.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace --output-format csv -d $O/waves -o run -- python3 $R/tools/gat_fwd_probe.py > $O/waves.log 2>&1
rc=$?
echo pmc_rc=$rc
exit $rc
