#!/bin/bash
# kernel trace + PMC FETCH_SIZE / WRITE_SIZE passes over tools/rmat_spmm_probe.py
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_rmat
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/rmat_spmm_probe.py > $O/trace.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 $R/tools/rmat_spmm_probe.py > $O/fetch.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python3 $R/tools/rmat_spmm_probe.py > $O/write.log 2>&1
rc=$?
echo pmc_rc=$rc
exit $rc
