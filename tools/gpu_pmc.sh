#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM -d $R/gpurun_out/pmc/a -o run --output-format csv -- python3 $R/tools/pmc_probe.py pset_ml2 > $R/gpurun_out/pmc/a.log 2>&1 || { tail -20 $R/gpurun_out/pmc/a.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH -d $R/gpurun_out/pmc/b -o run --output-format csv -- python3 $R/tools/pmc_probe.py pset_ml2 > $R/gpurun_out/pmc/b.log 2>&1 || { tail -20 $R/gpurun_out/pmc/b.log; exit 1; }
find $R/gpurun_out/pmc -name "*.csv" | head
