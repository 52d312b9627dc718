#!/bin/bash
# SQ stall counters of the C4 prox (one rocprofv3 pass): dev/pmc_sq.sh OUTDIR [LIB]
mkdir -p gpurun_out
[ -n "$2" ] && export MMADMM_LIB=$PWD/dev/$2/libmmadmm.so
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d $GRAFT_REPO_ROOT/gpurun_out/$1 -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/profiles/r02/prox_time.py
