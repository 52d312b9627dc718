set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4final
mkdir -p $O
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- python3 $B --no-bfgs > /dev/null 2> $O/fetch.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o run -- python3 $B --no-bfgs > /dev/null 2> $O/write.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 -f csv -d $O/f64 -o run -- python3 $B --no-bfgs > /dev/null 2> $O/f64.err || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 -f csv -d $O/f64b -o run -- python3 profiles/r04/bfgs_only.py > $O/bfgs_only.json 2> $O/f64b.err || exit $?
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES"
timeout -s KILL 200 rocprofv3 --pmc $SQ -f csv -d $O/sq_c3 -o run -- python3 profiles/r04/variant_bench.py --one c3 3 > /dev/null 2> $O/sq_c3.err || exit $?
timeout -s KILL 200 rocprofv3 --pmc $SQ -f csv -d $O/sq_c4 -o run -- python3 profiles/r04/variant_bench.py --one c4 3 > /dev/null 2> $O/sq_c4.err
