set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4final
mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench_stderr.txt || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/kt.err
