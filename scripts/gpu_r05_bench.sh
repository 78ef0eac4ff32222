#!/bin/bash
# The default bench line (as the driver runs it) and the rocprofv3 kernel stats of the same command.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05_final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-400
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run --output-format csv -- python3 -u bench.py --no-e2e > $O/bench_prof.json 2> $O/bench_prof.err || { tail -5 $O/bench_prof.err; exit 1; }
cp $(find $O/prof_default -name 'run_kernel_stats.csv' | head -1) $O/kernel_stats_default_bench.csv
rm -rf $O/prof_default
