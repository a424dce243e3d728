# One GPU call: the streaming / split / sharded / CLI / >2 GiB tests, then the default bench
# line (config B, N=1) and its rocprofv3 kernel-trace summary.
set -o pipefail
T=${1:-r03g}
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
SBH_SPLIT_DEBUG=1 step tests 500 python -u -m pytest tests/test_stream_gpu.py tests/test_splits_gpu.py tests/test_sharded.py tests/test_cli.py tests/test_large_comp_offsets_gpu.py -m gpu -x -v -s --timeout 400 --timeout-method thread
step bench 300 python -u bench.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step bprof 300 rocprofv3 --kernel-trace --stats -d /tmp/${T}_bprof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-full --no-e2e
python3 tools/prof_stats.py "$(find /tmp/${T}_bprof -name '*.db' -print -quit)" > gpurun_out/${T}_kernel_stats.csv
