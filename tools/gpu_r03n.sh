# One GPU call: PMC passes at HEAD (tools/pmc_collect.sh), the whole -m gpu suite, smoke(),
# the default bench line and its kernel-trace summary.
set -o pipefail
T=${1:-r03n}
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pmc 600 bash tools/pmc_collect.sh gpurun_out/${T}_pmc
step gputests 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python -u bench.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step bprof 300 rocprofv3 --kernel-trace --stats -d /tmp/${T}_bprof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-full --no-e2e
python3 tools/prof_stats.py "$(find /tmp/${T}_bprof -name '*.db' -print -quit)" > gpurun_out/${T}_kernel_stats.csv
