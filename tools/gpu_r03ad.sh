# One GPU call: GPU suite on the in-tree library, inflate A/B vs the previous commit, and the
# bench step with the three-stream pipeline at 3 and 9 batches vs one batch.
set -o pipefail
T=${1:-r03ad}
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
A=spark-bam_amd/build/ab
step gputests 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step abB 300 python -u tools/ab_inflate.py --records 4000000 $A/lib_prevwalk.so
step bench1 200 python -u bench.py --no-cpu-baseline --no-full --no-e2e --steps 10
SBH_PIPE_MIN_BLOCKS=15283 step bench3 200 python -u bench.py --no-cpu-baseline --no-full --no-e2e --steps 10
SBH_PIPE_MIN_BLOCKS=5000 step bench9 200 python -u bench.py --no-cpu-baseline --no-full --no-e2e --steps 10
