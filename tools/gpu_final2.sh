# One GPU call: bench lines for configs D and E, and the strong-scaling configs[2] line (ONE
# 100.9 GiB file on this GPU).  usage: bash tools/gpu_final2.sh TAG
set -o pipefail
T=${1:-r03final}
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step benchD 300 python -u bench.py --config D --no-cpu-baseline --no-full --no-e2e
step benchE 300 python -u bench.py --config E --no-cpu-baseline --no-full --no-e2e
step strongC 700 python -u bench.py --config C --file-gib 100 --steps 2 --warmup 1 --no-cpu-baseline
