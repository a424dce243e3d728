# One GPU call: the GPU suite on the in-tree library, then the inflate A/B in-tree vs the named
# variants on configs B, D and E.   usage: bash tools/gpu_r03af.sh TAG v1 ...
set -o pipefail
T=${1:-r03af}; shift
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
L=""
for v in "$@"; do L="$L spark-bam_amd/build/ab/lib_$v.so"; done
step gputests 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step abB 300 python -u tools/ab_inflate.py --records 4000000 $L
step abD 200 python -u tools/ab_inflate.py --config D --records 25000 $L
step abE 200 python -u tools/ab_inflate.py --config E --records 2000000 $L
