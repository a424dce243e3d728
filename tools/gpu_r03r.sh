# One GPU call: inflate parity (gpu parity + large offsets + stream + splits) on the in-tree
# library, then the inflate A/B in-tree vs lib_base (the previous commit) on B, D, E.
set -o pipefail
T=${1:-r03r}; shift
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
step abB 300 python -u tools/ab_inflate.py --records 4000000 $A/lib_v2.so $A/lib_sp.so
step abD 200 python -u tools/ab_inflate.py --config D --records 25000 $A/lib_v2.so
step abE 200 python -u tools/ab_inflate.py --config E --records 2000000 $A/lib_v2.so
