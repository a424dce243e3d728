# One GPU call: inflate parity with predicated stream reloads, the A/B, and the phase probe.
set -o pipefail
T=${1:-r03m}
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
A=spark-bam_amd/build/ab
step parity 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread
step abinfl 300 python -u tools/ab_inflate.py --records 4000000 $A/lib_nx0.so $A/lib_hp.so $A/lib_lzp.so
step abinflD 200 python -u tools/ab_inflate.py --config D --records 25000 $A/lib_nx0.so
