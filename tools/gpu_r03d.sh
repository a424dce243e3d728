# One GPU call: inflate parity with the current k_huff, inflate A/B (in-tree: two chains per lane + literal pairs, vs each alone),
# k_full replica A/B, then the streaming / split / sharded / CLI / >2 GiB tests.
# A step that fails its tests (exit 1) lets the next run; any other status (fault, abort,
# time limit) ends the script.  usage (on the box): bash tools/gpu_r03d.sh TAG
set -o pipefail
T=${1:-r03d}
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step parity 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread
step abinfl 300 python -u tools/ab_inflate.py --records 4000000 spark-bam_amd/build/ab/lib_i2l0.so spark-bam_amd/build/ab/lib_i1l2.so spark-bam_amd/build/ab/lib_ilp1.so
step abfull 300 bash -c 'for l in "" spark-bam_amd/build/ab/lib_fnh.so spark-bam_amd/build/ab/lib_r8.so spark-bam_amd/build/ab/lib_r16.so; do SBH_LIB_PATH=$l python -u tools/full_ab.py --records 4000000 --rtc 10 || exit $?; done'
