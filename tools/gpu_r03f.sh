# One GPU call: parity of the in-tree build, inflate checkpoint A/B, k_full word-batching A/B,
# then the streaming / split / sharded / CLI / >2 GiB tests (host-path splits printed).
# A step that fails its tests (exit 1) lets the next run; any other status ends the script.
set -o pipefail
T=${1:-r03f}
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
step parity 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread
step abinfl 300 python -u tools/ab_inflate.py --records 4000000 $A/lib_ck0.so $A/lib_ck48.so $A/lib_ck96.so $A/lib_ck128.so
step abfull 240 bash -c "for l in '' $A/lib_fbase.so $A/lib_g2o5.so $A/lib_g4o4.so $A/lib_g8o4.so; do SBH_LIB_PATH=\$l python -u tools/full_ab.py --records 4000000 --rtc 10 || exit \$?; done"
SBH_SPLIT_DEBUG=1 step tests 400 python -u -m pytest tests/test_stream_gpu.py tests/test_splits_gpu.py tests/test_sharded.py tests/test_cli.py tests/test_large_comp_offsets_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread
