# round 5: the chain proof with overlapped round trips (k_verify_chain_b, build/ab/lib_vb8.so and
# lib_vb4.so) -- its chain / count tests against the oracle first, then kernel traces of the bench
# step with the in-tree library and each variant (k_verify_chain_w vs k_verify_chain_b time).
set -o pipefail
mkdir -p gpurun_out
for v in vb8 vb4; do
  SBH_LIB_PATH=spark-bam_amd/build/ab/lib_$v.so timeout -k 10 600 python -u -m pytest -m gpu --timeout 300 \
    --timeout-method thread -x -q tests/test_gpu_parity.py tests/test_records_gpu.py tests/test_canloadbam_gpu.py \
    > gpurun_out/r05u_pytest_$v.log 2>&1 || exit 1
done
timeout -k 10 400 bash tools/gpu_round.sh prof r05u_intree --steps 5 --warmup 2 --no-cpu-baseline --no-full --no-e2e || exit 2
for v in vb8 vb4; do
  SBH_LIB_PATH=spark-bam_amd/build/ab/lib_$v.so timeout -k 10 400 bash tools/gpu_round.sh prof r05u_$v --steps 5 \
    --warmup 2 --no-cpu-baseline --no-full --no-e2e || exit 3
done
for c in E D; do
  for v in intree vb8; do
    L=""; [ $v != intree ] && L=spark-bam_amd/build/ab/lib_$v.so
    SBH_LIB_PATH=$L timeout -k 10 400 bash tools/gpu_round.sh prof r05u_${v}_$c --config $c --steps 5 --warmup 2 \
      --no-cpu-baseline --no-full --no-e2e || exit 4
  done
done
echo done
