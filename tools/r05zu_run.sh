# round 5, late: the configs[2] strong line (one 100.9 GiB file, 1 GPU) at the final kernel sources.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py --config C --file-gib 100 > gpurun_out/r05zu_bench_configC.json \
  2> gpurun_out/r05zu_bench_configC.err || exit 1
echo done
