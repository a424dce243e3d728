set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || exit 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-full --no-e2e > gpurun_out/bprof.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof3 -o run -- python3 tools/deflate_bench.py --mib 1024 --reps 1 > gpurun_out/dprof3.log 2>&1 || exit 4
