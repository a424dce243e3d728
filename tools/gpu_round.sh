# One GPU call: the full -m gpu suite, bench.py (N=1, default config B), the rocprofv3
# kernel-trace summary of the bench, and bench lines for configs D and E.
# usage (on the box): bash tools/gpu_round.sh TAG   -> gpurun_out/TAG_*
set -o pipefail
T=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/${T}_bprof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-full --no-e2e > gpurun_out/${T}_bprof.json 2> gpurun_out/${T}_bprof.log || exit 3
python3 tools/prof_stats.py "$(find /tmp/${T}_bprof -name '*.db' -print -quit)" > gpurun_out/${T}_kernel_stats.csv || exit 3
timeout -k 10 300 python -u bench.py --config D --no-cpu-baseline --no-full --no-e2e > gpurun_out/${T}_benchD.json 2> gpurun_out/${T}_benchD.err || exit 4
timeout -k 10 300 python -u bench.py --config E --no-cpu-baseline --no-full --no-e2e > gpurun_out/${T}_benchE.json 2> gpurun_out/${T}_benchE.err || exit 5
