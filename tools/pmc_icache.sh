#!/bin/bash
# One extra rocprofv3 counter pass over a short bench run: instruction-cache and issue counters
# (is a big kernel -- k_huff is 57 KB of code -- fetch-bound?).  Usage (on the GPU box):
#   bash tools/pmc_icache.sh gpurun_out/pmc_ic
set -euo pipefail
OUT=${1:-gpurun_out/pmc_ic}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd - > /dev/null
pass() {  # name, counters...
  local name=$1
  shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-e2e --no-full --steps 2 --warmup 1 > "$OUT/$name.bench.json" 2> "$OUT/$name.log"
  local f
  f=$(find "$OUT/$name" -name "*counter_collection.csv" -print -quit)
  cp "$f" "$OUT/$name.csv"
  python3 tools/pmc_summary.py "$OUT/$name.csv" > "$OUT/$name.txt"
  echo "pass $name done"
}
pass ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES
pass sca SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_LEVEL_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES
echo "pmc icache ok"
