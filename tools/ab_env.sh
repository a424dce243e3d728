# A/B of one environment toggle on bench.py, ABAB order: tools/ab_env.sh TAG "ENV_A" "ENV_B" ARGS...
# (e.g. "SBH_SIEVE=1" "SBH_SIEVE=0" --config B); each line lands in gpurun_out/TAG_ab.jsonl with its env
set -o pipefail
T=$1; A=$2; B=$3; shift 3
mkdir -p gpurun_out
for r in 1 2; do
  for e in "$A" "$B"; do
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-full --no-e2e --no-facade "$@" \
      > gpurun_out/${T}_one.json 2>> gpurun_out/${T}_ab.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${T}_one.json').read()); d['ab_env']=sys.argv[1]; print(json.dumps(d))" "$e" \
      >> gpurun_out/${T}_ab.jsonl || exit 1
  done
done
