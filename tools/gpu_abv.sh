# One GPU call: inflate A/B of in-tree vs the named variants (spark-bam_amd/build/ab/lib_<v>.so).
# usage: bash tools/gpu_abv.sh TAG CONFIG RECORDS v1 v2 ...
set -o pipefail
T=$1; C=$2; N=$3; shift 3
mkdir -p gpurun_out
L=""
for v in "$@"; do L="$L spark-bam_amd/build/ab/lib_$v.so"; done
timeout -k 10 500 python -u tools/ab_inflate.py --config $C --records $N $L > gpurun_out/${T}_ab$C.log 2>&1
echo "ab rc=$?"
