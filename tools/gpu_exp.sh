set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in NOSTORE NOPRE; do
KM_STAMPS_LIB=libccmi_stamps_$v.so timeout -k 10 200 python -u tools/km_stamps.py 256 > gpurun_out/exp_$v.txt 2>&1 || exit 1
echo "== $v"; grep -E "timings|wave 0|wave 3|post" gpurun_out/exp_$v.txt
done
