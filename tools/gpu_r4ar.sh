# k-means++ distance tiles with 4 row tiles per wave (libccmi_f64kpp4.so) against HEAD
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/gpu_f64_var.sh f64kpp4 || exit 1
