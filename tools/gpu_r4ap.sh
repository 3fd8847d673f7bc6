# M-sum prefetch depth 8 / 6 (libccmi_f64msg8/6.so) against HEAD (libccmi_f64_base.so)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/gpu_f64_var.sh f64msg8 || exit 1
bash tools/gpu_f64_var.sh f64msg6 || exit 1
