# HEAD float64 engine: budget/grid throughput + f64 tests (gpu_r4ak.sh), then the A/B of the
# centre/candidate fragment-image variant (libccmi_f64cf.so) and the fused E+M pass variant
# (libccmi_f64fused.so) against HEAD (libccmi_f64_base.so)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4ak.sh || exit 1
bash tools/gpu_f64_var.sh f64cf || exit 1
bash tools/gpu_f64_var.sh f64fused || exit 1
