# S50 at 50M to convergence: sensitivity of the iteration count to 1e-15 rhs perturbations
# (in-tree library), and the same unperturbed with a variant library abx/<name> if given
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in 1 2 3; do
  timeout -k 10 600 python bench.py --config s50 --itmax 3000 --steps 1 --warmup 0 --no-cpu-baseline --no-pmc --rhs-perturb 1e-15 --perturb-seed $s > gpurun_out/s50_sens_$s.json 2> gpurun_out/s50_sens_$s.err
done
for v in "$@"; do
  CPK_LIB_PATH=$GRAFT_REPO_ROOT/abx/$v/libcpk.so timeout -k 10 600 python bench.py --config s50 --itmax 3000 --steps 1 --warmup 0 --no-cpu-baseline --no-pmc --rhs-perturb 1e-15 --perturb-seed 1 > gpurun_out/s50_sens_$v.json 2> gpurun_out/s50_sens_$v.err
done
