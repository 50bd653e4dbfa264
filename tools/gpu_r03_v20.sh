# r03 v20: the refinement turn kernel at 3 waves per SIMD (in-tree: 168 VGPRs, 22 spilled), 2
# (abv/turnw2: 191 VGPRs, no spills) and 4 (abv/turnw4: 128 VGPRs, 70 spilled), against no_turn
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_ab2.sh noturn:CPK_NO_TURN=1 base turnw2 turnw4 noturn2:CPK_NO_TURN=1 || exit $?
