# r03 v39: round-0 subtree cap (engine option sweep, 7th field sub0): the peeling takes lower
# subtrees into round 0 (S10: 9.75 -> 8.57 levels per round-0 block, 83 K rows to the upper
# rounds, round 1 512 -> 1024 blocks). S10 bench A/B under rocprofv3.
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab2.sh base s480:CPK_SWEEP=192,576,64,1024,4096,512,480 s384:CPK_SWEEP=192,576,64,1024,4096,512,384 base2 s480b:CPK_SWEEP=192,576,64,1024,4096,512,480
