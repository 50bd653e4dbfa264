# r03 v12: cooperative launch inside a captured hipGraph (tools/micro/coop_graph.hip) and the
# construction phases with the layout / setup sub-phases; the upper rounds in one cooperative
# launch (engine option upper_chain): parity and A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
mkdir -p build && /opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/micro/coop_graph.hip -o build/coop_graph || exit 1
timeout -k 10 60 ./build/coop_graph > gpurun_out/r03_v12_coop.log 2>&1
echo "coop rc $?"
timeout -k 10 300 python -u tools/ptime.py > gpurun_out/r03_v12_ptime.log 2>&1
echo "ptime rc $?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 240 --timeout-method thread -k "fused_last or assignment" > gpurun_out/r03_v12_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh base chain:CPK_UPPER_CHAIN=1 base2 chain2:CPK_UPPER_CHAIN=1 || exit $?
