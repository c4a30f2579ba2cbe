cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== B (working tree)"; timeout -k 10 180 python3 scripts/wgrad_exp.py > gpurun_out/wgB.log 2>&1; rc=$?; cat gpurun_out/wgB.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
echo "== A (HEAD kernel)"; MEP_LIB=$PWD/exp_build/libA.so timeout -k 10 180 python3 scripts/wgrad_exp.py > gpurun_out/wgA.log 2>&1; rc=$?; cat gpurun_out/wgA.log | grep -v amdgpu.ids; exit $rc
