cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/sweep.py --spp 64 --rounds 2 --grid variant=0,1,2,3,4,5,6,7,8 > gpurun_out/sweep_var.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep_var.txt
timeout -k 10 300 python scripts/diag.py --spp 16 > gpurun_out/diag.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/diag.txt
