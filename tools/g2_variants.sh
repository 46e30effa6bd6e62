set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
for v in A B C D; do
  FILGPU_LIB=crypto3-fil-proofs_amd/build/var/lib_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k g2 -x -q --timeout 120 --timeout-method thread > gpurun_out/var/t_$v.log 2>&1
  FILGPU_LIB=crypto3-fil-proofs_amd/build/var/lib_$v.so timeout -k 10 200 python -u tools/msm_bench.py --log-rows 26 --reps 2 --query 4 > gpurun_out/var/b_$v.log 2>&1
  echo "$v: $(tail -1 gpurun_out/var/t_$v.log) | $(tail -1 gpurun_out/var/b_$v.log)"
done
