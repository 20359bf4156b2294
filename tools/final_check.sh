set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_bench.sh -r 3 -c c3 ab/librtg_rc.so ab/librtg_ou.so > gpurun_out/ab_ou_c3.log 2>&1 && cat gpurun_out/ab_ou_c3.log &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 && tail -2 gpurun_out/pytest_gpu_final.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 && tail -3 gpurun_out/smoke_final.log &&
TAG=r02 bash tools/round_profiles.sh
