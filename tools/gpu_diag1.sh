set -o pipefail
mkdir -p gpurun_out/r03_diag1
timeout -k 10 120 tools/ubench/issue_rate > gpurun_out/r03_diag1/issue_rate.txt 2>&1 && cat gpurun_out/r03_diag1/issue_rate.txt && \
timeout -k 10 200 python tools/xb_diag.py gpurun_out/r03_diag1/xb_good.npz > gpurun_out/r03_diag1/xb_good.txt 2>&1 && tail -4 gpurun_out/r03_diag1/xb_good.txt && \
MMPC_LIB_PATH=$PWD/lib_var/xbb_norestrict/libmmpc.so timeout -k 10 200 python tools/xb_diag.py gpurun_out/r03_diag1/xb_bad.npz > gpurun_out/r03_diag1/xb_bad.txt 2>&1; cat gpurun_out/r03_diag1/xb_bad.txt
