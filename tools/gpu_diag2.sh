set -o pipefail
mkdir -p gpurun_out/r03_diag2
timeout -k 10 120 python tools/xb_ws_diag.py gpurun_out/r03_diag2/ws_good.npz > gpurun_out/r03_diag2/good.txt 2>&1 && tail -1 gpurun_out/r03_diag2/good.txt && \
MMPC_LIB_PATH=$PWD/lib_var/xbb_norestrict/libmmpc.so timeout -k 10 120 python tools/xb_ws_diag.py gpurun_out/r03_diag2/ws_bad.npz > gpurun_out/r03_diag2/bad.txt 2>&1; tail -3 gpurun_out/r03_diag2/bad.txt
