# exo state-bounded + exact Hessian on the 16-lane kernel failed vs the oracle: which combination diverges
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s5; mkdir -p $O
timeout -k 10 200 python tools/xb_exact_diag.py 20 70 > $O/diag.txt 2>&1; cat $O/diag.txt
MMPC_LIB_PATH=$PWD/lib_var/vbasic/libmmpc.so timeout -k 10 200 python tools/xb_exact_diag.py 20 70 > $O/diag_vbasic.txt 2>&1; cat $O/diag_vbasic.txt
