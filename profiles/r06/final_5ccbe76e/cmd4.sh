# the committed tree's whole GPU suite and smoke once more (the lazy-step test was tightened after cmd1)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final7d; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so > $O/sha.txt
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -4 $O/smoke.log
