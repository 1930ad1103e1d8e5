# Round-6 session-2 baseline: full GPU suite + smoke + the driver's default bench line on HEAD's build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6base; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so > $O/sha.txt
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json | cut -c1-400
