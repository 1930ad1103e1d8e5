# Lane kernel: a full step rejected after the first iteration hands the instance to the 16-lane resume launch (cur)
# instead of line-searching with its wave waiting (lsh0).  Full GPU suite on cur; per-block kernel times (the
# blocks of bench.py's timed steps; blocks 10 and 13 hold the instances that line-search late); V* of block 0 bit
# for bit; same-box A/B of the cfg#3 / cfg#5 lines (value includes the timed blocks)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lsh; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/*/libmmpc.so > $O/sha.txt
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python tools/block_stats.py --config cfg3 --blocks 24 > $O/blocks_cur.jsonl || exit 1
python3 -c "
import json
for l in open('$O/blocks_cur.jsonl'):
    d=json.loads(l); print(d['block'], d['kernel_ms'], d['max_iters'])" | tr '\n' ';'; echo
for c in cfg3 cfg5; do
  timeout -k 10 120 python tools/v_dump.py --config $c --out /tmp/v_cur_$c.npz > /dev/null || exit 1
  MMPC_LIB_PATH=$PWD/lib_var/lsh0/libmmpc.so timeout -k 10 120 python tools/v_dump.py --config $c --out /tmp/v_lsh0_$c.npz > /dev/null || exit 1
  python tools/v_dump.py --compare /tmp/v_cur_$c.npz /tmp/v_lsh0_$c.npz | tee -a $O/compare.txt
  rm -f /tmp/v_*_$c.npz
done
OUT=$O/ab VARIANTS="lsh0 cur" CONFIGS="cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
for f in $O/ab/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f'.split('/')[-1], round(d['ms_per_step'],4), round(d['kernel_ms'],4), round(d['value']))"; done
echo ok
