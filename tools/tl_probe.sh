set -o pipefail
O=gpurun_out/tl; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k timeline --timeout 120 --timeout-method thread > $O/pytest_tl.log 2>&1; rc=$?; tail -2 $O/pytest_tl.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/timeline.py --config c3 --waves-per-block 1 --json $O/c3_full.json --raw $O/c3_full.npz > /dev/null &&
timeout -k 10 200 python tools/timeline.py --config c3 --waves-per-block 1 --shard 0 --shards 8 --json $O/c3_s0of8.json --raw $O/c3_s0of8.npz > /dev/null &&
RTG_LPT_MIN=65 timeout -k 10 200 python tools/timeline.py --config c3 --waves-per-block 1 --shard 0 --shards 8 --json $O/c3_s0of8_nolpt.json --raw $O/c3_s0of8_nolpt.npz > /dev/null &&
timeout -k 10 200 python tools/timeline.py --config c4 --waves-per-block 1 --shard 0 --shards 8 --json $O/c4_s0of8.json --raw $O/c4_s0of8.npz > /dev/null &&
echo done
