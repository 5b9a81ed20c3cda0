set -o pipefail
O=gpurun_out/r01s; mkdir -p $O
F=$PWD/fs-dkr_amd/fsdkr/libfsdkr_fence.so
for v in new fence new fence; do
  if [ $v = fence ]; then export FSDKR_LIB=$F; else unset FSDKR_LIB; fi
  timeout -k 10 120 python tools/bench_modexp.py --count 7680 --reps 3 --widths 128,64 --groups 16,8 > $O/mx_$v.jsonl 2>&1 || exit 1
  echo "$v $(grep -o '"mod_bits": [0-9]*\|"kernel_ms": [0-9.]*\|"group": [0-9]*' $O/mx_$v.jsonl | tr '\n' ' ')"
  timeout -k 10 200 python tools/ab_collect.py --shard 8 --rounds 3 - > $O/ab8_$v.log 2>&1 || exit 1
  timeout -k 10 200 python tools/ab_collect.py --shard 1 --rounds 3 - > $O/ab1_$v.log 2>&1 || exit 1
  echo "$v shard8 $(grep -o '"median_ms": [0-9.]*' $O/ab8_$v.log) shard1 $(grep -o '"median_ms": [0-9.]*' $O/ab1_$v.log)"
done
