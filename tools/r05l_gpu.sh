set -o pipefail
bash tools/ab_env.sh r05l_ab_w4_lanes 2 "--n 64 --t 32 --joins 4 --steps 5 --warmup 1 --emulate-shard 4" "" "FSDKR_GA_LANES=16" || exit 1
bash tools/ab_env.sh r05l_ab_w16_lanes 2 "--n 64 --t 32 --joins 4 --steps 5 --warmup 1 --emulate-shard 16" "" "FSDKR_GA_LANES=16" "FSDKR_GA_LANES=8" || exit 1
