# round-6 final records, part A: suite, smoke, bench lines (driver-shaped and 1000-step), every workload's
# 1000-step line, the shard lines, RCCL
set -o pipefail
bash tools/gpu_session.sh r06fa tests smoke bench driver benchlong:cfg2 benchlong:cfg3 benchlong:cfg4 benchlong:train shards rccl
