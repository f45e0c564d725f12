# round-6 final records, part B: rocprofv3 kernel stats + PMC (configs[4], configs[1]), the configs[1]
# latency record, the SB3 adapter, the 2/4/8-rank digest rehearsal
set -o pipefail
bash tools/gpu_session.sh r06fb profile:cfg5,cfg2 stampsjson:cfg2 adapter ranks
