mkdir -p gpurun_out/r04s9
timeout -k 10 90 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04s9/first.json 2> gpurun_out/r04s9/first.err && python tools/bench_line.py gpurun_out/r04s9/first.json && \
PGTG_PERSIST=1 PGTG_LIB=$PWD/pgtg_amd/libpgtg_hip_tuning.so timeout -k 10 90 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04s9/firstp.json 2> gpurun_out/r04s9/firstp.err && python tools/bench_line.py gpurun_out/r04s9/firstp.json && \
PGTG_PERSIST=1 PGTG_HELPERS=2 PGTG_LIB=$PWD/pgtg_amd/libpgtg_hip_tuning.so timeout -k 10 90 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04s9/firstp2.json 2> gpurun_out/r04s9/firstp2.err && python tools/bench_line.py gpurun_out/r04s9/firstp2.json && \
bash tools/gpu_session.sh r04s9 tests && \
PGTG_PERSIST=1 bash tools/gpu_session.sh r04s9 "libtests:pgtg_amd/libpgtg_hip_tuning.so:exhaustive or bench_sizes or state or parity" && \
bash tools/persist_ab.sh r04s9
