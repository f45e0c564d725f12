set -o pipefail
O=gpurun_out/r06p2; mkdir -p $O
export TMPDIR=/tmp
for g in 256 512 768 1024 1536 3072; do
  PGTG_FLAT_WGS=$g timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/g$g -o run --output-format csv -- python bench.py --adapter device --steps 60 --warmup 10 > $O/g$g.json 2> $O/g$g.err || { tail $O/g$g.err; exit 1; }
  f=$(find $O/g$g -name "*kernel_stats.csv" | head -1); echo "G=$g $(grep k_flatten $f | cut -d, -f3-4) $(cat $O/g$g.json | tail -1 | cut -c1-80)"
done
