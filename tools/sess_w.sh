set -u
# Bloom as run-pair polynomials: GPU parity (bit-exact vs the oracle), C3 and
# C5 bench lines with the regenerated counters, bloom kernel trace and PMC.
O=gpurun_out/r05w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bloom.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_bloom.log 2>&1 || { tail -30 $O/pytest_bloom.log; exit 2; }
tail -1 $O/pytest_bloom.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bloom -o run -- python tools/post_probe.py bloom 4096 4096 20 > $O/trace_bloom.log 2>&1 || { tail -5 $O/trace_bloom.log; exit 3; }
find $O/trace_bloom -name "*kernel_stats.csv" -exec cp {} $O/bloom_kernel_stats.csv \;
cut -d, -f1-8 $O/bloom_kernel_stats.csv
timeout -k 10 300 python bench.py > $O/bench_C3.json 2> $O/bench_C3.err || { tail -20 $O/bench_C3.err; exit 4; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); b=d['bloom_pass']; print('C3', round(d['ms_per_step'],4), 'frac', d['roofline']['frac'], 'bloom', round(b['ms'],4), 'GB/s', round(b['achieved']), 'fxaa', round(d['post_pass']['ms'],4))" $O/bench_C3.json
timeout -k 10 300 python bench.py --scene O --size 8192 --max-steps 512 --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_C5frame.json 2> $O/bench_C5frame.err || { tail -20 $O/bench_C5frame.err; exit 5; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('C5', round(d['ms_per_step'],4), 'frac', r['frac'], r.get('valu_issue'), r.get('salu_issue'), r.get('frac_null_reason'))" $O/bench_C5frame.json
bash tools/pmc_post.sh bloom && mv gpurun_out/pmc_bloom $O/pmc_bloom || exit 6
python -c "import json; d=json.load(open('$O/pmc_bloom/summary.json')); [print(k[:60], {c: round(v/1e6,2) for c,v in d[k].items() if c in ('FETCH_SIZE','WRITE_SIZE','SQ_INSTS_VALU','SQ_WAVES')}) for k in d]"
