set -u
# bloom round-5 redesign: parity + kernel traces (tools/sess_x.sh), the C3 bench
# line's bloom_pass, and the bloom PMC passes
O=gpurun_out/$1
bash tools/sess_x.sh $1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_C3.json 2> $O/bench_C3.err || { tail -20 $O/bench_C3.err; exit 4; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); b=d['bloom_pass']; print('C3', round(d['ms_per_step'],4), 'frac', d['roofline']['frac'], 'bloom', round(b['ms'],4), 'GB/s', round(b['achieved']), 'fxaa', round(d['post_pass']['ms'],4))" $O/bench_C3.json
bash tools/pmc_post.sh bloom && mv gpurun_out/pmc_bloom $O/pmc_bloom || exit 6
python -c "import json; d=json.load(open('$O/pmc_bloom/summary.json')); [print(k[:50], {c: round(v/1e6,3) for c,v in d[k].items() if c in ('FETCH_SIZE','WRITE_SIZE','SQ_INSTS_VALU','SQ_WAVES')}) for k in d if 'bloom' in k or 'mip' in k]"
