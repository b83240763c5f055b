set -u
# bloom A/B: parity (bit-exact vs the oracle) and the kernel trace of 20 passes at 4096^2
O=gpurun_out/${1:-r05x}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bloom.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_bloom.log 2>&1 || { tail -30 $O/pytest_bloom.log; exit 2; }
tail -1 $O/pytest_bloom.log
for sz in "4096 4096" "1920 1080"; do
  t=$(echo $sz | tr ' ' x)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$t -o run -- python tools/post_probe.py bloom $sz 20 > $O/trace_$t.log 2>&1 || { tail -5 $O/trace_$t.log; exit 3; }
  f=$(find $O/trace_$t -name "*kernel_stats.csv"); echo "== $t"; grep -E "bloom|mip" $f | cut -d, -f1-4 | sed 's/(.*)"/"/'
done
